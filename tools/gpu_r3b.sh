# round 2: host ReadFromDisk with the copy-out overlapped
OUT=${OUT:-r3b}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 &&
for mem in pinned pageable; do
timeout -k 10 200 python3 -u $B --mode readdisk --blocks 1000000 --mem $mem --steps 5 > gpurun_out/$OUT/readdisk_$mem.json 2>> gpurun_out/$OUT/err.log || exit 1
HC_COPY_THREADS=16 timeout -k 10 200 python3 -u $B --mode readdisk --blocks 1000000 --mem $mem --steps 5 > gpurun_out/$OUT/readdisk_${mem}_t16.json 2>> gpurun_out/$OUT/err.log || exit 1
done
