# round 2: final host-path numbers after the AddCRCsToData / gather changes
OUT=${OUT:-r2z}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 &&
for mem in pinned pageable; do
timeout -k 10 200 python3 -u $B --mode addcrcs --blocks 1000000 --mem $mem --steps 5 > gpurun_out/$OUT/addcrcs_$mem.json 2>> gpurun_out/$OUT/err.log || exit 1
timeout -k 10 200 python3 -u $B --mode host8k --mem $mem --steps 5 > gpurun_out/$OUT/host8k_$mem.json 2>> gpurun_out/$OUT/err.log || exit 1
timeout -k 10 300 python3 -u $B --mode replay --records 2000000 --mem $mem --steps 4 > gpurun_out/$OUT/replay2m_$mem.json 2>> gpurun_out/$OUT/err.log || exit 1
timeout -k 10 300 python3 -u $B --mode config5 --records 2000000 --mem $mem --steps 4 > gpurun_out/$OUT/config5_2m_$mem.json 2>> gpurun_out/$OUT/err.log || exit 1
done
