# round 2: host ReadFromDisk throughput
OUT=${OUT:-r3a}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
for mem in pinned pageable; do
timeout -k 10 200 python3 -u $B --mode readdisk --blocks 1000000 --mem $mem --steps 5 > gpurun_out/$OUT/readdisk_$mem.json 2>> gpurun_out/$OUT/err.log || exit 1
done
