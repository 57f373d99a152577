# round 2: gather into pinned staging, streamed vs plain stores (pageable sources), one box
OUT=${OUT:-r2y}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
for rep in 1 2; do
for g in 1 0; do
HC_GATHER_NT=$g HC_ADD_CRCS_NT=0 timeout -k 10 200 python3 -u $B --mode addcrcs --blocks 1000000 --mem pageable --steps 5 > gpurun_out/$OUT/add_g${g}_r$rep.json 2>> gpurun_out/$OUT/err.log || exit 1
HC_GATHER_NT=$g timeout -k 10 200 python3 -u $B --mode host8k --mem pageable --steps 5 > gpurun_out/$OUT/h8k_g${g}_r$rep.json 2>> gpurun_out/$OUT/err.log || exit 1
HC_GATHER_NT=$g timeout -k 10 300 python3 -u $B --mode replay --records 2000000 --mem pageable --steps 4 > gpurun_out/$OUT/replay_g${g}_r$rep.json 2>> gpurun_out/$OUT/err.log || exit 1
done; done
