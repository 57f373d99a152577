# round 2: AddCRCsToData framing A/B (streamed vs plain stores), one box
OUT=${OUT:-r2x}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
for rep in 1 2; do
for mem in pinned pageable; do
for nt in 1 0; do
for th in 8 16; do
HC_ADD_CRCS_NT=$nt HC_COPY_THREADS=$th timeout -k 10 200 python3 -u $B --mode addcrcs --blocks 1000000 --mem $mem --steps 5 > gpurun_out/$OUT/add_${mem}_nt${nt}_t${th}_r$rep.json 2>> gpurun_out/$OUT/err.log || exit 1
done; done; done; done
