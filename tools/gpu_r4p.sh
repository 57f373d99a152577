# --input scatter rehearsal: two ranks sharing the GPU (gloo), and the resident default for comparison
OUT=${OUT:-r4p}
mkdir -p gpurun_out/$OUT
HC_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --blocks 500000 --input scatter --json-out gpurun_out/$OUT/scatter_n2.json > gpurun_out/$OUT/scatter_n2.log 2>&1 || { tail -20 gpurun_out/$OUT/scatter_n2.log; exit 1; }
HC_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --blocks 500000 --json-out gpurun_out/$OUT/resident_n2.json > gpurun_out/$OUT/resident_n2.log 2>&1 || { tail -20 gpurun_out/$OUT/resident_n2.log; exit 1; }
