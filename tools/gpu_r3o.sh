# round 2: 4-rank strong-scaling rehearsal (gloo, ranks sharing the one GPU)
OUT=${OUT:-r3o}
mkdir -p gpurun_out/$OUT
HC_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 4 --blocks 4000000 --steps 10 --warmup 3 --json-out gpurun_out/$OUT/bench_gloo_n4.json > gpurun_out/$OUT/bench.log 2>&1
