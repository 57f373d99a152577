# Round-2 re-entry check: RCCL one-rank test, every GPU test, smoke, default
# bench, rocprofv3 stats of the same bench (CSV).
OUT=${OUT:-r4a}
R=$PWD
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 240 --timeout-method thread > gpurun_out/$OUT/pytest_rccl.log 2>&1 || { tail -30 gpurun_out/$OUT/pytest_rccl.log; exit 1; }
PART=1 OUT=$OUT bash tools/gpu_final_r2.sh
cd tools && timeout -k 10 200 ./kread 8192 5 5 > ../gpurun_out/$OUT/kread.txt 2>&1
