OUT=${OUT:-r2k}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 tools/kcopy2 8192 5 5 > gpurun_out/$OUT/kcopy2.txt 2>&1
