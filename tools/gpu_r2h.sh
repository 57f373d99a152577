OUT=${OUT:-r2h}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 tools/kcopy2 4096 5 5 > gpurun_out/$OUT/kcopy2.txt 2>&1 && timeout -k 10 300 tools/kframe 1000000 5 5 > gpurun_out/$OUT/kframe.txt 2>&1
