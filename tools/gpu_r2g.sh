OUT=${OUT:-r2g}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 tools/kframe 1000000 6 5 > gpurun_out/$OUT/kframe.txt 2>&1
