set -e
OUT=${OUT:-r2a}
mkdir -p gpurun_out/$OUT
cd tools
for m in 4096 8192 16384 mixed offlen4k; do
  timeout -k 10 120 ./kbench2 $m 1000000 6 5 > ../gpurun_out/$OUT/kb2_$m.txt 2>&1
done
timeout -k 10 120 ./kcopy2 4096 6 5 > ../gpurun_out/$OUT/kcopy2.txt 2>&1
