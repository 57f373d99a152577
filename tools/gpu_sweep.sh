set -e
OUT=${OUT:-r2c}
mkdir -p gpurun_out/$OUT
cd tools
for m in 4096 8192 16384 mixed offlen4k; do
  HC_SWEEP=1 timeout -k 10 120 ./kbench2 $m 1000000 5 5 > ../gpurun_out/$OUT/sweep_$m.txt 2>&1
done
HC_SWEEP=1 timeout -k 10 200 ./kbench2 8192 16000000 2 3 > ../gpurun_out/$OUT/sweep_8192_16M.txt 2>&1
HC_SWEEP=1 timeout -k 10 120 ./kbench2 8192 250000 5 5 > ../gpurun_out/$OUT/sweep_8192_250k.txt 2>&1
