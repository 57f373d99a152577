# round 2: k_crc_grp refill order A/B (rolling per-row vs whole-group batch)
OUT=${OUT:-r3e}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in 4096 8192 16384 mixed; do
  timeout -k 10 150 ./kbench2 $m 1000000 6 5 > ../gpurun_out/$OUT/kb2_$m.txt 2>&1 || exit $?
done
