# round 2: k_crc_grp XCD-contiguous chunk slots A/B
OUT=${OUT:-r3r}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in 8192 4096 16384; do
  timeout -k 10 150 ./kbench2 $m 1000000 6 5 > ../gpurun_out/$OUT/kb2_$m.txt 2>&1 || exit $?
done
