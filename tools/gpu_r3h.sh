# round 2: k_crc_any body batch size A/B (2/4/6/8 rows)
OUT=${OUT:-r3h}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in msg eq9815 blk4092 msgbig; do
timeout -k 10 200 ./kbench2 $m 2000000 4 5 > ../gpurun_out/$OUT/any_$m.txt 2>&1 || exit $?
done
