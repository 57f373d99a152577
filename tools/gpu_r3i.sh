# round 2: k_crc_any batch 2 vs 4, second box
OUT=${OUT:-r3i}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in blk4092 msg msgsmall eq9815; do
timeout -k 10 200 ./kbench2 $m 2000000 4 5 > ../gpurun_out/$OUT/any_$m.txt 2>&1 || exit $?
done
