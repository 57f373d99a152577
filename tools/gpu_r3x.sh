# round 2: k_crc_any double-buffered body (kVar bit 5) A/B
OUT=${OUT:-r3x}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in msg msgbig eq9815; do
timeout -k 10 200 ./kbench2 $m 2000000 4 5 > ../gpurun_out/$OUT/any_$m.txt 2>&1 || exit $?
done
