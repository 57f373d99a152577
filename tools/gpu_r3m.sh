# round 2: k_crc_any small records lane-parallel (kVar bit 4) A/B
OUT=${OUT:-r3m}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in msgsmall msg eq9815 msgbig; do
timeout -k 10 200 ./kbench2 $m 2000000 4 5 > ../gpurun_out/$OUT/any_$m.txt 2>&1 || exit $?
done
