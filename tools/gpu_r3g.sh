# round 2: what config 5b's small records cost k_crc_any
OUT=${OUT:-r3g}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for m in msg msgsmall msgbig; do
timeout -k 10 200 ./kbench2 $m 2000000 4 5 > ../gpurun_out/$OUT/any_$m.txt 2>&1 || exit $?
done
