# production k_crc_grp at 0.5M / 1M / 2M / 4M x 8 KiB: fixed cost per launch
OUT=${OUT:-r4u}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for n in 500000 1000000 2000000 4000000; do
timeout -k 10 300 ./kbench2 8192 $n 5 5 > ../gpurun_out/$OUT/kb2_8k_$n.txt 2>&1 || exit $?
done
