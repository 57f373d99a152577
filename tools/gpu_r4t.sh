# nibble-table finalise (kNib) vs production k_crc_grp at 4 and 8 KiB
OUT=${OUT:-r4t}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
KB2_NIB=1 timeout -k 10 300 ./kbench2 4096 1000000 5 5 > ../gpurun_out/$OUT/nib_4k.txt 2>&1 || exit $?
KB2_NIB=1 timeout -k 10 300 ./kbench2 8192 1000000 5 5 > ../gpurun_out/$OUT/nib_8k.txt 2>&1 || exit $?
KB2_NIB=1 timeout -k 10 300 ./kbench2 4096 2000000 5 5 > ../gpurun_out/$OUT/nib_4k_2m.txt 2>&1 || exit $?
