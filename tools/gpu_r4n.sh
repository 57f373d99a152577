# k_crc_piece (4 KiB pieces of 8/16 KiB blocks) vs production k_crc_grp
OUT=${OUT:-r4n}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
KB2_PIECE=1 timeout -k 10 300 ./kbench2 8192 1000000 5 5 > ../gpurun_out/$OUT/piece_8k.txt 2>&1 || exit $?
KB2_PIECE=1 timeout -k 10 300 ./kbench2 16384 500000 5 5 > ../gpurun_out/$OUT/piece_16k.txt 2>&1 || exit $?
