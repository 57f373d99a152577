# production k_crc_grp: 2M x 4 KiB vs 1M x 8 KiB (both 8.19 GB) and the piece variant, same box
OUT=${OUT:-r4r}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 300 ./kbench2 4096 2000000 5 5 > ../gpurun_out/$OUT/kb2_4k_2m.txt 2>&1 || exit $?
KB2_PIECE=1 timeout -k 10 300 ./kbench2 8192 1000000 5 5 > ../gpurun_out/$OUT/kb2_8k_piece.txt 2>&1 || exit $?
timeout -k 10 200 ./kread 8192 4 5 > ../gpurun_out/$OUT/kread.txt 2>&1 || exit $?
