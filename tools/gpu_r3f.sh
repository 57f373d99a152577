# round 2: k_crc_any rolling body refills A/B
OUT=${OUT:-r3f}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 200 ./kbench2 msg 2000000 5 5 > ../gpurun_out/$OUT/any_msg.txt 2>&1 || exit $?
timeout -k 10 200 ./kbench2 eq9815 2000000 5 5 > ../gpurun_out/$OUT/any_eq9815.txt 2>&1 || exit $?
timeout -k 10 200 ./kbench2 blk4092 2000000 5 5 > ../gpurun_out/$OUT/any_blk4092.txt 2>&1 || exit $?
