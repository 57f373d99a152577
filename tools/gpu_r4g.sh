# seg stream: first_ev prefetch A/B
OUT=${OUT:-r4g}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 300 ./kbench2 msg 2000000 4 5 > ../gpurun_out/$OUT/seg_preev_msg.txt 2>&1 || exit $?
timeout -k 10 300 ./kbench2 eq9815 2000000 4 5 > ../gpurun_out/$OUT/seg_preev_eq.txt 2>&1 || exit $?
