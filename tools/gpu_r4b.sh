# seg stream chunk sweep (full dispatch, words checked) + read-pattern piece x chunk sweep
OUT=${OUT:-r4b}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
HC_SWEEP=1 timeout -k 10 300 ./kbench2 msg 2000000 4 5 > ../gpurun_out/$OUT/seg_sweep_msg.txt 2>&1 || exit $?
KREAD_DYN=1 timeout -k 10 200 ./kread 8192 4 5 > ../gpurun_out/$OUT/kread_dyn.txt 2>&1 || exit $?
