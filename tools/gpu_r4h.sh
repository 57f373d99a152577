# seg combine without the serial extra K: seg GPU tests + kbench2 msg/eq9815
OUT=${OUT:-r4h}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 240 --timeout-method thread > gpurun_out/$OUT/pytest_seg.log 2>&1 || { tail -30 gpurun_out/$OUT/pytest_seg.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_seg.log
cd tools || exit 1
timeout -k 10 300 ./kbench2 msg 2000000 4 5 > ../gpurun_out/$OUT/seg_msg.txt 2>&1 || exit $?
timeout -k 10 300 ./kbench2 eq9815 2000000 4 5 > ../gpurun_out/$OUT/seg_eq.txt 2>&1 || exit $?
