# seg combine rewrite: seg GPU tests, kbench2 (words checked), per-kernel times
OUT=${OUT:-r4j}
R=$PWD
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 240 --timeout-method thread > gpurun_out/$OUT/pytest_seg.log 2>&1 || { tail -30 gpurun_out/$OUT/pytest_seg.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_seg.log
cd tools || exit 1
timeout -k 10 300 ./kbench2 msg 2000000 4 5 > ../gpurun_out/$OUT/seg_msg.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof -o run -- $R/tools/kbench2 msg 2000000 2 3 > $R/gpurun_out/$OUT/prof_msg.txt 2>&1
