# k_seg_plan with batched loads: seg tests, fuzz, per-kernel times
OUT=${OUT:-r4w}
R=$PWD
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof -o run -- $R/tools/kbench2 msg 2000000 2 3 > $R/gpurun_out/$OUT/prof_msg.txt 2>&1
