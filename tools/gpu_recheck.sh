# Round-end style recheck: GPU tests, smoke, default bench, rocprofv3 kernel stats of the same bench
OUT=${OUT:-r2j}
R=$PWD
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/$OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/$OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --json-out gpurun_out/$OUT/bench.json > gpurun_out/$OUT/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$OUT/prof -o run -- python3 $R/bench.py --pmc off --cpu-seconds 0 --json-out $R/gpurun_out/$OUT/bench_under_rocprof.json > $R/gpurun_out/$OUT/rocprof.log 2>&1 || exit $?
cd $R/tools && timeout -k 10 200 ./kbench2 msg 2000000 5 5 > ../gpurun_out/$OUT/any_msg.txt 2>&1
