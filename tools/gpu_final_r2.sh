# Round-2 final evidence: GPU tests, smoke, default bench, rocprofv3 stats of the
# same bench (CSV), then every bench workload.  PART=1 or PART=all.
OUT=${OUT:-r2final}
R=$PWD
mkdir -p gpurun_out/$OUT
if [ "${PART:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/$OUT/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/$OUT/pytest_gpu.log | head -20; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || exit $?
  timeout -k 10 400 python bench.py --json-out gpurun_out/$OUT/bench.json > gpurun_out/$OUT/bench.log 2>&1 || exit $?
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof -o run -- python3 $R/bench.py --pmc off --cpu-seconds 0 --json-out $R/gpurun_out/$OUT/bench_under_rocprof.json > $R/gpurun_out/$OUT/rocprof.log 2>&1 || exit $?
else
  for w in northstar config2 config3 offlen4k 16k verify config4 frame unframe records; do
    timeout -k 10 400 python bench.py --workload $w --json-out gpurun_out/$OUT/bench_$w.json > gpurun_out/$OUT/bench_$w.log 2>&1 || exit $?
  done
fi
