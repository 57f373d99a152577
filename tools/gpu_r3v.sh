# round 2: chunk rule with the 4M-block cutoff -- tests and bench lines
OUT=${OUT:-r3v}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || exit $?
for w in northstar config4 16k config2; do
  timeout -k 10 400 python3 -u bench.py --workload $w --json-out gpurun_out/$OUT/bench_$w.json > gpurun_out/$OUT/bench_$w.log 2>&1 || exit $?
done
