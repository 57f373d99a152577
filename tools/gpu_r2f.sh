# framing-kernel chunk sweep + every BASELINE workload with the per-size chunk rule
OUT=${OUT:-r2f}
mkdir -p gpurun_out/$OUT
for c in 3 4 5 6 7 8; do
  for w in frame unframe; do
    HC_LG_CHUNK=$c timeout -k 10 200 python bench.py --workload $w --pmc off --cpu-seconds 0 --json-out gpurun_out/$OUT/sweep_${w}_c$c.json > gpurun_out/$OUT/sweep_${w}_c$c.log 2>&1 || exit $?
  done
done
for w in northstar config2 config3 16k offlen4k frame unframe config4; do
  timeout -k 10 400 python bench.py --workload $w --json-out gpurun_out/$OUT/bench_$w.json > gpurun_out/$OUT/bench_$w.log 2>&1 || exit $?
done
