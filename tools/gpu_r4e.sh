# unframe bench line, three runs (run-to-run spread)
OUT=${OUT:-r4e}
mkdir -p gpurun_out/$OUT
for k in 1 2 3; do
timeout -k 10 300 python bench.py --workload unframe --cpu-seconds 0 --pmc off --json-out gpurun_out/$OUT/bench_unframe_$k.json > gpurun_out/$OUT/bench_unframe_$k.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --workload frame --cpu-seconds 0 --pmc off --json-out gpurun_out/$OUT/bench_frame.json > gpurun_out/$OUT/bench_frame.log 2>&1 || exit $?
