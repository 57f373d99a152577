# round 2: XCD-contiguous slots adopted at 8/16 KiB -- tests, A/B, bench lines
OUT=${OUT:-r3t}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || exit $?
(cd tools && for m in 8192 16384 4096; do timeout -k 10 150 ./kbench2 $m 1000000 6 5 > ../gpurun_out/$OUT/kb2_$m.txt 2>&1 || exit $?; done) || exit $?
timeout -k 10 300 python3 -u bench.py --json-out gpurun_out/$OUT/bench_northstar.json > gpurun_out/$OUT/bench_northstar.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --workload 16k --json-out gpurun_out/$OUT/bench_16k.json > gpurun_out/$OUT/bench_16k.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --workload config4 --json-out gpurun_out/$OUT/bench_config4.json > gpurun_out/$OUT/bench_config4.log 2>&1
