# GPU validation after the k_crc_grp / dynamic frame+unframe change
OUT=${OUT:-r2d}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/$OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd tools
for m in 4096 8192 16384 mixed; do
  HC_SWEEP=1 timeout -k 10 120 ./kbench2 $m 1000000 5 5 > ../gpurun_out/$OUT/sweep_$m.txt 2>&1 || exit $?
done
cd ..
for w in frame unframe; do
  timeout -k 10 300 python bench.py --workload $w --pmc off --cpu-seconds 0 --json-out gpurun_out/$OUT/bench_$w.json > gpurun_out/$OUT/bench_$w.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --pmc off --json-out gpurun_out/$OUT/bench_northstar.json > gpurun_out/$OUT/bench_northstar.log 2>&1 || exit $?
HC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --blocks 2000000 --json-out gpurun_out/$OUT/bench_gloo_n2.json > gpurun_out/$OUT/bench_gloo_n2.log 2>&1 || exit $?
exit $rc
