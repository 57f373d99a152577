# multi-GPU edge tests; same-box comparison of config2/northstar bench with the read patterns
OUT=${OUT:-r4m}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 240 --timeout-method thread > gpurun_out/$OUT/pytest_multi.log 2>&1 || { tail -30 gpurun_out/$OUT/pytest_multi.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_multi.log
for w in config2 northstar; do
timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 --pmc off --json-out gpurun_out/$OUT/b_$w.json > gpurun_out/$OUT/b_$w.log 2>&1 || exit $?
done
cd tools && timeout -k 10 200 ./kread 8192 4 5 > ../gpurun_out/$OUT/kread.txt 2>&1 || exit $?
timeout -k 10 200 ./kread 4096 4 5 > ../gpurun_out/$OUT/kread_4g.txt 2>&1 || exit $?
timeout -k 10 300 ./kbench2 4096 1000000 4 5 > ../gpurun_out/$OUT/kb2_4096.txt 2>&1 || exit $?
