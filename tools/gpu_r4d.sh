# k_unframe store-after-group: every GPU test, the unframe bench line, A/B again
OUT=${OUT:-r4d}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload unframe --json-out gpurun_out/$OUT/bench_unframe.json > gpurun_out/$OUT/bench_unframe.log 2>&1 || exit $?
cd tools && timeout -k 10 300 ./kframe 1000000 6 5 > ../gpurun_out/$OUT/kframe_st3.txt 2>&1
