# random-layout fuzz against the oracle
OUT=${OUT:-r4o}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -v --timeout 240 --timeout-method thread > gpurun_out/$OUT/pytest_fuzz.log 2>&1
rc=$?; tail -3 gpurun_out/$OUT/pytest_fuzz.log; grep -E "FAILED|assert" gpurun_out/$OUT/pytest_fuzz.log | head -20; exit $rc
