# multi-GPU C-ABI entries: every GPU test
OUT=${OUT:-r4k}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$OUT/pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/$OUT/pytest_gpu.log | head; exit $rc
