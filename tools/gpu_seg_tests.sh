#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/segt
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 300 --timeout-method thread > gpurun_out/segt/pytest_seg.log 2>&1 || { echo "FAIL seg tests"; tail -40 gpurun_out/segt/pytest_seg.log; exit 1; }
tail -12 gpurun_out/segt/pytest_seg.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/segt/pytest_gpu.log 2>&1 || { echo "FAIL gpu suite"; tail -40 gpurun_out/segt/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/segt/pytest_gpu.log
