#!/bin/bash
# round 6, session r: the stream's chunk slot at 2^3 units (HC_SEG_LG_CHUNK default 3) -- the seg
# suites, then the record and block workload lines (TAG final2) and their kernel splits
set -u
mkdir -p gpurun_out/r6r
timeout -k 10 500 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py tests/test_gpu_seg_blocks.py tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py tests/test_gpu_bench_workloads.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6r/tests.log 2>&1 || { tail -30 gpurun_out/r6r/tests.log; exit 1; }
tail -2 gpurun_out/r6r/tests.log
TAG=final2 bash tools/sessions/r6final_b.sh
