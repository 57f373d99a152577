#!/bin/bash
# round 5, session l: uniform block batches k_crc_grp refuses (4092-B blocks, odd addresses) on the
# message stream (launch_seg_blocks).  Parity first (the new tests, the seg suites, every parity and
# fuzz test that runs such blocks), then blocks4092 on the stream and, for comparison, on k_crc_any
# (HC_SEG_MIN_BLOCKS above the batch), rocprof breakdowns of both.
TAG=r5l STEPS=tests,workloads,extras \
FILES="tests/test_gpu_seg_blocks.py tests/test_gpu_seg.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_any_windows.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="blocks4092" \
EXTRA1="HC_SEG_MIN_BLOCKS=2000000000 python bench.py --workload blocks4092 --cpu-seconds 0 --json-out gpurun_out/r5l/bench_blocks4092_any.json" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5l blocks4092" \
bash tools/gpu_session.sh
