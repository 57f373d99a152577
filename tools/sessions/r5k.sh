#!/bin/bash
# round 5, session k: k_seg_plan hashes the small gaps (r5j: 103 us of combine for the gap lines),
# the combine reads one word a record.
# The r5d fault repro first, the seg parity tests, rocprof breakdowns, the record benches.
TAG=r5k STEPS=extras,tests,workloads \
EXTRA1="python tools/repro/seg63.py || exit 3" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5k records records_gapped records4k_shuffled" \
FILES="tests/test_gpu_any_windows.py tests/test_gpu_seg.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="records records_gapped records4k_shuffled" \
bash tools/gpu_session.sh
