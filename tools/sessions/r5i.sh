#!/bin/bash
# round 5, session i: the small-gap combine issues every gap load before hashing (r5h: 233 us combine),
# and the gap range rounded up to a word (r5h: a record after a 1-B gap was wrong).
# The r5d fault repro first, the seg parity tests, rocprof breakdowns, the record benches.
TAG=r5i STEPS=extras,tests,workloads \
EXTRA1="python tools/repro/seg63.py || exit 3" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5i records records_gapped records4k_shuffled" \
FILES="tests/test_gpu_any_windows.py tests/test_gpu_seg.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="records records_gapped records4k_shuffled" \
bash tools/gpu_session.sh
