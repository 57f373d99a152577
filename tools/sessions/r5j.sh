#!/bin/bash
# round 5, session j: the small-gap combine with per-lane global loads (r5i: a per-lane buffer
# resource became a 64-pass waterfall per load: 369 us of combine).
# The r5d fault repro first, the seg parity tests, rocprof breakdowns, the record benches.
TAG=r5j STEPS=extras,tests,workloads \
EXTRA1="python tools/repro/seg63.py || exit 3" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5j records records_gapped records4k_shuffled" \
FILES="tests/test_gpu_any_windows.py tests/test_gpu_seg.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="records records_gapped records4k_shuffled" \
bash tools/gpu_session.sh
