#!/bin/bash
# round 5, session h: the small-gap stream mode (gaps <= 64 B: the stream does a packed batch's
# work over the record ends, the combine hashes each gap itself), after the zeroed-gap mode's
# 77-80 %.  The r5d fault repro first (the session stops unless it passes), rocprof breakdowns,
# the seg parity tests, the record benches.
TAG=r5h STEPS=extras,tests,workloads \
EXTRA1="python tools/repro/seg63.py || exit 3" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5h records records_gapped records4k_shuffled" \
FILES="tests/test_gpu_any_windows.py tests/test_gpu_seg.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="records records_gapped records4k_shuffled" \
bash tools/gpu_session.sh
