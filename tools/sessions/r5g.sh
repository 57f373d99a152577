#!/bin/bash
# round 5, session g: one gated k_crc_grp launch for all-conforming refused batches, gaps capped at
# 4 MiB (the plan wrote O(n x units) first_ev entries for shuffled batches: 33 ms).  The r5d
# fault repro first (the session stops unless it passes), rocprof breakdowns, the seg parity
# tests, the record benches.
TAG=r5g STEPS=extras,tests,workloads \
EXTRA1="python tools/repro/seg63.py || exit 3" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5g records records_gapped records4k_shuffled" \
FILES="tests/test_gpu_any_windows.py tests/test_gpu_seg.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="records records_gapped records4k_shuffled" \
bash tools/gpu_session.sh
