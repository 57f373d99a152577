#!/bin/bash
# round 5, session e: r5d's fault fixed by moving the k_crc_grp fallback out of k_seg_combine
# (gated launches after it); the gapped stream with zeroed gap bytes (one placement per record,
# H(s_j) derived in the combine).  The repro of r5d's fault first (the session stops unless it
# passes), then rocprof breakdowns of the record workloads, the seg parity tests, the benches.
TAG=r5e STEPS=extras,tests,workloads \
EXTRA1="python tools/repro/seg63.py || exit 3" \
EXTRA2="bash tools/prof_workloads.sh gpurun_out/r5e records records_gapped records4k_shuffled" \
FILES="tests/test_gpu_any_windows.py tests/test_gpu_seg.py tests/test_gpu_graphs.py tests/test_gpu_threads.py" \
WORKLOADS="records records_gapped records4k_shuffled" \
bash tools/gpu_session.sh
