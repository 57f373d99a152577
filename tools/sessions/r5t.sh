#!/bin/bash
# round 5, session t: k_crc_grp ahead of the stream's modes for large aligned-record batches; the
# seg suites, then the aligned-records probe and records4k_shuffled.
TAG=r5t STEPS=tests,extras,workloads \
FILES="tests/test_gpu_seg.py tests/test_gpu_seg_blocks.py tests/test_gpu_threads.py tests/test_gpu_graphs.py" \
EXTRA1="python tools/seg_aligned_probe.py" \
WORKLOADS="records4k_shuffled records" \
bash tools/gpu_session.sh
