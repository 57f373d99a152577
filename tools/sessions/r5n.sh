#!/bin/bash
# round 5, session n: uniform non-conforming blocks routed by the r5m sweep (k_crc_any keeps 4-B
# aligned 2-8 KiB blocks); the block and parity suites; blocks4092 / blocks8188 / records_gapped.
TAG=r5n STEPS=tests,workloads,extras \
FILES="tests/test_gpu_seg_blocks.py tests/test_gpu_parity.py tests/test_gpu_seg.py" \
WORKLOADS="blocks4092 blocks8188 records_gapped" \
EXTRA1="bash tools/prof_workloads.sh gpurun_out/r5n blocks8188 records_gapped" \
bash tools/gpu_session.sh
