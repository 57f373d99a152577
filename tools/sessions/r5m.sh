#!/bin/bash
# round 5, session m: the small-gap combine's wave max taken before any lane leaves (r5l: fuzz
# seed 79, a record after a 38-B gap in wave 0 lost words); the fuzz and seg suites; then the
# block-length sweep of k_crc_any against the message stream (r5l: 4092-B blocks 70.0 vs 67.4 %).
TAG=r5m STEPS=tests,extras \
FILES="tests/test_gpu_fuzz.py tests/test_gpu_seg_blocks.py tests/test_gpu_seg.py tests/test_gpu_any_windows.py tests/test_gpu_threads.py tests/test_gpu_graphs.py" \
EXTRA1="python tools/seg_blocks_sweep.py --out gpurun_out/r5m/sweep.jsonl" \
bash tools/gpu_session.sh
