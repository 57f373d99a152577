#!/bin/bash
# round 5, session o: the small-gap combine issues the gap loads of all four sub-passes before
# hashing when every gap fits 8 words (r5n: 103 us of combine on records_gapped); seg + fuzz suites,
# records_gapped and records under rocprof.
TAG=r5o STEPS=tests,extras \
FILES="tests/test_gpu_seg.py tests/test_gpu_seg_blocks.py tests/test_gpu_fuzz.py" \
EXTRA1="bash tools/prof_workloads.sh gpurun_out/r5o records_gapped records" \
bash tools/gpu_session.sh
