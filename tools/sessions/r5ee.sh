#!/bin/bash
# round 5, session ee: the stream and combine skip their table fills when the batch falls back
# (k_crc_grp or k_crc_any takes it); seg suites and fuzz, records4k_shuffled / records /
# records_gapped and their breakdowns
TAG=r5ee STEPS=tests,workloads,extras \
FILES="tests/test_gpu_seg.py tests/test_gpu_seg_blocks.py tests/test_gpu_any_windows.py tests/test_gpu_graphs.py tests/test_gpu_threads.py tests/test_gpu_fuzz.py" \
WORKLOADS="records4k_shuffled records records_gapped" \
EXTRA1="bash tools/prof_workloads.sh gpurun_out/r5ee records4k_shuffled records" \
EXTRA2="python tools/seg_aligned_probe.py" \
bash tools/gpu_session.sh
