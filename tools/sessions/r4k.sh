#!/bin/bash
# round 4, session k: paired placements in k_seg_stream (an event's H and a
# unit's raw CRC wait for a partner and share one mat-vec); seg, thread and
# fuzz parity through the variant, then A/B on the records workload
TAG=r4k STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/seg4_pair/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py tests/test_gpu_fuzz.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4k/ab_seg 3 prod=hunddb_amd/libhundcrc.so pair=tools/ab/seg4_pair/libhundcrc.so noev=tools/ab/seg2_noev/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
