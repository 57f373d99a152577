#!/bin/bash
# round 4, session j: k_seg_* with 32 KiB units (half the unit-end placements),
# chunks of 128 or 64 units; seg parity through both variants, then A/B
TAG=r4j STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/seg3_u32/libhundcrc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="HUNDCRC_LIB=\$PWD/tools/ab/seg3_u32c6/libhundcrc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4j/ab_seg 3 prod=hunddb_amd/libhundcrc.so u32=tools/ab/seg3_u32/libhundcrc.so u32c6=tools/ab/seg3_u32c6/libhundcrc.so noev=tools/ab/seg2_noev/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
