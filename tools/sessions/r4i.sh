#!/bin/bash
# round 4, session i: k_seg_stream variants on the records workload --
# placement columns in LDS (ldscol), two groups (8 rows) in flight per wave
# (deep, with ldscol), no event work (noev), one select per event (evcheap),
# a 4-accumulator mat-vec (ilp); the seg parity tests through the deep variant
TAG=r4i STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/seg2_deep/libhundcrc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4i/ab_seg 3 prod=hunddb_amd/libhundcrc.so deep=tools/ab/seg2_deep/libhundcrc.so ldscol=tools/ab/seg2_ldscol/libhundcrc.so noev=tools/ab/seg2_noev/libhundcrc.so evcheap=tools/ab/seg2_evcheap/libhundcrc.so ilp=tools/ab/seg2_ilp/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
