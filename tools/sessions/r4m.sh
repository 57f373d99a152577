#!/bin/bash
# round 4, session m: k_seg_stream with an event row's work before its refill
# (no row copy: 4 v_mov a row fewer); seg parity, A/B on records
TAG=r4m STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/seg6_noc/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4m/ab_seg 4 prod=hunddb_amd/libhundcrc.so noc=tools/ab/seg6_noc/libhundcrc.so noev=tools/ab/seg2_noev/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
