#!/bin/bash
# round 4, session ff: cache-policy bits of k_seg_stream's / k_crc_any's buffer
# row loads -- nt (production) against sc0|nt, nt|sc1, sc0|nt|sc1 on records
TAG=r4ff STEPS=extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4ff/ab_rec 3 prod=hunddb_amd/libhundcrc.so aux3=tools/ab/buf_aux3/libhundcrc.so aux18=tools/ab/buf_aux18/libhundcrc.so aux19=tools/ab/buf_aux19/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
