#!/bin/bash
# round 4, session n: what in an event's placement costs the clock --
# diagnostics (wrong words) against the no-copy build: events without the
# 3-shift fold (nofold), events without the mat-vec (nomat), no events (noev)
TAG=r4n STEPS=extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4n/ab_seg 3 noc=tools/ab/seg6_noc/libhundcrc.so nofold=tools/ab/seg7_nofold/libhundcrc.so nomat=tools/ab/seg7_nomat/libhundcrc.so noev=tools/ab/seg2_noev/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
