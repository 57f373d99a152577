#!/bin/bash
# round 4, session mm: k_frame's row-0 store change against the library before
# it (30077ad's kernels), alternating processes on one box
TAG=r4mm STEPS=extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4mm/ab_frame 5 old=tools/ab/frame_old/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload frame" \
bash tools/gpu_session.sh
