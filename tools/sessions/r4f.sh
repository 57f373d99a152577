#!/bin/bash
# round 4, session f: GPU suite + smoke with k_seg_plan's grid capped at 2048
# workgroups, the headline bench + rocprof, the mixed and records workloads;
# the paired placement against round 3's finalise on mixed blocks, four more pairs
TAG=r4f STEPS=tests,smoke,bench,rocprof,workloads,extras \
WORKLOADS="config3 records" \
EXTRA1="bash tools/ab_lib.sh gpurun_out/r4f/ab_pair_mixed tools/ab/libhundcrc_r4base.so hunddb_amd/libhundcrc.so 4 --workload config3" \
bash tools/gpu_session.sh
