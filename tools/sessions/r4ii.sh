#!/bin/bash
# round 4, session ii: full run at HEAD after the fallback moved into
# k_seg_combine -- GPU suite + smoke, headline bench + rocprof, every workload, N = 2 rehearsal
TAG=r4ii STEPS=tests,smoke,bench,rocprof,workloads,rehearse \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k records" \
bash tools/gpu_session.sh
