#!/bin/bash
# round 4, session ss: full run at HEAD after k_unframe's 4 KiB head-store change --
# GPU suite + smoke, headline bench + rocprof, every workload, N = 2 rehearsal
TAG=r4ss STEPS=tests,smoke,bench,rocprof,workloads,rehearse \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k unframe16k records" \
bash tools/gpu_session.sh
