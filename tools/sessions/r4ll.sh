#!/bin/bash
# round 4, session ll: full run at HEAD after k_frame's row-0 store change --
# GPU suite + smoke, headline bench + rocprof, every workload, N = 2 rehearsal
TAG=r4ll STEPS=tests,smoke,bench,rocprof,workloads,rehearse \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k unframe16k records" \
bash tools/gpu_session.sh
