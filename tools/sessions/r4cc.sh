#!/bin/bash
# round 4, session cc: full run at HEAD after the small-batch and routing
# changes -- GPU suite + smoke, headline bench + rocprof, every workload, N = 2 rehearsal
TAG=r4cc STEPS=tests,smoke,bench,rocprof,workloads,rehearse \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe records" \
bash tools/gpu_session.sh
