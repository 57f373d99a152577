#!/bin/bash
# round 4, session xx: the round's closing full run at HEAD (the misaligned-output parity cases included) --
# GPU suite + smoke, headline bench + rocprof, every workload, N = 2 rehearsal
TAG=r4xx STEPS=tests,smoke,bench,rocprof,workloads,rehearse \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k unframe16k records" \
bash tools/gpu_session.sh
