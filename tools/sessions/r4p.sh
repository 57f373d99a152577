#!/bin/bash
# round 4, session p: full run at HEAD -- GPU suite + smoke, the headline bench
# + rocprof, every BASELINE workload, and the N = 2 rehearsal over gloo
TAG=r4p STEPS=tests,smoke,bench,rocprof,workloads,rehearse \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe records" \
bash tools/gpu_session.sh
