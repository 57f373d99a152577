#!/bin/bash
# round 6, closing run part c at HEAD: every other workload's line
TAG=${TAG:-final} STEPS=workloads \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k unframe16k" \
bash tools/gpu_session.sh
