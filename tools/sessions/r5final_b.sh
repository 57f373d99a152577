#!/bin/bash
# round 5, closing run part b at HEAD: every workload's line and the rocprof breakdowns of the
# record and block workloads
TAG=${TAG:-final} STEPS=workloads,extras \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k unframe16k records records_gapped records4k_shuffled blocks4092 blocks8188" \
EXTRA1="bash tools/prof_workloads.sh gpurun_out/${TAG:-final} records records_gapped records4k_shuffled blocks8188" \
bash tools/gpu_session.sh
