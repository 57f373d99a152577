#!/bin/bash
# round 6, closing run part b at HEAD: the record and block workloads' lines (PMC traffic summed
# over each dispatch's kernels, cpu_baseline) and their rocprofv3 kernel splits
TAG=${TAG:-final} STEPS=workloads,extras \
WORKLOADS="records records_gapped records_shuffled records4k_shuffled blocks4092 blocks8188" \
EXTRA1="bash tools/prof_workloads.sh gpurun_out/${TAG:-final} records records_gapped records_shuffled records4k_shuffled blocks8188" \
bash tools/gpu_session.sh
