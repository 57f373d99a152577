#!/bin/bash
# round 5, closing run part b at HEAD: every workload's line, the rocprof breakdowns of the record
# workloads, DESIGN §5's host-resident table, the MD5 leaves (row f4)
H="python tools/bench_host.py"
TAG=${TAG:-final} STEPS=workloads,extras \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe unframe8k unframe16k records records_gapped records4k_shuffled blocks4092 blocks8188" \
EXTRA1="bash tools/prof_workloads.sh gpurun_out/${TAG:-final} records records_gapped records4k_shuffled blocks8188" \
EXTRA2="$H --mode host8k --mem pinned && $H --mode host8k --mem pageable && $H --mode config5 --records 2000000 --mem pinned && $H --mode config5 --records 2000000 --mem pageable" \
EXTRA3="$H --mode replay --mem pinned && $H --mode replay --mem pageable && $H --mode addcrcs --mem pinned && $H --mode addcrcs --mem pageable && $H --mode readdisk --mem pinned && $H --mode readdisk --mem pageable" \
EXTRA4="$H --mode config5 --records 10000000 --mem pinned --steps 2" \
EXTRA5="python tools/bench_md5.py --only loguniform --cpu-seconds 0 && python tools/bench_md5.py --only 4096 --cpu-seconds 0" \
bash tools/gpu_session.sh
