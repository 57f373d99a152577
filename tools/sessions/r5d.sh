#!/bin/bash
# round 5, session d: the full GPU suite at HEAD (gapped stream, fallback_grp, full-oracle
# configs[3] / config 5), smoke, the headline line with its new host_inclusive leg, rocprof,
# the record workloads (records4k_shuffled also by the pre-stream route), k_crc_grp's body
# refactor against round 4's library (north star, alternating processes), DESIGN §5's host
# table at full-size warm-up
H="python tools/bench_host.py"
TAG=r5d STEPS=tests,smoke,bench,rocprof,workloads,extras \
WORKLOADS="records records_gapped records4k_shuffled" \
EXTRA1="HC_SEG_MIN_MSGS=1000000000000 python bench.py --workload records4k_shuffled --cpu-seconds 0 --json-out gpurun_out/r5d/bench_records4k_shuffled_grpany.json" \
EXTRA2="bash tools/ab_lib.sh gpurun_out/r5d/ab_grp tools/ab/r4lib/libhundcrc.so hunddb_amd/libhundcrc.so 3" \
EXTRA3="$H --mode host8k --mem pinned && $H --mode host8k --mem pageable && $H --mode config5 --records 2000000 --mem pinned && $H --mode config5 --records 2000000 --mem pageable" \
EXTRA4="$H --mode replay --mem pinned && $H --mode replay --mem pageable && $H --mode addcrcs --mem pinned && $H --mode addcrcs --mem pageable && $H --mode readdisk --mem pinned && $H --mode readdisk --mem pageable" \
EXTRA5="$H --mode config5 --records 10000000 --mem pinned --steps 2" \
bash tools/gpu_session.sh
