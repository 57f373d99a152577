#!/bin/bash
# round 5, closing run part c at HEAD: DESIGN §5's host-resident table (tools/bench_host.py) and
# the MD5 leaves (row f4)
H="python tools/bench_host.py"
TAG=${TAG:-final} STEPS=extras \
EXTRA1="$H --mode host8k --mem pinned && $H --mode host8k --mem pageable && $H --mode config5 --records 2000000 --mem pinned && $H --mode config5 --records 2000000 --mem pageable" \
EXTRA2="$H --mode replay --mem pinned && $H --mode replay --mem pageable && $H --mode addcrcs --mem pinned && $H --mode addcrcs --mem pageable && $H --mode readdisk --mem pinned && $H --mode readdisk --mem pageable" \
EXTRA3="$H --mode config5 --records 10000000 --mem pinned --steps 2" \
EXTRA4="python tools/bench_md5.py --only loguniform --cpu-seconds 0 && python tools/bench_md5.py --only 4096 --cpu-seconds 0" \
bash tools/gpu_session.sh
