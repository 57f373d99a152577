#!/bin/bash
# round 4, session e: the paired placement against round 3's finalise at 8 KiB and on mixed
# off/len blocks (more pairs, another box); k_seg_plan's grid cap swept on the records workload
TAG=r4e STEPS=extras \
EXTRA1="bash tools/ab_lib.sh gpurun_out/r4e/ab_pair8k tools/ab/libhundcrc_r4base.so hunddb_amd/libhundcrc.so 3 --workload northstar" \
EXTRA2="bash tools/ab_lib.sh gpurun_out/r4e/ab_pair_mixed tools/ab/libhundcrc_r4base.so hunddb_amd/libhundcrc.so 2 --workload config3" \
EXTRA3="for w in 16384 1024 4096 2048 16384 1024 4096 2048; do HC_SEG_PLAN_WGS=\$w timeout -k 10 300 python bench.py --workload records --cpu-seconds 0 --pmc off --json-out gpurun_out/r4e/plan_\$w.json > gpurun_out/r4e/plan_\$w.log 2>&1 || exit \$?; python3 -c \"import json; d=json.load(open('gpurun_out/r4e/plan_\$w.json')); print(\$w, d['roofline']['achieved'], d['roofline']['frac'])\"; done" \
EXTRA4="cd /tmp && HC_SEG_PLAN_WGS=2048 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4e/prof_rec2048 -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4e/prof_rec -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10" \
bash tools/gpu_session.sh
