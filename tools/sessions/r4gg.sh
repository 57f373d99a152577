#!/bin/bash
# round 4, session gg: the packed-record fallback folded into k_seg_combine (three
# launches a dispatch instead of four): GPU suite + smoke, small-batch timings,
# records A/B against 3ef75f8 + rocprof
TAG=r4gg STEPS=tests,smoke,extras \
EXTRA1="timeout -k 10 300 python tools/seg_threshold.py --ns 16,256,1024,4096,65536 > gpurun_out/r4gg/seg_threshold.jsonl" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4gg/ab_rec 3 base=tools/ab/base3ef/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload records" \
EXTRA3="cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4gg/prof_rec -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10" \
bash tools/gpu_session.sh
