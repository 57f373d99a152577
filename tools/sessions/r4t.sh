#!/bin/bash
# round 4, session t: small packed-record batches on both paths (16 - 4096
# records) and the kernel times behind them (rocprofv3)
TAG=r4t STEPS=extras \
EXTRA1="timeout -k 10 300 python tools/seg_threshold.py --ns 16,64,256,1024,4096 > gpurun_out/r4t/seg_small.jsonl" \
EXTRA2="cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4t/prof -o run -- python3 \$GRAFT_REPO_ROOT/tools/seg_threshold.py --ns 4096 --calls 10 --laws 1k" \
bash tools/gpu_session.sh
