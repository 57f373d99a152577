#!/bin/bash
# round 4, session v: small device block batches by layout (uniform, off/len,
# off/len the streaming kernel leaves to the sweep) and their kernel times
TAG=r4v STEPS=extras \
EXTRA1="timeout -k 10 300 python tools/small_offlen.py > gpurun_out/r4v/small_offlen.jsonl" \
EXTRA2="cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4v/prof -o run -- python3 \$GRAFT_REPO_ROOT/tools/small_offlen.py --ns 4096 --calls 10" \
bash tools/gpu_session.sh
