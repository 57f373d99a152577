#!/bin/bash
# round 4, session jj: k_unframe 4 KiB vs 8 KiB write/read requests at the
# L2's memory side (partial output lines at block boundaries?)
TAG=r4jj STEPS=extras \
EXTRA1="cd /tmp && for w in unframe unframe8k frame; do timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex 'k_(un)?frame' --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4jj/pmc_\$w -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload \$w --steps 5 --warmup 1 --cpu-seconds 0 --pmc off || exit \$?; done" \
bash tools/gpu_session.sh
