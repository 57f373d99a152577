#!/bin/bash
# round 6, session b: the records_shuffled workload as it runs today (k_crc_any's
# work in the combine), its rocprofv3 summary, and route (a) priced with a library sort (torch.sort)
# before it is built; the bench workloads test (kernel names, the new workload); pinned CPU baseline
TAG=${TAG:-r6b} STEPS=tests,workloads,extras FILES=tests/test_gpu_bench_workloads.py \
WORKLOADS="records_shuffled northstar" \
EXTRA1="timeout -k 10 300 python tools/sort_route_probe.py --records 2000000,500000" \
EXTRA2="cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6b/prof_records_shuffled -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_shuffled --pmc off --cpu-seconds 0 --steps 10" \
bash tools/gpu_session.sh
