#!/bin/bash
# round 4, session o: GPU suite + smoke with k_seg_stream's events before the
# refill (no row copy), the records bench + rocprof, A/B against 4c3f930's library
TAG=r4o STEPS=tests,smoke,extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4o/ab_seg 3 base=tools/ab/base00c/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload records" \
EXTRA2="timeout -k 10 300 python bench.py --workload records --json-out gpurun_out/r4o/bench_records.json" \
EXTRA3="cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4o/prof_rec -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10" \
bash tools/gpu_session.sh
