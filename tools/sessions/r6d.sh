#!/bin/bash
# round 6, session d: the sorted view after the thread-0 barrier fences -- its tests (short limit),
# its phase clock at 2M / 0.5M records, and an alternating A/B of the stream paths against the
# library before the sort (tools/ab/pre_sort: commit 8929892) with a kernel trace of each
TAG=${TAG:-r6d} STEPS=extras \
EXTRA1="timeout -k 10 300 python -u -m pytest tests/test_gpu_seg_sort.py -x -q --timeout 120 --timeout-method thread" \
EXTRA2="timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000,500000" \
EXTRA3="bash tools/ab_lib.sh gpurun_out/r6d/ab_records tools/ab/pre_sort/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records && bash tools/ab_lib.sh gpurun_out/r6d/ab_records_gapped tools/ab/pre_sort/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_gapped" \
EXTRA4="cd /tmp && HUNDCRC_LIB=\$GRAFT_REPO_ROOT/tools/ab/pre_sort/libhundcrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6d/prof_A_records_gapped -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --steps 10 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6d/prof_B_records_gapped -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --steps 10" \
EXTRA5="timeout -k 10 300 python bench.py --workload records_shuffled --cpu-seconds 0 --host-leg off --json-out gpurun_out/r6d/bench_records_shuffled.json" \
bash tools/gpu_session.sh
