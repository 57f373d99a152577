#!/bin/bash
# round 6, session i: the LDS-tiled plan (k_seg_plan and the sort's plan of the sorted view) --
# the seg suites, then an alternating A/B against HEAD before it (tools/ab/pre_tile) on the record
# workloads with kernel traces, and the sort's phase clock
TAG=${TAG:-r6i} STEPS=extras \
EXTRA1="timeout -k 10 500 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py tests/test_gpu_seg_blocks.py tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py tests/test_gpu_graphs.py -x -q --timeout 240 --timeout-method thread" \
EXTRA2="bash tools/ab_lib.sh gpurun_out/r6i/ab_records tools/ab/pre_tile/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records && bash tools/ab_lib.sh gpurun_out/r6i/ab_records_gapped tools/ab/pre_tile/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_gapped && bash tools/ab_lib.sh gpurun_out/r6i/ab_records_shuffled tools/ab/pre_tile/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_shuffled" \
EXTRA3="cd /tmp && HUNDCRC_LIB=\$GRAFT_REPO_ROOT/tools/ab/pre_tile/libhundcrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6i/prof_A_records_gapped -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --steps 10 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6i/prof_B_records_gapped -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --steps 10" \
EXTRA4="timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000 --calls 2" \
bash tools/gpu_session.sh
