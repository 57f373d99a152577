#!/bin/bash
# round 6, session e: the sorted view with batched atomics / one 16-B scatter, the key range
# computed inside the sort (the plan back to round 5's work) and one prologue reduction --
# its tests, the phase clock, the in-order stream paths A/B against the pre-sort library
# (with kernel traces), and the records_shuffled line
TAG=${TAG:-r6e} STEPS=extras \
EXTRA1="timeout -k 10 300 python -u -m pytest tests/test_gpu_seg_sort.py -x -q --timeout 120 --timeout-method thread" \
EXTRA2="timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000,500000 --calls 2" \
EXTRA3="bash tools/ab_lib.sh gpurun_out/r6e/ab_records tools/ab/pre_sort/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records && bash tools/ab_lib.sh gpurun_out/r6e/ab_records_gapped tools/ab/pre_sort/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_gapped" \
EXTRA4="cd /tmp && HUNDCRC_LIB=\$GRAFT_REPO_ROOT/tools/ab/pre_sort/libhundcrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6e/prof_A_records -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --pmc off --cpu-seconds 0 --steps 10 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6e/prof_B_records -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --pmc off --cpu-seconds 0 --steps 10" \
EXTRA5="timeout -k 10 300 python bench.py --workload records_shuffled --cpu-seconds 0 --host-leg off --json-out gpurun_out/r6e/bench_records_shuffled.json" \
bash tools/gpu_session.sh
