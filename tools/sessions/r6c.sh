#!/bin/bash
# round 6, session c: the sorted view (seg_sort in k_seg_stream, grid barriers) -- its own tests
# first, then the seg / window / fuzz suites it touches, records_shuffled / records / records_gapped
# benches (the main stream paths must not lose), and a kernel trace of records_shuffled
TAG=${TAG:-r6c} STEPS=tests,workloads,extras \
FILES="tests/test_gpu_seg_sort.py tests/test_gpu_seg.py tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py tests/test_gpu_seg_blocks.py tests/test_gpu_graphs.py" \
WORKLOADS="records_shuffled records records_gapped" BENCH_ARGS="--cpu-seconds 0 --host-leg off" \
EXTRA1="cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6c/prof_records_shuffled -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_shuffled --pmc off --cpu-seconds 0 --steps 10" \
bash tools/gpu_session.sh
