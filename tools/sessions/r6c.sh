#!/bin/bash
# round 6, session c: the sorted view (seg_sort in k_seg_stream, grid barriers) -- its own tests
# first under a short limit, then the seg / window / fuzz / graph suites it touches, then
# records_shuffled / records / records_gapped benches (the main stream paths must not lose) and a
# kernel trace of records_shuffled
R='$GRAFT_REPO_ROOT'
TAG=${TAG:-r6c} STEPS=extras \
EXTRA1="timeout -k 10 240 python -u -m pytest tests/test_gpu_seg_sort.py -x -v --timeout 120 --timeout-method thread" \
EXTRA2="timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py tests/test_gpu_seg_blocks.py tests/test_gpu_graphs.py -x -q --timeout 240 --timeout-method thread" \
EXTRA3="for w in records_shuffled records records_gapped; do timeout -k 10 300 python bench.py --workload \$w --cpu-seconds 0 --host-leg off --json-out gpurun_out/r6c/bench_\$w.json || exit \$?; done" \
EXTRA4="cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6c/prof_records_shuffled -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_shuffled --pmc off --cpu-seconds 0 --steps 10" \
bash tools/gpu_session.sh
