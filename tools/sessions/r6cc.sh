#!/bin/bash
# round 6, session cc: the sort from 2^18 records (HC_SEG_SORT_MIN's default after r6bb) -- the
# seg suites, windows, graphs, fuzz and workload tests, then records_shuffled at 128k, 256k and 2M
set -u
mkdir -p gpurun_out/r6cc
timeout -k 10 700 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py tests/test_gpu_any_windows.py tests/test_gpu_graphs.py tests/test_gpu_fuzz.py tests/test_gpu_bench_workloads.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6cc/tests.log 2>&1 || { tail -30 gpurun_out/r6cc/tests.log; exit 1; }
tail -2 gpurun_out/r6cc/tests.log
for n in 131072 262144 2000000; do
  timeout -k 10 200 python bench.py --workload records_shuffled --blocks $n --pmc off --host-leg off --cpu-seconds 0 \
    --json-out gpurun_out/r6cc/shuf_$n.json > gpurun_out/r6cc/shuf_$n.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r6cc/shuf_$n.json')); print($n, d['ms_per_step'], d['roofline']['frac'], d['config'].get('stream_mode'))"
done
