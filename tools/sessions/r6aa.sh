#!/bin/bash
# round 6, session aa: every uniform block length k_crc_grp refuses goes to the stream (the 2-8 KiB
# 4-B aligned exception retired after r6z) -- the block, workload, parity and fuzz suites, then the
# blocks4092 / blocks8188 lines
set -u
mkdir -p gpurun_out/r6aa
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg_blocks.py tests/test_gpu_bench_workloads.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6aa/tests.log 2>&1 || { tail -30 gpurun_out/r6aa/tests.log; exit 1; }
tail -2 gpurun_out/r6aa/tests.log
for w in blocks4092 blocks8188 blocks4092; do
  timeout -k 10 200 python bench.py --workload $w --pmc off --host-leg off --cpu-seconds 0 --json-out gpurun_out/r6aa/bench_$w.json > gpurun_out/r6aa/bench_$w.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r6aa/bench_$w.json')); r=d['roofline']; print('$w', r['kernel'], r['frac'], d['config'].get('stream_mode'))"
done
