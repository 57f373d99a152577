#!/bin/bash
# round 6, session j: the sort with batched loads (kSB records a thread per pass) -- its tests and
# the phase clock (what batching buys the sort before deciding where it lives)
TAG=${TAG:-r6j} STEPS=extras \
EXTRA1="timeout -k 10 300 python -u -m pytest tests/test_gpu_seg_sort.py -x -q --timeout 120 --timeout-method thread" \
EXTRA2="timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000,500000 --calls 2" \
EXTRA3="timeout -k 10 300 python bench.py --workload records_shuffled --cpu-seconds 0 --host-leg off --json-out gpurun_out/r6j/bench_records_shuffled.json" \
bash tools/gpu_session.sh
