#!/bin/bash
# round 4, session u: GPU suite + smoke with every whole-message device batch
# offered to the packed-record stream (HC_SEG_MIN_MSGS default 1), records bench
TAG=r4u STEPS=tests,smoke,extras \
EXTRA1="timeout -k 10 300 python bench.py --workload records --json-out gpurun_out/r4u/bench_records.json" \
EXTRA2="timeout -k 10 300 python tools/seg_threshold.py --ns 16,256,4096,65536 > gpurun_out/r4u/seg_threshold.jsonl" \
bash tools/gpu_session.sh
