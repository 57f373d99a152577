#!/bin/bash
# round 4, session d: GPU suite + smoke at the paired-placement commit, the
# headline bench + rocprof, every BASELINE workload, host-entry crossover again
TAG=r4d STEPS=tests,smoke,bench,rocprof,workloads,extras \
WORKLOADS="config2 config3 offlen4k 16k verify config4 frame unframe records" \
EXTRA1="python tools/crossover.py --json-out gpurun_out/r4d/crossover.jsonl" \
bash tools/gpu_session.sh
