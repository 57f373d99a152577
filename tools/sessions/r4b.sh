#!/bin/bash
# round 4, session b: GPU suite after the plan-free k_seg_stream fix (waits) and the host task pool;
# k_seg A/B against round 3's dispatch; host-entry crossover with the pool; paired placement A/B, more rounds
TAG=r4b STEPS=tests,extras \
EXTRA1="bash tools/ab_lib.sh gpurun_out/r4b/ab_seg tools/ab/libhundcrc_r4base.so hunddb_amd/libhundcrc.so 3 --workload records" \
EXTRA2="python tools/crossover.py --json-out gpurun_out/r4b/crossover.jsonl" \
EXTRA3="bash tools/ab_lib.sh gpurun_out/r4b/ab_pair4k hunddb_amd/libhundcrc.so tools/ab/libhundcrc_pair.so 3 --workload config2" \
EXTRA4="bash tools/ab_lib.sh gpurun_out/r4b/ab_pair8k hunddb_amd/libhundcrc.so tools/ab/libhundcrc_pair.so 2 --workload northstar" \
bash tools/gpu_session.sh
