#!/bin/bash
# round 4, session a: HEAD tests + smoke + bench + rocprof, host-entry crossover, k_seg A/B, paired-placement parity + A/B
TAG=r4a STEPS=tests,smoke,bench,rocprof,extras \
EXTRA1="python tools/crossover.py --json-out gpurun_out/r4a/crossover.jsonl" \
EXTRA2="bash tools/ab_lib.sh gpurun_out/r4a/ab_seg tools/ab/libhundcrc_r4base.so hunddb_amd/libhundcrc.so 2 --workload records" \
EXTRA3="HUNDCRC_LIB=\$PWD/tools/ab/libhundcrc_pair.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -q -x --timeout 120 --timeout-method thread -k 'uniform or full_size or config3 or verify or general or offlen or random'" \
EXTRA4="bash tools/ab_lib.sh gpurun_out/r4a/ab_pair4k hunddb_amd/libhundcrc.so tools/ab/libhundcrc_pair.so 2 --workload config2" \
EXTRA5="bash tools/ab_lib.sh gpurun_out/r4a/ab_pair8k hunddb_amd/libhundcrc.so tools/ab/libhundcrc_pair.so 2 --workload northstar" \
bash tools/gpu_session.sh
