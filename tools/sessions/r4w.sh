#!/bin/bash
# round 4, session w: k_crc_any's windows shrink on small batches (every wave
# gets one) and k_crc_grp's skip word is read before its atomic: GPU suite +
# smoke, small-batch timings against 3ef75f8's library, the off/len workloads
TAG=r4w STEPS=tests,smoke,extras \
EXTRA1="timeout -k 10 300 python tools/small_offlen.py > gpurun_out/r4w/small_offlen.jsonl && HUNDCRC_LIB=\$PWD/tools/ab/base3ef/libhundcrc.so timeout -k 10 300 python tools/small_offlen.py > gpurun_out/r4w/small_offlen_base.jsonl" \
EXTRA2="HC_SEG_MIN_MSGS=1000000000 timeout -k 10 300 python tools/seg_threshold.py --ns 16,256,4096,65536,262144 > gpurun_out/r4w/any_msgs.jsonl" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4w/ab_cfg3 2 base=tools/ab/base3ef/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload config3" \
bash tools/gpu_session.sh
