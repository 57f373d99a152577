#!/bin/bash
# round 4, session x: idle workgroups of k_seg_stream / k_seg_combine / k_crc_any
# leave before their LDS table fill (small batches), on top of r4w's windows:
# GPU suite + smoke, small-batch timings, records and config3 against 3ef75f8
TAG=r4x STEPS=tests,smoke,extras \
EXTRA1="timeout -k 10 300 python tools/small_offlen.py > gpurun_out/r4x/small_offlen.jsonl" \
EXTRA2="timeout -k 10 300 python tools/seg_threshold.py --ns 16,256,1024,4096,65536,262144 > gpurun_out/r4x/seg_threshold.jsonl" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4x/ab 3 base=tools/ab/base3ef/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload config3 && bash tools/ab_multi.sh gpurun_out/r4x/ab_rec 2 base=tools/ab/base3ef/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload records" \
bash tools/gpu_session.sh
