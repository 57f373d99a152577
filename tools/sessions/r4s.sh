#!/bin/bash
# round 4, session s: the packed-record stream against k_crc_any by batch size
# (where HC_SEG_MIN_MSGS should sit), config 5's law and equal 1 KiB records
TAG=r4s STEPS=extra \
EXTRA="timeout -k 10 600 python tools/seg_threshold.py > gpurun_out/r4s/seg_threshold.jsonl" \
bash tools/gpu_session.sh
