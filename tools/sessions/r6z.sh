#!/bin/bash
# round 6, session z: round 5's per-length route choice for uniform block batches re-measured with
# the stream's 128 KiB chunk slots -- tools/seg_blocks_sweep.py on a build that offers every length
# to the stream (va_pref), k_crc_any against the stream, alternating in one process
set -u
mkdir -p gpurun_out/r6z
HUNDCRC_LIB=$GRAFT_REPO_ROOT/tools/ab/va_pref/libhundcrc.so timeout -k 10 500 python tools/seg_blocks_sweep.py --gib 4 --steps 10 --out gpurun_out/r6z/sweep.jsonl > gpurun_out/r6z/sweep.log 2>&1 || { tail -20 gpurun_out/r6z/sweep.log; exit 1; }
cut -c1-300 gpurun_out/r6z/sweep.jsonl
