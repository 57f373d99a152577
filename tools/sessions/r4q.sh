#!/bin/bash
# round 4, session q: k_md5 with the next block's message words read from LDS
# before the current block is compressed; Merkle parity through it, A/B
TAG=r4q STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/md5_pf/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_merkle.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="bash tools/ab_md5.sh gpurun_out/r4q/ab_md5 hunddb_amd/libhundcrc.so tools/ab/md5_pf/libhundcrc.so 3" \
bash tools/gpu_session.sh
