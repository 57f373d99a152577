#!/bin/bash
# round 5, session y: the 12800-layout fuzz sweep at HEAD (the small-gap mode, the block route and
# k_crc_grp-first are new this round)
TAG=r5y STEPS=extra \
EXTRA="HC_FUZZ_SCALE=40 timeout -k 10 800 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -x --timeout 240 --timeout-method thread" \
bash tools/gpu_session.sh
