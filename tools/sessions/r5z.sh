#!/bin/bash
# round 5, session z: the fuzz sweep (3840 layouts) with the block route (HC_SEG_MIN_BLOCKS=1) on
# half the uniform cases
TAG=r5z STEPS=extra \
EXTRA="HC_FUZZ_SCALE=20 timeout -k 10 800 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -x --timeout 240 --timeout-method thread" \
bash tools/gpu_session.sh
