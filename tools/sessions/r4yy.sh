#!/bin/bash
# round 4, session yy: the seeded random-layout suite at 10x its seeds
# (HC_FUZZ_SCALE=10: 3200 layouts through every batch entry, against the oracle)
TAG=r4yy STEPS=extras \
EXTRA1="HC_FUZZ_SCALE=10 timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fuzz.py > gpurun_out/r4yy/fuzz_x10.log 2>&1; rc=\$?; tail -3 gpurun_out/r4yy/fuzz_x10.log; exit \$rc" \
bash tools/gpu_session.sh
