#!/bin/bash
# round 4, session zz: the seeded random-layout suite at 40x its seeds
# (HC_FUZZ_SCALE=40: 12800 layouts through every batch entry, against the oracle)
TAG=r4zz STEPS=extras \
EXTRA1="HC_FUZZ_SCALE=40 timeout -k 10 1100 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fuzz.py > gpurun_out/r4zz/fuzz_x40.log 2>&1; rc=\$?; tail -3 gpurun_out/r4zz/fuzz_x40.log; exit \$rc" \
bash tools/gpu_session.sh
