#!/bin/bash
# round 4, session tt: k_unframe with payload_out at every byte alignment
# (the new parity test), plus the read-block tests around it
TAG=r4tt STEPS=extras \
EXTRA1="timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k 'dev_read_blocks or frame_unframe' > gpurun_out/r4tt/tests.log 2>&1; rc=\$?; tail -3 gpurun_out/r4tt/tests.log; exit \$rc" \
bash tools/gpu_session.sh
