#!/bin/bash
# round 4, session uu: k_unframe 16 KiB in 8-wave workgroups of two blocks
# (unf16_w8): parity, bench A/B against production
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe or read_from_disk"
TAG=r4uu STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/unf16_w8/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4uu/parity_unf16_w8.log 2>&1; rc=\$?; tail -1 gpurun_out/r4uu/parity_unf16_w8.log; exit \$rc" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4uu/ab_unf16 4 prod=hunddb_amd/libhundcrc.so w8=tools/ab/unf16_w8/libhundcrc.so -- --workload unframe16k" \
bash tools/gpu_session.sh
