#!/bin/bash
# round 4, session vv: k_unframe in 8-wave workgroups at every block size
# (unf_w8all: one LDS fill of the placement columns per 8 waves): parity,
# bench A/B against production at 4 / 8 / 16 KiB
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe or read_from_disk"
TAG=r4vv STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/unf_w8all/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4vv/parity_unf_w8all.log 2>&1; rc=\$?; tail -1 gpurun_out/r4vv/parity_unf_w8all.log; exit \$rc" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4vv/ab_unf 3 prod=hunddb_amd/libhundcrc.so w8=tools/ab/unf_w8all/libhundcrc.so -- --workload unframe" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4vv/ab_unf8 3 prod=hunddb_amd/libhundcrc.so w8=tools/ab/unf_w8all/libhundcrc.so -- --workload unframe8k" \
EXTRA4="bash tools/ab_multi.sh gpurun_out/r4vv/ab_unf16 3 prod=hunddb_amd/libhundcrc.so w8=tools/ab/unf_w8all/libhundcrc.so -- --workload unframe16k" \
bash tools/gpu_session.sh
