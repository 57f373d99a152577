#!/bin/bash
# round 4, session ab: k_unframe 8/16 KiB without the overlapping head store,
# group 0 stores row 0 as the 4 KiB form, the other groups keep the global store (unf_g96b, a wave-uniform branch): parity, bench A/B
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe or read_from_disk"
TAG=r4ab STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/unf_g96b/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4ab/parity_unf_g96b.log 2>&1; rc=\$?; tail -1 gpurun_out/r4ab/parity_unf_g96b.log; exit \$rc" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4ab/ab_unf8 4 prod=hunddb_amd/libhundcrc.so g96u=tools/ab/unf_g96b/libhundcrc.so -- --workload unframe8k" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4ab/ab_unf16 4 prod=hunddb_amd/libhundcrc.so g96u=tools/ab/unf_g96b/libhundcrc.so -- --workload unframe16k" \
bash tools/gpu_session.sh
