#!/bin/bash
# round 4, session rr: k_unframe 8/16 KiB without the overlapping head store,
# the row-0 buffer base from wave-uniform values (unf_g96v; g96 and g96u built it from a VGPR, a readfirstlane loop): parity, bench A/B
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe or read_from_disk"
TAG=r4rr STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/unf_g96v/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4rr/parity_unf_g96v.log 2>&1; rc=\$?; tail -1 gpurun_out/r4rr/parity_unf_g96v.log; exit \$rc" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4rr/ab_unf8 4 prod=hunddb_amd/libhundcrc.so g96u=tools/ab/unf_g96v/libhundcrc.so -- --workload unframe8k" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4rr/ab_unf16 4 prod=hunddb_amd/libhundcrc.so g96u=tools/ab/unf_g96v/libhundcrc.so -- --workload unframe16k" \
bash tools/gpu_session.sh
