#!/bin/bash
# round 4, session pp: k_unframe without the overlapping head store, two forms
# at 4 KiB (noov: every lane shifted by one word; h96: lane 0's 12 bytes by a
# 12-B store) and the h96 form for 8/16 KiB (g96): parity, bench A/B
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe or read_from_disk"
TAG=r4pp STEPS=extras \
EXTRA1="for v in unf_h96 unf_g96; do HUNDCRC_LIB=\$PWD/tools/ab/\$v/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4pp/parity_\$v.log 2>&1 || exit \$?; tail -1 gpurun_out/r4pp/parity_\$v.log; done" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4pp/ab_unf 4 prod=hunddb_amd/libhundcrc.so noov=tools/ab/unf_noov/libhundcrc.so h96=tools/ab/unf_h96/libhundcrc.so -- --workload unframe" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4pp/ab_unf8 3 prod=hunddb_amd/libhundcrc.so g96=tools/ab/unf_g96/libhundcrc.so -- --workload unframe8k" \
EXTRA4="bash tools/ab_multi.sh gpurun_out/r4pp/ab_unf16 3 prod=hunddb_amd/libhundcrc.so g96=tools/ab/unf_g96/libhundcrc.so -- --workload unframe16k" \
bash tools/gpu_session.sh
