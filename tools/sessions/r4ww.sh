#!/bin/bash
# round 4, session ww: k_frame store order after the row-0 change (rows 1-3
# after the hash / after the folds) and 8-wave workgroups: parity, bench A/B
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_add_crcs or add_crcs_to_data_gpu or frame_unframe"
TAG=r4ww STEPS=extras \
EXTRA1="for v in frame_after frame_mid frame_w8; do HUNDCRC_LIB=\$PWD/tools/ab/\$v/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4ww/parity_\$v.log 2>&1 || exit \$?; tail -1 gpurun_out/r4ww/parity_\$v.log; done" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4ww/ab_frame 3 prod=hunddb_amd/libhundcrc.so after=tools/ab/frame_after/libhundcrc.so mid=tools/ab/frame_mid/libhundcrc.so w8=tools/ab/frame_w8/libhundcrc.so -- --workload frame" \
bash tools/gpu_session.sh
