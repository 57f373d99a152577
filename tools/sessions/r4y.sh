#!/bin/bash
# round 4, session y: k_crc_any's small-batch windows + k_crc_grp's guarded skip
# atomic (the r4w build, without r4x's early exits) against 3ef75f8 on the
# off/len workloads, four rounds each
TAG=r4y STEPS=extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4y/ab_cfg3 4 base=tools/ab/base3ef/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload config3" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4y/ab_ol4k 3 base=tools/ab/base3ef/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload offlen4k" \
bash tools/gpu_session.sh
