#!/bin/bash
# round 4, session nn: k_unframe 4 KiB block-to-workgroup spread S = 1 / 2 / 4
# against production's 8: parity, bench A/B and the L2's partial write requests
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe"
TAG=r4nn STEPS=extras \
EXTRA1="for v in unf_s1 unf_s2 unf_s4; do HUNDCRC_LIB=\$PWD/tools/ab/\$v/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4nn/parity_\$v.log 2>&1 || exit \$?; tail -1 gpurun_out/r4nn/parity_\$v.log; done" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4nn/ab_unf 3 s8=hunddb_amd/libhundcrc.so s1=tools/ab/unf_s1/libhundcrc.so s2=tools/ab/unf_s2/libhundcrc.so s4=tools/ab/unf_s4/libhundcrc.so -- --workload unframe" \
EXTRA3="cd /tmp && for v in s8:hunddb_amd s1:tools/ab/unf_s1 s2:tools/ab/unf_s2 s4:tools/ab/unf_s4; do HUNDCRC_LIB=\$GRAFT_REPO_ROOT/\${v#*:}/libhundcrc.so timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_unframe --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4nn/pmc_\${v%%:*} -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload unframe --steps 5 --warmup 1 --cpu-seconds 0 --pmc off || exit \$?; done" \
bash tools/gpu_session.sh
