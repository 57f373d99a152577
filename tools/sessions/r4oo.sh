#!/bin/bash
# round 4, session oo: k_unframe 4 KiB without the overlapping head store
# (unf_noov): parity, bench A/B against production, the L2's partial writes
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_read_blocks or frame_unframe or read_from_disk"
TAG=r4oo STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/unf_noov/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4oo/parity_unf_noov.log 2>&1; rc=\$?; tail -3 gpurun_out/r4oo/parity_unf_noov.log; exit \$rc" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4oo/ab_unf 4 prod=hunddb_amd/libhundcrc.so noov=tools/ab/unf_noov/libhundcrc.so -- --workload unframe" \
EXTRA3="cd /tmp && for v in prod:hunddb_amd noov:tools/ab/unf_noov; do HUNDCRC_LIB=\$GRAFT_REPO_ROOT/\${v#*:}/libhundcrc.so timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex 'k_(un)?frame' --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4oo/pmc_\${v%%:*} -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload unframe --steps 5 --warmup 1 --cpu-seconds 0 --pmc off || exit \$?; done; HUNDCRC_LIB=\$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex 'k_(un)?frame' --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4oo/pmc_frame -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload frame --steps 5 --warmup 1 --cpu-seconds 0 --pmc off" \
bash tools/gpu_session.sh
