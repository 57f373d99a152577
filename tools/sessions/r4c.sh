#!/bin/bash
# round 4, session c: two-chain k_md5 (row f4) parity and A/B against production;
# SQ counters of k_crc_grp at 4 KiB, production against the paired placement
R="${GRAFT_REPO_ROOT:-$(pwd)}"
PCMD="python3 $R/bench.py --child --steps 3 --warmup 1 --workload config2 --cpu-seconds 0 --pmc off --settle 0"
PMC="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
TAG=r4c STEPS=tests,extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/libhundcrc_md5.so python -u -m pytest tests/test_gpu_merkle.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA5="bash tools/ab_lib.sh gpurun_out/r4c/ab_seg tools/ab/libhundcrc_r4base.so hunddb_amd/libhundcrc.so 3 --workload records" \
EXTRA2="bash tools/ab_md5.sh gpurun_out/r4c/ab_md5 hunddb_amd/libhundcrc.so tools/ab/libhundcrc_md5.so 3" \
EXTRA3="cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex k_crc_grp --output-format csv -d $R/gpurun_out/r4c/pmc_base -o run -- $PCMD" \
EXTRA4="cd /tmp && HUNDCRC_LIB=$R/tools/ab/libhundcrc_pair.so timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex k_crc_grp --output-format csv -d $R/gpurun_out/r4c/pmc_pair -o run -- $PCMD" \
bash tools/gpu_session.sh
