#!/bin/bash
# round 4, session l: k_seg_stream's 4-byte shifts through conflict-free nibble
# tables (nibtie), and with paired placements (pairnibtie); seg parity through
# both, A/B on records, and one LDS counter pass per build
TAG=r4l STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/seg5_nibtie/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="HUNDCRC_LIB=\$PWD/tools/ab/seg5_pairnibtie/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4l/ab_seg 3 prod=hunddb_amd/libhundcrc.so nibtie=tools/ab/seg5_nibtie/libhundcrc.so pairnibtie=tools/ab/seg5_pairnibtie/libhundcrc.so noev=tools/ab/seg2_noev/libhundcrc.so -- --workload records" \
EXTRA4="cd /tmp && for b in prod:hunddb_amd/libhundcrc.so nibtie:tools/ab/seg5_nibtie/libhundcrc.so; do HUNDCRC_LIB=\$GRAFT_REPO_ROOT/\${b#*:} timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex k_seg_stream --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4l/pmc_\${b%%:*} -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --steps 3 --warmup 1 --cpu-seconds 0 --pmc off || exit \$?; done" \
bash tools/gpu_session.sh
