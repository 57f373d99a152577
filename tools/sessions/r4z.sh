#!/bin/bash
# round 4, session z: k_seg_combine with every sub-pass's dependent loads issued
# first (comb_pf); seg parity through it, records A/B, and rocprof of both
TAG=r4z STEPS=extras \
EXTRA1="HUNDCRC_LIB=\$PWD/tools/ab/comb_pf/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_threads.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4z/ab_rec 3 prod=hunddb_amd/libhundcrc.so pf=tools/ab/comb_pf/libhundcrc.so -- --workload records" \
EXTRA3="cd /tmp && HUNDCRC_LIB=\$GRAFT_REPO_ROOT/tools/ab/comb_pf/libhundcrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4z/prof_pf -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4z/prof_prod -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10" \
bash tools/gpu_session.sh
