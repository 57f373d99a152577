#!/bin/bash
# round 4, session aa: k_crc_any's window sizes at every batch size around
# them (new test file), then k_seg_plan with a thread's 4 events' loads issued
# together (plan_pf): seg parity through it, records A/B + rocprof
TAG=r4aa STEPS=extras \
EXTRA1="timeout -k 10 600 python -u -m pytest tests/test_gpu_any_windows.py -m gpu -q -x --timeout 240 --timeout-method thread" \
EXTRA2="HUNDCRC_LIB=\$PWD/tools/ab/plan_pf/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py -m gpu -q -x --timeout 120 --timeout-method thread" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4aa/ab_rec 3 prod=hunddb_amd/libhundcrc.so pf=tools/ab/plan_pf/libhundcrc.so -- --workload records" \
EXTRA4="cd /tmp && HUNDCRC_LIB=\$GRAFT_REPO_ROOT/tools/ab/plan_pf/libhundcrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4aa/prof_pf -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10" \
bash tools/gpu_session.sh
