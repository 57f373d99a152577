#!/bin/bash
# round 4, session h: k_seg_stream's event words collected per group and
# stored by two straight-line buffer stores (hipcc's waits exact: vmcnt(6));
# GPU suite, then A/B against the 00c7711 library on the records workload
TAG=r4h STEPS=tests,extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4h/ab_seg 3 base=tools/ab/base00c/libhundcrc.so new=hunddb_amd/libhundcrc.so -- --workload records" \
EXTRA2="cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4h/prof_rec -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records --cpu-seconds 0 --pmc off --steps 10" \
bash tools/gpu_session.sh
