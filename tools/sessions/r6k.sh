#!/bin/bash
# round 6, session k: the plan counting k_crc_grp records in its checking loop (one pass, not two), and the small-gap combine's gap CRC as a word-wise inverse Horner chain with every
# sub-pass's gap dwords loaded together -- the seg suites, an alternating A/B against HEAD before it
# (tools/ab/r6k_head) on records_gapped and records, and kernel traces of both on records_gapped
TAG=${TAG:-r6k} STEPS=extras \
EXTRA1="timeout -k 10 500 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py tests/test_gpu_seg_blocks.py tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread" \
EXTRA2="bash tools/ab_lib.sh gpurun_out/r6k/ab_records_gapped tools/ab/r6k_head/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_gapped && bash tools/ab_lib.sh gpurun_out/r6k/ab_records tools/ab/r6k_head/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records && bash tools/ab_lib.sh gpurun_out/r6k/ab_blocks8188 tools/ab/r6k_head/libhundcrc.so hunddb_amd/libhundcrc.so 1 --workload blocks8188" \
EXTRA3="cd /tmp && HUNDCRC_LIB=\$GRAFT_REPO_ROOT/tools/ab/r6k_head/libhundcrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6k/prof_A_records_gapped -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --steps 10 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r6k/prof_B_records_gapped -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --steps 10" \
bash tools/gpu_session.sh
