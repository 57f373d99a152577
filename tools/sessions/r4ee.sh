#!/bin/bash
# round 4, session ee: cache policy of the row loads -- k_crc_grp with plain
# instead of nontemporal loads (north star, configs[1]); the buffer loads of
# k_seg_stream without nt (records); and the north-star target test
TAG=r4ee STEPS=extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4ee/ab_ns 3 prod=hunddb_amd/libhundcrc.so plain=tools/ab/grp_plain/libhundcrc.so -- --workload northstar" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4ee/ab_c2 2 prod=hunddb_amd/libhundcrc.so plain=tools/ab/grp_plain/libhundcrc.so -- --workload config2" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4ee/ab_rec 3 prod=hunddb_amd/libhundcrc.so plain=tools/ab/buf_plain/libhundcrc.so -- --workload records" \
EXTRA4="timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_workloads.py -m gpu -q -x -k north_star --timeout 240 --timeout-method thread" \
bash tools/gpu_session.sh
