#!/bin/bash
# round 4, session dd: k_crc_any with windows of 32 / 16 messages on large
# batches too (load balance at the end of a batch): the records workload forced
# onto k_crc_any (HC_SEG_MIN_MSGS huge), and configs[2] (its sweep), A/B
TAG=r4dd STEPS=extras \
EXTRA1="HC_SEG_MIN_MSGS=1000000000000 bash tools/ab_multi.sh gpurun_out/r4dd/ab_any 3 prod=hunddb_amd/libhundcrc.so w32=tools/ab/any_w5/libhundcrc.so w16=tools/ab/any_w4/libhundcrc.so -- --workload records" \
EXTRA2="HUNDCRC_LIB=\$PWD/tools/ab/any_w4/libhundcrc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py -m gpu -q -x --timeout 120 --timeout-method thread" \
bash tools/gpu_session.sh
