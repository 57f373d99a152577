#!/bin/bash
# round 4, session kk: framing store patterns (r4jj's partial write requests):
# k_unframe 4 KiB with plain stores on the boundary rows / on every row, and
# k_frame with the CRC written in row 0's store; parity of each variant, then
# alternating-process A/B through bench.py
T="-u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
K="dev_add_crcs or dev_read_blocks or frame_unframe or add_crcs_to_data_gpu"
TAG=r4kk STEPS=extras \
EXTRA1="for v in unf_edge_plain unf_all_plain frame_crc_row0; do HUNDCRC_LIB=\$PWD/tools/ab/\$v/libhundcrc.so timeout -k 10 300 python $T tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k '$K' > gpurun_out/r4kk/parity_\$v.log 2>&1 || exit \$?; tail -1 gpurun_out/r4kk/parity_\$v.log; done" \
EXTRA2="bash tools/ab_multi.sh gpurun_out/r4kk/ab_unf 4 prod=hunddb_amd/libhundcrc.so edge=tools/ab/unf_edge_plain/libhundcrc.so all=tools/ab/unf_all_plain/libhundcrc.so -- --workload unframe" \
EXTRA3="bash tools/ab_multi.sh gpurun_out/r4kk/ab_frame 4 prod=hunddb_amd/libhundcrc.so row0=tools/ab/frame_crc_row0/libhundcrc.so -- --workload frame" \
bash tools/gpu_session.sh
