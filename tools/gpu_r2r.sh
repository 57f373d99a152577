# round 2: what costs config 5's verify (4 KiB) against the 8 KiB CRC stream
OUT=${OUT:-r2r}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 200 python3 -u $B --mode host8k --bsize 4096 --blocks 2000000 > gpurun_out/$OUT/h4k_2m_crc.json 2> gpurun_out/$OUT/e1.err &&
timeout -k 10 200 python3 -u $B --mode host8k --bsize 4096 --blocks 2000000 --verify 1 > gpurun_out/$OUT/h4k_2m_verify.json 2> gpurun_out/$OUT/e2.err &&
timeout -k 10 240 python3 -u $B --mode host8k --bsize 4096 --blocks 5264137 > gpurun_out/$OUT/h4k_5m_crc.json 2> gpurun_out/$OUT/e3.err &&
timeout -k 10 240 python3 -u $B --mode host8k --bsize 4096 --blocks 5264137 --verify 1 > gpurun_out/$OUT/h4k_5m_verify.json 2> gpurun_out/$OUT/e4.err &&
timeout -k 10 240 python3 -u $B --mode host8k --bsize 8192 --blocks 2632068 > gpurun_out/$OUT/h8k_20g_crc.json 2> gpurun_out/$OUT/e5.err &&
HC_CHUNK_MB=256 timeout -k 10 240 python3 -u $B --mode host8k --bsize 4096 --blocks 5264137 > gpurun_out/$OUT/h4k_5m_crc_c256.json 2> gpurun_out/$OUT/e6.err
