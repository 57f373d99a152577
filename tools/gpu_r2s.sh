# round 2: GPU-side verify / overlapped stamping in host batches
OUT=${OUT:-r2s}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 240 python3 -u $B --mode host8k --bsize 4096 --blocks 5264137 > gpurun_out/$OUT/h4k_5m_crc.json 2> gpurun_out/$OUT/e1.err &&
timeout -k 10 240 python3 -u $B --mode host8k --bsize 4096 --blocks 5264137 --verify 1 > gpurun_out/$OUT/h4k_5m_verify.json 2> gpurun_out/$OUT/e2.err &&
timeout -k 10 300 python3 -u $B --mode config5 --records 2000000 --mem pinned > gpurun_out/$OUT/config5_2m_pinned.json 2> gpurun_out/$OUT/e3.err &&
timeout -k 10 300 python3 -u $B --mode replay --records 2000000 --mem pinned > gpurun_out/$OUT/replay2m_pinned.json 2> gpurun_out/$OUT/e4.err &&
timeout -k 10 300 python3 -u $B --mode replay --records 2000000 --mem pageable > gpurun_out/$OUT/replay2m_pageable.json 2> gpurun_out/$OUT/e5.err
