# round 2: config 5 at full size (10M records, 100 GiB pinned) + pageable replay again
OUT=${OUT:-r2t}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 400 python3 -u $B --mode config5 --records 10000000 --mem pinned > gpurun_out/$OUT/config5_10m_pinned.json 2> gpurun_out/$OUT/e1.err &&
timeout -k 10 300 python3 -u $B --mode replay --records 2000000 --mem pageable > gpurun_out/$OUT/replay2m_pageable.json 2> gpurun_out/$OUT/e2.err &&
timeout -k 10 300 python3 -u $B --mode config5 --records 2000000 --mem pageable > gpurun_out/$OUT/config5_2m_pageable.json 2> gpurun_out/$OUT/e3.err &&
timeout -k 10 240 python3 -u $B --mode host8k --mem pageable > gpurun_out/$OUT/host8k_pageable.json 2> gpurun_out/$OUT/e4.err
