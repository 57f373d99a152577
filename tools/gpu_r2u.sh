# round 2: host AddCRCsToData throughput
OUT=${OUT:-r2u}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 240 python3 -u $B --mode addcrcs --blocks 1000000 --mem pageable > gpurun_out/$OUT/addcrcs_pageable.json 2> gpurun_out/$OUT/e1.err &&
timeout -k 10 240 python3 -u $B --mode addcrcs --blocks 1000000 --mem pinned > gpurun_out/$OUT/addcrcs_pinned.json 2> gpurun_out/$OUT/e2.err
