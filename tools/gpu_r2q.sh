# round 2: host-resident (PCIe-inclusive) rates with the pooled pipelines
OUT=${OUT:-r2q}
mkdir -p gpurun_out/$OUT
set -o pipefail
timeout -k 10 240 python3 -u tools/bench_host.py --mode host8k --mem pinned > gpurun_out/$OUT/host8k_pinned.json 2> gpurun_out/$OUT/host8k_pinned.err &&
timeout -k 10 240 python3 -u tools/bench_host.py --mode host8k --mem pageable > gpurun_out/$OUT/host8k_pageable.json 2> gpurun_out/$OUT/host8k_pageable.err &&
timeout -k 10 300 python3 -u tools/bench_host.py --mode replay --records 2000000 --mem pinned > gpurun_out/$OUT/replay2m_pinned.json 2> gpurun_out/$OUT/replay2m_pinned.err &&
timeout -k 10 300 python3 -u tools/bench_host.py --mode replay --records 2000000 --mem pageable > gpurun_out/$OUT/replay2m_pageable.json 2> gpurun_out/$OUT/replay2m_pageable.err &&
timeout -k 10 300 python3 -u tools/bench_host.py --mode config5 --records 2000000 --mem pinned > gpurun_out/$OUT/config5_2m_pinned.json 2> gpurun_out/$OUT/config5_2m_pinned.err
