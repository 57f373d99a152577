# round 2: host AddCRCsToData, framing overlapped with a GPU batch over the source
OUT=${OUT:-r2v}
mkdir -p gpurun_out/$OUT
set -o pipefail
B=tools/bench_host.py
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "add_crc or AddCRC or frame or cpp" > gpurun_out/$OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 240 python3 -u $B --mode addcrcs --blocks 1000000 --mem pageable > gpurun_out/$OUT/addcrcs_pageable.json 2> gpurun_out/$OUT/e1.err &&
timeout -k 10 240 python3 -u $B --mode addcrcs --blocks 1000000 --mem pinned > gpurun_out/$OUT/addcrcs_pinned.json 2> gpurun_out/$OUT/e2.err &&
HC_COPY_THREADS=16 timeout -k 10 240 python3 -u $B --mode addcrcs --blocks 1000000 --mem pageable > gpurun_out/$OUT/addcrcs_pageable_t16.json 2> gpurun_out/$OUT/e3.err
