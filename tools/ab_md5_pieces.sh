#!/bin/bash
# round 5: k_md5 with aligned stage pieces (the variant then under test) against the unaligned
# pieces of r5p (tools/ab/md5old, built from hunddb_amd/csrc/hc_md5.hip: production), alternating
set -e
O=gpurun_out/${TAG:-r5w}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_merkle.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python tools/md5_probe.py > $O/new$r.log 2>&1
  HUNDCRC_LIB=$PWD/tools/ab/md5old/libhundcrc.so timeout -k 10 200 python tools/md5_probe.py > $O/old$r.log 2>&1
done
timeout -k 10 200 python tools/bench_md5.py --only loguniform --cpu-seconds 0 > $O/bench_lu.log 2>&1
timeout -k 10 200 python tools/bench_md5.py --only 4096 --cpu-seconds 0 > $O/bench_4096.log 2>&1
