#!/bin/bash
# round 5: k_md5 with 3-block stages, one stage in flight, 3 workgroups per CU (tools/ab/md5s3)
# against production (4-block stages, two in flight, 2 per CU), alternating; the Merkle suite on
# the variant first
set -e
O=gpurun_out/${TAG:-r5dd}
mkdir -p $O
HUNDCRC_LIB=$PWD/tools/ab/md5s3/libhundcrc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_merkle.py -q -x --timeout 120 --timeout-method thread > $O/tests_variant.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python tools/md5_probe.py > $O/prod$r.log 2>&1
  HUNDCRC_LIB=$PWD/tools/ab/md5s3/libhundcrc.so timeout -k 10 200 python tools/md5_probe.py > $O/s3_$r.log 2>&1
done
