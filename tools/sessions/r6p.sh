#!/bin/bash
# round 6, session p: the stream's chunk slot size (HC_SEG_LG_CHUNK: 2^k units of 16 KiB per slot,
# 7 = 2 MiB, round 2's choice) swept on records, records_gapped and records_shuffled
set -u
mkdir -p gpurun_out/r6p
for w in records records_gapped records_shuffled; do
  for k in 7 5 6 8 9 7; do
    HC_SEG_LG_CHUNK=$k timeout -k 10 200 python bench.py --workload $w --cpu-seconds 0 --pmc off --host-leg off \
      --json-out gpurun_out/r6p/${w}_$k.json > gpurun_out/r6p/${w}_$k.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r6p/${w}_$k.json')); print('$w', $k, d['roofline']['frac'])"
  done
done
