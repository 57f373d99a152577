#!/bin/bash
# round 6, session q: HC_SEG_LG_CHUNK below r6p's best (5) on the record workloads and blocks8188
set -u
mkdir -p gpurun_out/r6q
for w in records records_gapped records_shuffled blocks8188; do
  for k in 5 2 3 4 5 7; do
    HC_SEG_LG_CHUNK=$k timeout -k 10 200 python bench.py --workload $w --cpu-seconds 0 --pmc off --host-leg off \
      --json-out gpurun_out/r6q/${w}_$k.json > gpurun_out/r6q/${w}_$k.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r6q/${w}_$k.json')); print('$w', $k, d['roofline']['frac'])"
  done
done
