#!/bin/bash
# round 6, session bb: where the sorted view starts to pay -- records_shuffled at 16k .. 2M records
# with the sort (HC_SEG_SORT_MIN=1) and without it (0: k_crc_any's work in the combine)
set -u
mkdir -p gpurun_out/r6bb
for n in 16384 32768 65536 131072 262144 524288 1048576; do
  for sm in 1 0; do
    HC_SEG_SORT_MIN=$sm timeout -k 10 200 python bench.py --workload records_shuffled --blocks $n --steps 20 --warmup 5 --pmc off --host-leg off --cpu-seconds 0 \
      --json-out gpurun_out/r6bb/shuf_${n}_$sm.json > gpurun_out/r6bb/shuf_${n}_$sm.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r6bb/shuf_${n}_$sm.json')); print($n, 'sort' if $sm else 'any', d['ms_per_step'], d['roofline']['frac'], d['config'].get('stream_mode'))"
  done
done
