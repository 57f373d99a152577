#!/bin/bash
# round 6, session t: more, smaller coarse buckets in the sort (HC_SEG_SORT_UC caps the units of a
# bucket: 0 = one bucket a workgroup at 2M records, ~4500 units; 2250, 1125, 563 = 2, 4, 8 a
# workgroup) on records_shuffled, alternating, with the phase clock
set -u
mkdir -p gpurun_out/r6t
for i in 1 2; do
  for uc in 0 2250 1125 563; do
    HC_SEG_SORT_UC=$uc timeout -k 10 200 python bench.py --workload records_shuffled --cpu-seconds 0 --pmc off --host-leg off \
      --json-out gpurun_out/r6t/shuf_${uc}_$i.json > gpurun_out/r6t/shuf_${uc}_$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r6t/shuf_${uc}_$i.json')); print('records_shuffled uc', $uc, $i, d['roofline']['frac'])"
  done
done
for uc in 0 1125; do
  HC_SEG_SORT_UC=$uc timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000 --calls 2 > gpurun_out/r6t/phase_$uc.log 2>&1 || exit $?
  sed "s/^/uc=$uc /" gpurun_out/r6t/phase_$uc.log | grep records | cut -c1-600
done
