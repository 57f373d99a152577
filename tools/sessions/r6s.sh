#!/bin/bash
# round 6, session s: HC_SEG_LG_CHUNK 3 against 7 on one box, alternating processes, three rounds
set -u
mkdir -p gpurun_out/r6s
for i in 1 2 3; do
  for w in records records_gapped records_shuffled; do
    for k in 7 3; do
      HC_SEG_LG_CHUNK=$k timeout -k 10 200 python bench.py --workload $w --cpu-seconds 0 --pmc off --host-leg off \
        --json-out gpurun_out/r6s/${w}_${k}_$i.json > gpurun_out/r6s/${w}_${k}_$i.log 2>&1 || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/r6s/${w}_${k}_$i.json')); print('$w', $k, $i, d['roofline']['frac'])"
    done
  done
done
# and k_crc_grp's chunk (HC_LG_CHUNK, 2^5 blocks for 8 KiB blocks since round 2) on the north star
for i in 1 2; do
  for k in 5 3 4 6; do
    HC_LG_CHUNK=$k timeout -k 10 200 python bench.py --cpu-seconds 0 --pmc off --host-leg off \
      --json-out gpurun_out/r6s/northstar_${k}_$i.json > gpurun_out/r6s/northstar_${k}_$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r6s/northstar_${k}_$i.json')); print('northstar', $k, $i, d['roofline']['frac'])"
  done
done
