#!/bin/bash
# timing only: the record stream with and without its event work (alternating builds)
set -e
O=gpurun_out/${TAG:-r5cc}
mkdir -p $O
for r in 1 2; do
  for w in records records_gapped; do
    timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --pmc off --cpu-seconds 0 --json-out $O/prod_${w}_$r.json > $O/prod_${w}_$r.log 2>&1
    HUNDCRC_LIB=$PWD/tools/ab/noev/libhundcrc.so timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --pmc off --cpu-seconds 0 --json-out $O/noev_${w}_$r.json > $O/noev_${w}_$r.log 2>&1
  done
done
