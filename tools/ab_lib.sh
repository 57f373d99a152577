#!/bin/bash
# A/B of two builds of libhundcrc through bench.py (one process per run,
# alternating): ab_lib.sh <out_dir> <libA> <libB> <rounds> <bench args...>
# e.g. HC_SEG_MIN_MSGS=1000000000000 bash tools/ab_lib.sh gpurun_out/x tools/build/libhundcrc_a.so \
#        hunddb_amd/libhundcrc.so 2 --workload records
set -u
out=$1; A=$2; B=$3; n=$4; shift 4
mkdir -p "$out"
for i in $(seq 1 "$n"); do
  for t in A B; do
    lib=$A; [ $t = B ] && lib=$B
    HUNDCRC_LIB=$(readlink -f "$lib") timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --pmc off \
      --json-out "$out/ab_${t}_$i.json" > "$out/ab_${t}_$i.log" 2>&1 || exit $?
    python3 -c "import json,sys; d=json.load(open('$out/ab_${t}_$i.json')); r=d['roofline']; print('$t', $i, d['config']['workload'], r['kernel'], r['achieved'], r['frac'])"
  done
done
