#!/bin/bash
# A/B of two builds of libhundcrc on the row-f4 MD5 leaves (tools/bench_md5.py),
# alternating processes: ab_md5.sh <out_dir> <libA> <libB> <rounds> [parts]
set -u
out=$1; A=$2; B=$3; n=$4; parts=${5:-loguniform,4096}
mkdir -p "$out"
for i in $(seq 1 "$n"); do
  for t in A B; do
    lib=$A; [ $t = B ] && lib=$B
    for p in ${parts//,/ }; do
      HUNDCRC_LIB=$(readlink -f "$lib") timeout -k 10 300 python tools/bench_md5.py --only "$p" --cpu-seconds 0 \
        > "$out/ab_${t}_${p}_$i.log" 2>&1 || exit $?
      echo "$t $i $p $(grep -o '"GBps": [0-9.]*' "$out/ab_${t}_${p}_$i.log")"
    done
  done
done
