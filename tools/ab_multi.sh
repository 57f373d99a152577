#!/bin/bash
# A/B/C/... of several builds of libhundcrc through bench.py, one process per
# run, the builds alternating within each round:
#   ab_multi.sh <out_dir> <rounds> name=lib [name=lib ...] -- <bench args...>
set -u
out=$1; n=$2; shift 2
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p "$out"
for i in $(seq 1 "$n"); do
  for nl in "${libs[@]}"; do
    t=${nl%%=*}; lib=${nl#*=}
    HUNDCRC_LIB=$(readlink -f "$lib") timeout -k 10 300 python bench.py "$@" --cpu-seconds 0 --pmc off \
      --json-out "$out/ab_${t}_$i.json" > "$out/ab_${t}_$i.log" 2>&1 || exit $?
    python3 -c "import json,sys; d=json.load(open('$out/ab_${t}_$i.json')); r=d['roofline']; print('$t', $i, d['config']['workload'], r['kernel'], r['achieved'], r['frac'])"
  done
done
