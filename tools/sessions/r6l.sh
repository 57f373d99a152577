#!/bin/bash
# round 6, session l: which half of r6k's small-gap combine change cost it 33 us -- kernel traces of
# records_gapped with HEAD before it (r6k_head), r6k's build (loads hoisted + inverse word chain),
# per-sub-pass loads + inverse chain (va_perpass), hoisted loads + round 5's byte chain (va_sarwate)
set -u
mkdir -p gpurun_out/r6l
for v in r6k_head cur va_perpass va_sarwate; do
  lib=$GRAFT_REPO_ROOT/tools/ab/$v/libhundcrc.so; [ $v = cur ] && lib=$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so
  (cd /tmp && HUNDCRC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $GRAFT_REPO_ROOT/gpurun_out/r6l/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload records_gapped \
     --pmc off --cpu-seconds 0 --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/r6l/bench_$v.log 2>&1) || exit $?
  python3 - $GRAFT_REPO_ROOT/gpurun_out/r6l/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "seg_" in r["Name"]: print(sys.argv[2], r["Name"].split("(")[0].split("::")[-1], r["Calls"], r["AverageNs"])
PY
done
