#!/bin/bash
# round 6, session o: kernel split of records_shuffled and records at HEAD (rocprofv3 kernel trace)
set -u
mkdir -p gpurun_out/r6o
for w in records_shuffled records; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6o/prof_$w -o run \
     -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --pmc off --cpu-seconds 0 --host-leg off --steps 10 \
     > $GRAFT_REPO_ROOT/gpurun_out/r6o/bench_$w.log 2>&1) || exit $?
  python3 - $GRAFT_REPO_ROOT/gpurun_out/r6o/prof_$w/run_kernel_stats.csv $w <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(sys.argv[2], r["Name"].split("(")[0].split("::")[-1], r["Calls"], r["AverageNs"])
PY
done
