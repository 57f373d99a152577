#!/bin/bash
# round 6, session w: k_seg_plan's grid cap (HC_SEG_PLAN_WGS) re-swept after the plan lost its
# first pass (r6k): kernel traces on records and records_gapped
set -u
mkdir -p gpurun_out/r6w
for w in records records_gapped; do
  for g in 2048 1024 4096 8192 2048; do
    (cd /tmp && HC_SEG_PLAN_WGS=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6w/prof_${w}_$g -o run \
       -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --pmc off --cpu-seconds 0 --host-leg off --steps 10 \
       > $GRAFT_REPO_ROOT/gpurun_out/r6w/bench_${w}_$g.log 2>&1) || exit $?
    python3 - $GRAFT_REPO_ROOT/gpurun_out/r6w/prof_${w}_$g/run_kernel_stats.csv "$w $g" <<'PY'
import csv, sys
print(sys.argv[2], [(r["Name"].split("(anonymous namespace)::")[-1][:12], round(float(r["AverageNs"]) / 1e3, 1)) for r in csv.DictReader(open(sys.argv[1])) if "seg_" in r["Name"]])
PY
  done
done
