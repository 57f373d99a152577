#!/bin/bash
# rocprofv3 --kernel-trace --stats of bench.py for each workload given (one
# profiler run per workload, no PMC passes, no CPU leg), for the per-kernel
# averages that back a workload's bench line:
#   bash tools/prof_workloads.sh <out_dir> frame unframe unframe16k records
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
out=$(readlink -f "$1"); shift
mkdir -p "$out"
export TMPDIR=/tmp
for w in "$@"; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$w" -o run \
     -- python3 "$R/bench.py" --workload "$w" --pmc off --cpu-seconds 0 --host-leg off --json-out "$out/bench_${w}_under_rocprof.json" \
     > "$out/prof_$w.log" 2>&1) || exit $?
  python3 - "$out/prof_$w/run_kernel_stats.csv" "$out/bench_${w}_under_rocprof.json" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
print(d["config"]["workload"], "bench mean launch ms", d["roofline"]["mean_launch_ms"])
for r in rows[:4]:
    print("   ", r["Name"].split("(")[0][-40:], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 2), r["Percentage"] + " %")
PY
done
