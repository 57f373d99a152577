#!/bin/bash
# round 6, session x: k_seg_plan loads four records a thread before checking the first (the plan of
# the sorted view keeps one) -- the seg suites and fuzz, kernel traces, an alternating A/B against
# HEAD before it (r6x_head) on the three record workloads
set -u
mkdir -p gpurun_out/r6x
H=$GRAFT_REPO_ROOT/tools/ab/r6x_head/libhundcrc.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py tests/test_gpu_seg_blocks.py tests/test_gpu_any_windows.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6x/tests.log 2>&1 || { tail -30 gpurun_out/r6x/tests.log; exit 1; }
tail -2 gpurun_out/r6x/tests.log
for v in head cur; do
  lib=$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so; [ $v = head ] && lib=$H
  for w in records records_gapped; do
    (cd /tmp && HUNDCRC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6x/prof_${v}_$w -o run \
       -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --pmc off --cpu-seconds 0 --host-leg off --steps 10 \
       > $GRAFT_REPO_ROOT/gpurun_out/r6x/bench_${v}_$w.log 2>&1) || exit $?
    python3 - $GRAFT_REPO_ROOT/gpurun_out/r6x/prof_${v}_$w/run_kernel_stats.csv "$v $w" <<'PY'
import csv, sys
print(sys.argv[2], [(r["Name"].split("(anonymous namespace)::")[-1][:12], round(float(r["AverageNs"]) / 1e3, 1)) for r in csv.DictReader(open(sys.argv[1])) if "seg_" in r["Name"]])
PY
  done
done
for w in records records_gapped records_shuffled; do
  bash tools/ab_lib.sh gpurun_out/r6x/ab_$w $H hunddb_amd/libhundcrc.so 2 --workload $w || exit $?
done
