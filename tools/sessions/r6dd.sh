#!/bin/bash
# round 6, session dd: the packed combine with 8 sub-passes of 63 records an iteration (va_ksub8)
# against 4 (HEAD) -- packed seg tests on the variant, kernel traces of both on records
set -u
mkdir -p gpurun_out/r6dd
V=$GRAFT_REPO_ROOT/tools/ab/va_ksub8/libhundcrc.so
HUNDCRC_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6dd/tests.log 2>&1 || { tail -30 gpurun_out/r6dd/tests.log; exit 1; }
tail -2 gpurun_out/r6dd/tests.log
for i in 1 2; do
for v in head ksub8; do
  lib=$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so; [ $v = ksub8 ] && lib=$V
  (cd /tmp && HUNDCRC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6dd/prof_${v}_$i -o run \
     -- python3 $GRAFT_REPO_ROOT/bench.py --workload records --pmc off --cpu-seconds 0 --host-leg off --steps 10 \
     > $GRAFT_REPO_ROOT/gpurun_out/r6dd/bench_${v}_$i.log 2>&1) || exit $?
  python3 - $GRAFT_REPO_ROOT/gpurun_out/r6dd/prof_${v}_$i/run_kernel_stats.csv "$v $i" <<'PY'
import csv, sys
print(sys.argv[2], [(r["Name"].split("(anonymous namespace)::")[-1][:12], round(float(r["AverageNs"]) / 1e3, 1)) for r in csv.DictReader(open(sys.argv[1])) if "seg_" in r["Name"]])
PY
done
done
