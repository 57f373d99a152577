#!/bin/bash
# round 6, session v: the small-gap combine's gap from the two aligned 16-B chunks ending at the record (va_gap2)
# against <= 3 chunk loads (HEAD) -- the seg suites on the variant, kernel traces of both on
# records_gapped, an alternating A/B
set -u
mkdir -p gpurun_out/r6v
V=$GRAFT_REPO_ROOT/tools/ab/va_gap2/libhundcrc.so
HUNDCRC_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_seg_sort.py tests/test_gpu_seg_blocks.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6v/tests.log 2>&1 || { tail -30 gpurun_out/r6v/tests.log; exit 1; }
tail -2 gpurun_out/r6v/tests.log
for v in head gap2; do
  lib=$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so; [ $v = gap2 ] && lib=$V
  (cd /tmp && HUNDCRC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6v/prof_$v -o run \
     -- python3 $GRAFT_REPO_ROOT/bench.py --workload records_gapped --pmc off --cpu-seconds 0 --host-leg off --steps 10 \
     > $GRAFT_REPO_ROOT/gpurun_out/r6v/bench_$v.log 2>&1) || exit $?
  python3 - $GRAFT_REPO_ROOT/gpurun_out/r6v/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "seg_" in r["Name"]: print(sys.argv[2], r["Name"].split("(anonymous namespace)::")[-1][:14], r["Calls"], r["AverageNs"])
PY
done
bash tools/ab_lib.sh gpurun_out/r6v/ab_records_gapped hunddb_amd/libhundcrc.so $V 2 --workload records_gapped
