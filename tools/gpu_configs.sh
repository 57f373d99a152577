#!/bin/bash
# Full-size measurements of every BASELINE config (1 GPU), each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-cfg}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "[cfg] $(date +%T) $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[cfg] $name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400; return $rc; }
for w in ${WORKLOADS:-config2 northstar 16k config3 config4}; do
  run bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3 --pmc off --cpu-seconds 0 --json-out "$OUT/bench_$w.json" || exit $?
done
if [ "${HOST:-1}" = "1" ]; then
  run config5_pinned 900 python tools/bench_host.py --mode config5 --mem pinned --records ${RECORDS:-10000000} --steps 2 || exit $?
fi
echo "[cfg] done"
