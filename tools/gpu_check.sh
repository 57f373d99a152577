#!/bin/bash
# One GPU session: parity tests, smoke, bench (+ rocprofv3 kernel-trace stats).
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures, anything else = stop
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[gpu_check] $(date +%T) $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[gpu_check] $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  return $rc
}
rocm-smi --showproductname > "$OUT/rocm-smi.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"; lscpu | grep "Model name" >> "$OUT/nproc.txt"; (command -v go && go version) >> "$OUT/nproc.txt" 2>&1 || echo "go: absent" >> "$OUT/nproc.txt"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; ok_rc $rc || exit $rc
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}; rc=$?; ok_rc $rc || exit $rc
step bench 600 python bench.py ${BENCH_ARGS:-} --json-out "$OUT/bench.json"; rc=$?; ok_rc $rc || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --pmc off; rc=$?; ok_rc $rc || exit $rc
fi
echo "[gpu_check] done"
