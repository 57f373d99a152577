#!/bin/bash
# Staged GPU session: small/new-code tests first, then the full suite, smoke,
# bench (+ rocprof), an N=2 rehearsal of bench.py (ranks share the GPU, gloo),
# and optional extra steps.  Each step has its own time limit; any failure
# other than plain test failures (rc 1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sess}; mkdir -p "$OUT"; export TMPDIR=/tmp
st() { local name=$1 secs=$2; shift 2; echo "[sess] $(date +%T) $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[sess] $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-600; return $rc; }
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -n "${FIRST:-}" ]; then st first 300 python -m pytest tests -m gpu -x -q -k "$FIRST"; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
st pytest_gpu 900 python -m pytest tests -m gpu -x -q; rc=$?; ok $rc || exit $rc
st smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; ok $rc || exit $rc
if [ "${BENCH:-1}" = "1" ]; then
  st bench 600 python bench.py --json-out "$OUT/bench.json"; rc=$?; ok $rc || exit $rc
  st rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --pmc off; rc=$?; ok $rc || exit $rc
fi
if [ "${REHEARSE:-1}" = "1" ]; then
  HC_DIST_BACKEND=gloo st rehearse_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --blocks 200000 --cpu-seconds 0 --pmc off; rc=$?; ok $rc || exit $rc
fi
if [ -n "${EXTRA:-}" ]; then st extra 900 bash -c "$EXTRA"; rc=$?; ok $rc || exit $rc; fi
echo "[sess] done"
