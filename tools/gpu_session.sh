#!/bin/bash
# One parameterised GPU session: the exact command behind every GPU call of
# round 3 (rounds 1-2 kept one gpu_r*.sh script per call; they are in git
# history up to commit d623f6c).  Run as
#   gpurun --timeout 1200 -- 'TAG=r3a STEPS=tests,smoke,bench,rocprof bash tools/gpu_session.sh'
# Every step runs under its own `timeout -k 10`, writes gpurun_out/$TAG/<step>.log
# and prints its tail.  The session ends at the first step that fails with
# anything other than plain test failures (rc 1): a fault, an abort, a time
# limit or a hang starts nothing more on the GPU.
#
# STEPS (comma-separated, in order):
#   tests      pytest -m gpu (FILES narrows the paths, K selects with -k)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py $BENCH_ARGS -> bench.json
#   rocprof    rocprofv3 --kernel-trace --stats of bench.py $BENCH_ARGS (no PMC passes, no CPU leg)
#   workloads  bench.py --workload W for every W in $WORKLOADS -> bench_W.json
#   pmc        one rocprofv3 --pmc pass per ';'-separated counter group of $PMC over $PMC_CMD
#   rehearse   bench.py --gpus 2 over gloo, two ranks sharing the one GPU
#   extra      bash -c "$EXTRA"
#   extras     bash -c "$EXTRA1" ... "$EXTRA9", one step each
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${TAG:-sess}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench,rocprof}
BENCH_ARGS=${BENCH_ARGS:-}
WORKLOADS=${WORKLOADS:-northstar config2 config3 offlen4k 16k verify config4 frame unframe records}

st() {  # st <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "[sess] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[sess] $name rc=$rc"
  tail -4 "$OUT/$name.log" | cut -c1-800
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
stop() { echo "[sess] stopping after rc=$1"; exit "$1"; }

IFS=',' read -ra LIST <<< "$STEPS"
for s in "${LIST[@]}"; do
  case "$s" in
  tests)
    args=(-u -m pytest ${FILES:-tests} -m gpu -q -x --timeout 240 --timeout-method thread)
    [ -n "${K:-}" ] && args+=(-k "$K")
    st tests 1100 python "${args[@]}"; rc=$?; ok $rc || stop $rc
    [ $rc -eq 1 ] && grep -E "FAILED|Error" "$OUT/tests.log" | head -20 ;;
  smoke)
    st smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || stop $? ;;
  bench)
    st bench 600 python bench.py $BENCH_ARGS --json-out "$OUT/bench.json" || stop $? ;;
  rocprof)
    (cd /tmp && st rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
      -- python3 "$R/bench.py" $BENCH_ARGS --pmc off --cpu-seconds 0 --host-leg off --json-out "$OUT/bench_under_rocprof.json") || stop $? ;;
  workloads)
    for w in $WORKLOADS; do
      st "bench_$w" 600 python bench.py --workload "$w" $BENCH_ARGS --json-out "$OUT/bench_$w.json" || stop $?
    done ;;
  pmc)
    IFS=';' read -ra GROUPS_ <<< "${PMC:?PMC=counter groups}"
    k=0
    for g in "${GROUPS_[@]}"; do
      k=$((k + 1))
      (cd /tmp && st "pmc$k" 120 rocprofv3 --pmc $g --kernel-include-regex "${PMC_KERNEL:-k_crc_grp}" \
        --output-format csv -d "$OUT/pmc$k" -o run -- ${PMC_CMD:?PMC_CMD=program and args}) || stop $?
    done ;;
  rehearse)
    HC_DIST_BACKEND=gloo st rehearse_n2 600 python bench.py --gpus 2 --steps 5 --warmup 2 --blocks 2000000 \
      --cpu-seconds 0 --pmc off --json-out "$OUT/rehearse_n2.json" || stop $? ;;
  extra)
    st extra 900 bash -c "${EXTRA:?EXTRA=command}" || stop $? ;;
  extras)
    # EXTRA1 .. EXTRA9, each its own step (extra1.log ...); a plain failure
    # (rc 1) goes on to the next, a fault / abort / time limit ends the session
    for k in 1 2 3 4 5 6 7 8 9; do
      v="EXTRA$k"
      [ -n "${!v:-}" ] || continue
      st "extra$k" 600 bash -c "${!v}"; rc=$?; ok $rc || stop $rc
    done ;;
  *)
    echo "[sess] unknown step $s"; exit 2 ;;
  esac
done
echo "[sess] done"
