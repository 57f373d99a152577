#!/bin/bash
# Host-resident / per-record measurements (tools/bench_host.py), each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-host}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "[gpu_host] $(date +%T) $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[gpu_host] $name rc=$rc"; tail -3 "$OUT/$name.log"; return $rc; }
free -g > "$OUT/free.txt" 2>&1
run host8k_pinned 300 python tools/bench_host.py --mode host8k --mem pinned && \
run host8k_pageable 300 python tools/bench_host.py --mode host8k --mem pageable && \
run config5b 300 python tools/bench_host.py --mode config5b --records ${RECORDS_B:-2000000} && \
run config5_pinned 600 python tools/bench_host.py --mode config5 --mem pinned --records ${RECORDS:-10000000} && \
run config5_pageable 600 python tools/bench_host.py --mode config5 --mem pageable --records ${RECORDS:-10000000}
echo "[gpu_host] done rc=$?"
