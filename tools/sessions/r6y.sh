#!/bin/bash
# round 6, session y: the sort's key-range pass over each workgroup's own tile (A1 and A3 then
# re-read it from their XCD's L2) -- the sort suite, the phase clock of both builds, an alternating
# A/B against HEAD before it (r6x_head)
set -u
mkdir -p gpurun_out/r6y
H=$GRAFT_REPO_ROOT/tools/ab/r6x_head/libhundcrc.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg_sort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6y/tests.log 2>&1 || { tail -30 gpurun_out/r6y/tests.log; exit 1; }
tail -2 gpurun_out/r6y/tests.log
for v in head cur; do
  lib=$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so; [ $v = head ] && lib=$H
  HUNDCRC_LIB=$lib timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000 --calls 3 > gpurun_out/r6y/phase_$v.log 2>&1 || exit $?
  grep records gpurun_out/r6y/phase_$v.log | sed "s/^/$v /" | cut -c1-420
done
bash tools/ab_lib.sh gpurun_out/r6y/ab_records_shuffled $H hunddb_amd/libhundcrc.so 3 --workload records_shuffled && \
bash tools/ab_lib.sh gpurun_out/r6y/ab_records $H hunddb_amd/libhundcrc.so 1 --workload records
