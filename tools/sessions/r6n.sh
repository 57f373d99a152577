#!/bin/bash
# round 6, session n: phase B of the sort timed inside (workgroup 0's count / scan / scatter / rank
# stamps), and its ranks taken against LDS copies of the bucket's keys -- the sort suite, the phase
# clock of both builds (r6n_base: stamps only), an alternating A/B on records_shuffled and records
set -u
mkdir -p gpurun_out/r6n
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg_sort.py tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6n/tests.log 2>&1 || { tail -20 gpurun_out/r6n/tests.log; exit 1; }
tail -2 gpurun_out/r6n/tests.log
for v in base cur; do
  lib=$GRAFT_REPO_ROOT/tools/ab/r6n_base/libhundcrc.so; [ $v = cur ] && lib=$GRAFT_REPO_ROOT/hunddb_amd/libhundcrc.so
  HUNDCRC_LIB=$lib timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000 --calls 3 > gpurun_out/r6n/phase_$v.log 2>&1 || exit $?
  sed "s/^/$v /" gpurun_out/r6n/phase_$v.log | cut -c1-700
done
bash tools/ab_lib.sh gpurun_out/r6n/ab_records_shuffled tools/ab/r6n_base/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_shuffled && \
bash tools/ab_lib.sh gpurun_out/r6n/ab_records tools/ab/r6n_base/libhundcrc.so hunddb_amd/libhundcrc.so 1 --workload records
