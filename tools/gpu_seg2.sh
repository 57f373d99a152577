#!/bin/bash
# packed-record stream (k_seg_*): per-kernel times under rocprofv3 + A/B
set -o pipefail
mkdir -p gpurun_out/seg9
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/seg9/prof -o run -- $R/tools/kbench2 msg 2000000 1 2 > $R/gpurun_out/seg9/prof_msg.txt 2>&1 || { echo FAIL prof; tail -20 $R/gpurun_out/seg9/prof_msg.txt; exit 1; }
cd $R
for m in msg eq9815 msgbig; do
  timeout -k 10 120 ./tools/kbench2 $m 2000000 3 3 > gpurun_out/seg9/$m.txt 2>&1 || { echo "FAIL $m rc=$?"; cat gpurun_out/seg9/$m.txt; exit 1; }
  cat gpurun_out/seg9/$m.txt
done
cat $(find gpurun_out/seg9/prof -name "*kernel_stats.csv") | cut -c1-160
