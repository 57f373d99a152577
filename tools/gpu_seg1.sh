#!/bin/bash
# packed-record stream (k_seg_*) against k_crc_any: words checked, timing
set -o pipefail
mkdir -p gpurun_out/seg1
for m in msg eq9815 msgbig msgsmall; do
  timeout -k 10 120 ./tools/kbench2 $m 2000000 3 3 > gpurun_out/seg1/$m.txt 2>&1 || { echo "FAIL $m rc=$?"; cat gpurun_out/seg1/$m.txt; exit 1; }
  cat gpurun_out/seg1/$m.txt
done
