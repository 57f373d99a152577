#!/bin/bash
# k_seg_plan's grid cap (HC_SEG_PLAN_WGS) on the record workloads: rocprofv3 kernel stats per
# setting (round 5: the plan grew the gapped and small-gap checks and the k_crc_grp count)
set -e
O=gpurun_out/${TAG:-r5aa}
mkdir -p $O
export TMPDIR=/tmp
for w in records records_gapped blocks8188; do
  for g in 512 1024 2048 4096 8192; do
    (cd /tmp && HC_SEG_PLAN_WGS=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OLDPWD/$O/${w}_$g -o run -- python3 $OLDPWD/bench.py --workload $w --steps 10 --warmup 2 --pmc off \
      --cpu-seconds 0 --host-leg off --json-out $OLDPWD/$O/${w}_$g.json > $OLDPWD/$O/${w}_$g.log 2>&1)
  done
done
