set -e
mkdir -p gpurun_out/r5u
for lib in prod wide prod2 wide2; do
  case $lib in prod*) L="";; *) L=$PWD/tools/ab/widefirst/libhundcrc.so;; esac
  for w in blocks8188 records_gapped; do
    HUNDCRC_LIB=$L HC_SEG_MIN_BLOCKS=1 timeout -k 10 200 python bench.py --workload $w --cpu-seconds 0 --pmc off --json-out gpurun_out/r5u/${lib}_$w.json > gpurun_out/r5u/${lib}_$w.log 2>&1
  done
done
