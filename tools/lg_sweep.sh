mkdir -p gpurun_out/lgs
WL=${WL:-config2 offlen4k}; LGS=${LGS:-5 6 7}
for r in 1 2; do for w in $WL; do for lg in $LGS; do
  HC_LG_CHUNK=$lg timeout -k 10 200 python bench.py --workload $w --steps 100 --warmup 10 --pmc off --cpu-seconds 0 --json-out gpurun_out/lgs/${w}_${lg}_$r.json > /dev/null 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/lgs/${w}_${lg}_$r.json')); print('$w lg $lg r $r', d['roofline']['frac'])"
done; done; done
