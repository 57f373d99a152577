# bench timing: per-launch events vs one pair around the K launches (wall value and launch mean)
OUT=${OUT:-r4l}
mkdir -p gpurun_out/$OUT
for k in 1 2 3; do
for m in step bracket; do
timeout -k 10 300 python bench.py --cpu-seconds 0 --pmc off --kernel-events $m --json-out gpurun_out/$OUT/b_${m}_$k.json > gpurun_out/$OUT/b_${m}_$k.log 2>&1 || exit $?
done
done
timeout -k 10 300 python bench.py --cpu-seconds 0 --pmc off --steps 100 --kernel-events step --json-out gpurun_out/$OUT/b_step_100.json > gpurun_out/$OUT/b_step_100.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 --pmc off --steps 100 --kernel-events bracket --json-out gpurun_out/$OUT/b_bracket_100.json > gpurun_out/$OUT/b_bracket_100.log 2>&1 || exit $?
