# k_unframe: buffer placement (kframe default vs bench.py's allocation order)
OUT=${OUT:-r4f}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 300 ./kframe 1000000 4 5 > ../gpurun_out/$OUT/kframe_default.txt 2>&1 || exit $?
KFRAME_ORDER=bench timeout -k 10 300 ./kframe 1000000 4 5 > ../gpurun_out/$OUT/kframe_benchorder.txt 2>&1 || exit $?
cd .. && timeout -k 10 300 python bench.py --workload unframe --cpu-seconds 0 --pmc off --json-out gpurun_out/$OUT/bench_unframe.json > gpurun_out/$OUT/bench_unframe.log 2>&1
