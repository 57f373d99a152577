# k_unframe store order / store policy A/B (tools/kframe)
OUT=${OUT:-r4c}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 300 ./kframe 1000000 6 5 > ../gpurun_out/$OUT/kframe_pol.txt 2>&1 || exit $?
