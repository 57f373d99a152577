# balanced last round of the per-CU chunk hand-out (kBal) vs production
OUT=${OUT:-r4v}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
for cfg in "8192 1000000" "4096 1000000" "16384 500000" "8192 2000000"; do
set -- $cfg
KB2_BAL=1 timeout -k 10 300 ./kbench2 $1 $2 5 5 > ../gpurun_out/$OUT/bal_$1_$2.txt 2>&1 || exit $?
done
