# round 2: k_frame / k_unframe XCD-contiguous chunk slots A/B
OUT=${OUT:-r3w}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 300 ./kframe 1000000 6 5 > ../gpurun_out/$OUT/kframe.txt 2>&1
