# round 2: XCD-contiguous slots at 16M x 8 KiB (config4 at N=1) vs the old order
OUT=${OUT:-r3u}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 400 ./kbench2 8192 16000000 3 3 > ../gpurun_out/$OUT/kb2_8192_16M.txt 2>&1 || exit $?
timeout -k 10 150 ./kbench2 8192 1000000 6 5 > ../gpurun_out/$OUT/kb2_8192.txt 2>&1
