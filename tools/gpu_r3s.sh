# round 2: XCD-contiguous slots at 8 KiB, third box, more rounds
OUT=${OUT:-r3s}
mkdir -p gpurun_out/$OUT
cd tools || exit 1
timeout -k 10 250 ./kbench2 8192 1000000 10 5 > ../gpurun_out/$OUT/kb2_8192.txt 2>&1
