# per-kernel times of the seg dispatch (rocprofv3 kernel trace)
OUT=${OUT:-r4i}
R=$PWD
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof -o run -- $R/tools/kbench2 msg 2000000 2 3 > $R/gpurun_out/$OUT/prof_msg.txt 2>&1
