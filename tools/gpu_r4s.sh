# SQ counters of k_crc_grp at 1M x 4 KiB vs 1M x 8 KiB (one pass each, 8 SQ counters)
OUT=${OUT:-r4s}
R=$PWD
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
for w in config2 northstar; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --kernel-include-regex k_crc_grp --output-format csv -d $R/gpurun_out/$OUT/$w -o run -- python3 $R/bench.py --child --workload $w --steps 3 --warmup 1 --cpu-seconds 0 --pmc off --settle 0 > $R/gpurun_out/$OUT/$w.log 2>&1 || exit $?
done
