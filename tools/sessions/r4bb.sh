#!/bin/bash
# round 4, session bb: the integer VALU rate of MD5's step mix against f32 FMA
# at 8 waves per SIMD (tools/valu_rate.hip), with one PMC pass for the clock
TAG=r4bb STEPS=extras \
EXTRA1="timeout -k 10 120 ./tools/valu_rate > gpurun_out/r4bb/valu_rate.jsonl" \
EXTRA2="cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4bb/pmc -o run -- \$GRAFT_REPO_ROOT/tools/valu_rate" \
bash tools/gpu_session.sh
