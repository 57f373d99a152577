#!/bin/bash
# round 4, session r: where k_md5's issue slots go -- two PMC passes over
# tools/bench_md5.py at 4096-B records (wave cycles, waits, VALU/SALU/LDS issue, clock)
TAG=r4r STEPS=extras \
EXTRA1="cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex k_md5 --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4r/pmc1 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_md5.py --only 4096 --cpu-seconds 0" \
EXTRA2="cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex k_md5 --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4r/pmc2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_md5.py --only 4096 --cpu-seconds 0" \
bash tools/gpu_session.sh
