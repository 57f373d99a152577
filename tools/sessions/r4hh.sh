#!/bin/bash
# round 4, session hh: k_unframe at 4 KiB against 8 KiB blocks -- one PMC pass
# each (instructions, waits, clock) over bench.py's device ReadFromDisk
TAG=r4hh STEPS=extras \
EXTRA1="cd /tmp && for w in unframe unframe8k; do timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex k_unframe --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r4hh/pmc_\$w -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --workload \$w --steps 5 --warmup 1 --cpu-seconds 0 --pmc off || exit \$?; done" \
bash tools/gpu_session.sh
