#!/bin/bash
# round 6, session h: the whole GPU suite at HEAD (the MSD sort in k_seg_stream, every other path),
# smoke, then the sort's phase clock with the 32-bit bucket division and the records_shuffled line
TAG=${TAG:-r6h} STEPS=tests,smoke,extras \
EXTRA1="timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000,500000 --calls 2" \
EXTRA2="timeout -k 10 300 python bench.py --workload records_shuffled --cpu-seconds 0 --host-leg off --json-out gpurun_out/r6h/bench_records_shuffled.json" \
bash tools/gpu_session.sh
