#!/bin/bash
# round 6, session g: the sort rebuilt as an MSD pass (coarse buckets with workgroup-local LDS
# histograms, then per-bucket LDS unit counts) on the two-level barrier tree -- its tests (short
# limit), the phase clock, the records_shuffled line, and the in-order small-gap path A/B
TAG=${TAG:-r6g} STEPS=extras \
EXTRA1="timeout -k 10 300 python -u -m pytest tests/test_gpu_seg_sort.py -x -q --timeout 120 --timeout-method thread" \
EXTRA2="timeout -k 10 200 python tools/sort_phase_probe.py --records 2000000,500000 --calls 2" \
EXTRA3="timeout -k 10 300 python bench.py --workload records_shuffled --cpu-seconds 0 --host-leg off --json-out gpurun_out/r6g/bench_records_shuffled.json" \
EXTRA4="bash tools/ab_lib.sh gpurun_out/r6g/ab_records_gapped tools/ab/pre_sort/libhundcrc.so hunddb_amd/libhundcrc.so 2 --workload records_gapped" \
bash tools/gpu_session.sh
