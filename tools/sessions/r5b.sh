#!/bin/bash
# round 5, session b: the gapped packed-record stream -- its parity tests
# and the fallback tests that moved to unsorted batches, records / records_gapped benches;
# then DESIGN §5's host-resident table at HEAD (item 1; r5a found no box)
H="python tools/bench_host.py"
TAG=r5b STEPS=tests,workloads,extras \
FILES="tests/test_gpu_seg.py tests/test_gpu_any_windows.py tests/test_gpu_graphs.py" \
WORKLOADS="records records_gapped" \
EXTRA1="python tools/h2d_peak.py --json-out gpurun_out/r5b/h2d.json" \
EXTRA2="$H --mode host8k --mem pinned && $H --mode host8k --mem pageable" \
EXTRA3="$H --mode config5 --records 2000000 --mem pinned && $H --mode config5 --records 2000000 --mem pageable" \
EXTRA4="$H --mode replay --mem pinned && $H --mode replay --mem pageable" \
EXTRA5="$H --mode addcrcs --mem pinned && $H --mode addcrcs --mem pageable" \
EXTRA6="$H --mode readdisk --mem pinned && $H --mode readdisk --mem pageable" \
EXTRA7="$H --mode config5 --records 10000000 --mem pinned --steps 2" \
bash tools/gpu_session.sh
