#!/bin/bash
# round 5, session p: k_md5's waves take ranges of equal work on off/len batches (r4: the heaviest
# of 2048 count-split ranges is 16.8 % above the mean on 2M log-uniform records).  The Merkle
# suite, then tools/bench_md5.py log-uniform and 4096 B twice, and a rocprof of one log-uniform run.
TAG=r5p STEPS=tests,extras \
FILES="tests/test_gpu_merkle.py" \
EXTRA1="python tools/bench_md5.py --only loguniform --cpu-seconds 0" \
EXTRA2="python tools/bench_md5.py --only 4096 --cpu-seconds 0" \
EXTRA3="python tools/bench_md5.py --only loguniform --cpu-seconds 0" \
EXTRA4="cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5p/prof_md5 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_md5.py --only loguniform --cpu-seconds 0" \
bash tools/gpu_session.sh
