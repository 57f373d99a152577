#!/bin/bash
# round 5, session c: the host-resident regressions r5b found (AddCRCsToData 53 -> 36 GB/s
# pinned, ReadFromDisk pageable 54 -> 37): HEAD's library (task pool: the caller runs task 0;
# read-once knobs) against the last pre-pool build (efc9ddf^, tools/ab/r3lib), alternating
# processes, and HEAD at 4 / 6 copy threads, with the cgroup's throttled time per run
H="python tools/bench_host.py"
R3=tools/ab/r3lib/libhundcrc.so
A="for m in addcrcs readdisk; do for mem in pinned pageable; do $H --mode \$m --mem \$mem; HUNDCRC_LIB=$R3 $H --mode \$m --mem \$mem; done; done"
TAG=r5c STEPS=extras \
EXTRA1="$A" \
EXTRA2="$A" \
EXTRA3="for c in 4 6; do for m in addcrcs readdisk; do HC_COPY_THREADS=\$c $H --mode \$m --mem pageable; done; done" \
EXTRA4="$H --mode replay --mem pageable && HUNDCRC_LIB=$R3 $H --mode replay --mem pageable && $H --mode replay --mem pageable && HUNDCRC_LIB=$R3 $H --mode replay --mem pageable" \
bash tools/gpu_session.sh
