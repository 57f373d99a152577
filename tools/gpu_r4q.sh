# the host link's ceiling (pinned H2D) beside the host batches on the same box
OUT=${OUT:-r4q}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python tools/h2d_peak.py --json-out gpurun_out/$OUT/h2d.json > gpurun_out/$OUT/h2d.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_host.py --mode host8k --mem pinned > gpurun_out/$OUT/host8k_pinned.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_host.py --mode config5 --mem pinned --records 2000000 > gpurun_out/$OUT/config5_2m_pinned.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_host.py --mode replay --mem pinned --records 2000000 > gpurun_out/$OUT/replay_2m_pinned.log 2>&1 || exit $?
