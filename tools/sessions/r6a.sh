#!/bin/bash
# round 6, session a: the whole GPU suite at HEAD (the r5d fault's regression cases, the uniform
# message route, the inject suffix), smoke, the headline line (per-dispatch PMC traffic, converging
# CPU warm-up), and the stream workloads whose roofline now sums every kernel of the dispatch
TAG=${TAG:-r6a} STEPS=tests,smoke,bench,workloads \
WORKLOADS="records4k_shuffled records records_gapped blocks8188" \
bash tools/gpu_session.sh
