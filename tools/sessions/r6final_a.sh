#!/bin/bash
# round 6, closing run part a at HEAD: the whole GPU suite (full-oracle configs[3] and config 5
# included), smoke, the headline line (host_inclusive leg, cpu_baseline, PMC traffic) and its
# rocprofv3 summary, the N = 2 gloo rehearsal with the launcher's deadline
TAG=${TAG:-final} STEPS=tests,smoke,bench,rocprof,rehearse \
bash tools/gpu_session.sh
