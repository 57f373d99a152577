#!/bin/bash
# round 5, session x: the GPU suite and smoke at HEAD after the closing run (docs and the k_md5
# A/B since; the library rebuilt from the closing run's sources)
TAG=r5x STEPS=tests,smoke bash tools/gpu_session.sh
