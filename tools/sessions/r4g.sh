#!/bin/bash
# round 4, session g: where k_seg_stream loses to k_crc_grp at 16 KiB --
# production against timing-only builds without the event work, without the
# event windows, and with events reduced to one store each (tools/ab_variant.py)
TAG=r4g STEPS=extras \
EXTRA1="bash tools/ab_multi.sh gpurun_out/r4g/ab_seg 3 prod=hunddb_amd/libhundcrc.so noev=tools/ab/seg_noev/libhundcrc.so nowin=tools/ab/seg_nowin/libhundcrc.so evcheap=tools/ab/seg_evcheap/libhundcrc.so -- --workload records" \
EXTRA2="timeout -k 10 300 python bench.py --workload 16k --cpu-seconds 0 --pmc off --json-out gpurun_out/r4g/bench_16k.json" \
bash tools/gpu_session.sh
