#!/bin/bash
# Round-4 session L: the row-split pre-pass (0.85 ms of an R = 8 share): caps with saturated keys, 1-spp.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6l; mkdir -p $OUT
V=raytrace-we-gpu_amd/lib/variants
timeout -k 10 600 python tools/heavy_sweep.py --parts 8 4 --rounds 2 --sets "default;capS=24;capS=32;capS=48;capS=64" > $OUT/hsweep.jsonl 2>&1 &&
timeout -k 10 300 python tools/part_scaling.py $V/librtx_base.so $V/librtx_cspp1.so --parts 1 8 4 > $OUT/parts_cspp.jsonl 2>&1 &&
timeout -k 10 300 python tools/part_scaling.py $V/librtx_base.so $V/librtx_cspp1.so --parts 1 8 4 >> $OUT/parts_cspp.jsonl 2>&1
echo "session L rc=$?"
