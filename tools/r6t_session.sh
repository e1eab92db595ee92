#!/bin/bash
# Round-4 session T: dynamic lane-mode wave priority (projected remaining chain vs the mean pixel), 3 threshold
# sets, against the static hot slots; parts 1/2/4/8.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6t; mkdir -p $OUT
L=raytrace-we-gpu_amd/lib; V=$L/variants
for r in 0 1; do
  timeout -k 10 300 python tools/part_scaling.py $L/librtx.so $V/librtx_dyn.so $V/librtx_dynlo.so $V/librtx_dynhi.so --parts 1 2 4 8 >> $OUT/parts.jsonl 2>&1 || { echo "parts rc=$?"; exit 1; }
done
timeout -k 10 300 python tools/cost_maps.py $OUT/cost_maps.npz > $OUT/cost_maps.log 2>&1
echo "session T ok rc=$?"
