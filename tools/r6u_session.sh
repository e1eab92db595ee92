#!/bin/bash
# Round-4 session U: dynamic lane-mode priority thresholds (A1/A2/A3 x the mean pixel), parts 1/2/4/8.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6u; mkdir -p $OUT
L=raytrace-we-gpu_amd/lib; V=$L/variants
for r in 0 1; do
  timeout -k 10 400 python tools/part_scaling.py $L/librtx.so $V/librtx_dA.so $V/librtx_dB.so $V/librtx_dC.so $V/librtx_dD.so $V/librtx_dE.so --parts 1 2 4 8 >> $OUT/parts.jsonl 2>&1 || { echo "parts rc=$?"; exit 1; }
done
echo "session U ok"
