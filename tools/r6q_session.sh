#!/bin/bash
# Round-4 session Q: the queue poll (RTX_EXHAUST_POLL) A/B with no tier 2 for medium shares, parts 1/2/4/8.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6q; mkdir -p $OUT
L=raytrace-we-gpu_amd/lib
for r in 0 1; do
  timeout -k 10 300 python tools/part_scaling.py $L/librtx.so $L/variants/librtx_nopoll.so --parts 1 2 4 8 >> $OUT/parts.jsonl 2>&1 || { echo "parts rc=$?"; exit 1; }
done
echo "session Q ok"
