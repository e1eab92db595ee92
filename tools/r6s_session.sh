#!/bin/bash
# Round-4 session S: GPU parity on the tree (k_trace in 4-wave workgroups, rolling LDS prefetch of the C5
# scan tile); parts 1/2/4/8 vs the previous commit (base) and the slot-mix A/B; C5 roll A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6s; mkdir -p $OUT
L=raytrace-we-gpu_amd/lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 0 1; do
  timeout -k 10 300 python tools/part_scaling.py $L/librtx.so $L/variants/librtx_base.so $L/variants/librtx_mix.so --parts 1 2 4 8 >> $OUT/parts.jsonl 2>&1 || { echo "parts rc=$?"; exit 1; }
done
timeout -k 10 300 python tools/variant_bench.py --grid 159 --max-spheres 100000 --spp 16 --rounds 2 --frames 1 head noroll > $OUT/c5.jsonl 2>&1
echo "session S rc=$?"
