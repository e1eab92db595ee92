#!/bin/bash
# Round-3 session: parity after the per-sample LDS tile, per-sample C5 A/B
# (tile vs SGPR scan), the C5 pixel timeline with big-scene promotion.
set -e
T=${1:-R4d}
tools/gpu_session.sh $T tests
timeout -k 10 400 python tools/variant_bench.py --rng per-sample --rounds 2 --frames 1 --spp 16 --grid 159 --max-spheres 100000 pstile psnotile > gpurun_out/$T/c5ps_ab.jsonl 2>&1
timeout -k 10 300 python tools/pixel_timeline.py raytrace-we-gpu_amd/lib/variants/librtx_ptime.so --parts 1 --grid 159 --cap 100000 --spp 16 > gpurun_out/$T/ptime_c5.jsonl 2>&1
