#!/bin/bash
# Round-3 session: GPU parity, smoke, C2/C5 bench lines, part scaling, pre-pass
# spp A/B, the C5 big-scene promotion threshold, the R = 8 pixel timeline.
set -e
T=${1:-R4c}
VROUNDS=5 VNAMES='base cspp1 cspp3' tools/gpu_session.sh $T tests smoke bench prof c5b parts variants
timeout -k 10 400 python tools/heavy_sweep.py --parts 1 --grid 159 --max-spheres 100000 --spp 16 --frames 1 --rounds 2 --set '' --set prB=40 --set prB=90 > gpurun_out/$T/c5_promB.jsonl 2>&1
timeout -k 10 300 python tools/pixel_timeline.py raytrace-we-gpu_amd/lib/variants/librtx_ptime.so --parts 8 4 > gpurun_out/$T/ptime_r8_r4.jsonl 2>&1
