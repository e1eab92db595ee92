#!/bin/bash
# Round-4 session C: where did C2 / R = 8 lose time since round 3? Whole-library A/B
# (round-3 tree r3, e9afe17 e9, HEAD head) at C2 and at R = 1 / 8 parts.
export VNAMES="r3 e9 c40 head" VROUNDS=3
export PLIBS="--parts 1 8 raytrace-we-gpu_amd/lib/variants/librtx_r3.so raytrace-we-gpu_amd/lib/variants/librtx_e9.so raytrace-we-gpu_amd/lib/variants/librtx_head.so"
bash tools/gpu_session.sh R6c variants parts
