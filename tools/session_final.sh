#!/bin/bash
# End-of-round measurement: GPU parity, smoke, the C2 bench line (with PMC
# traffic, VALU counters and the per-sample side line), its rocprof kernel
# stats, C3 and C5 lines in both RNG modes, the part-scaling rehearsal, and a
# whole-frame schedule check (promotion threshold, tail-coop size).
set -e
T=${1:-R4z}
tools/gpu_session.sh $T tests smoke bench prof c3b c5b c5ps parts
timeout -k 10 300 python tools/heavy_sweep.py --parts 1 --rounds 3 --set '' --set prL=250 --set prL=600 --set coop=16 --set coop=48 > gpurun_out/$T/r1_sweep.jsonl 2>&1
timeout -k 10 300 python tools/pixel_timeline.py raytrace-we-gpu_amd/lib/variants/librtx_ptime.so --parts 2 > gpurun_out/$T/ptime_r2.jsonl 2>&1
timeout -k 10 300 python tools/pixel_timeline.py raytrace-we-gpu_amd/lib/variants/librtx_ptime.so --parts 1 --grid 159 --cap 100000 --spp 16 > gpurun_out/$T/ptime_c5.jsonl 2>&1
