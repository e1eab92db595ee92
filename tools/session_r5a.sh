#!/bin/bash
# Round-3 session: the medium-share (R = 2) tier-2 bar and promotion, and the
# large-scene pre-pass refilling from private runs.
set -e
T=${1:-R5a}
mkdir -p gpurun_out/$T
timeout -k 10 300 python tools/heavy_sweep.py --parts 2 --rounds 3 --set '' --set a2m=1.0 --set a2m=0.85 --set a2m=0.7 --set prm=300 > gpurun_out/$T/r2_sweep.jsonl 2>&1
C5V='base ppch16 ppch64' tools/gpu_session.sh $T c5
