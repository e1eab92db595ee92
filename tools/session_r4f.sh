#!/bin/bash
# Round-3 session: C5 kernel split (rocprof), C5 pre-pass spp A/B, C3 line.
set -e
T=${1:-R4f}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_c5 -o run -- \
    python3 bench.py --spp 16 --grid 159 --max-spheres 100000 --steps 2 --warmup 1 --cpu-seconds 0 --pmc off --per-sample 0 > gpurun_out/$T/prof_c5.log 2>&1
C5V='base cpl2' tools/gpu_session.sh $T c5 c3b
