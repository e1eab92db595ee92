#!/bin/bash
# Round-4 session P: R = 4 / 2: tier 2 (coop waves, 8 rays each) against lane mode for the medium/low shares.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6p; mkdir -p $OUT
timeout -k 10 600 python tools/heavy_sweep.py --parts 4 2 --rounds 3 --sets "default;a2m=2.0;a2m=1.6;a2m=2.0,a1l=1.6;a2m=2.0,a1l=1.6,trl=0.4;a2m=2.0,a1l=1.4,trl=0.4;a2m=1.6,a1l=1.6;a2m=2.0,a1=1.4,trm=0.25" > $OUT/hsweep.jsonl 2>&1
echo "session P rc=$?"
