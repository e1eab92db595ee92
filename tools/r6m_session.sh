#!/bin/bash
# Round-4 session M: R = 8: the tier-1 bar below the tier-2 bar (a2s) was a no-op (k1 <= kh); sweep both.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6m; mkdir -p $OUT
timeout -k 10 600 python tools/heavy_sweep.py --parts 8 --rounds 3 --sets "default;a2s=1.6;a2s=1.4,a1s=1.4;a2s=1.2,a1s=1.2;a2s=1.4,a1s=2.0;a2s=1.2,a1s=1.6;a2s=1.0,a1s=1.6;a2s=1.6,prs=300;a2s=1.4,a1s=1.4,trs=0.45;a2s=1.4,a1s=1.4,capS=48" > $OUT/hsweep.jsonl 2>&1
echo "session M rc=$?"
