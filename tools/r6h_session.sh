#!/bin/bash
# Round-4 session H: pixel timelines at R = 8 and 4 with the best group schedule of R6g.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6h; mkdir -p $OUT
V=raytrace-we-gpu_amd/lib/variants
S8="tg=4,tsolo=8,a1s=1.4,a1l=2.0,trs=0.4,trl=0.3"
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 8 > $OUT/pt_default.jsonl 2>&1 &&
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 8 4 --set "$S8" > $OUT/pt_best.jsonl 2>&1 &&
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 4 --set "tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3,prs=300,prl=300" > $OUT/pt_r4_prom.jsonl 2>&1
echo "session H rc=$?"
