#!/bin/bash
# Round-4 session I: tight solo loop in k_trace: timeline + sweep at R = 8 / 4.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6i; mkdir -p $OUT
V=raytrace-we-gpu_amd/lib/variants
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 8 --set "tg=4,tsolo=8,a1s=1.4,a1l=2.0,trs=0.4,trl=0.3" > $OUT/pt_best.jsonl 2>&1 &&
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 8 > $OUT/pt_default.jsonl 2>&1 &&
timeout -k 10 600 python tools/heavy_sweep.py --parts 8 4 --rounds 2 --sets 'default;tg=4,tsolo=8,a1s=1.4,a1l=2.0,trs=0.4,trl=0.3;tg=4,tsolo=6,a1s=1.4,a1l=2.0,trs=0.4,trl=0.3;tg=4,tsolo=5,a1s=1.4,a1l=2.0,trs=0.45,trl=0.35;tg=4,tsolo=8,a1s=1.2,a1l=1.8,trs=0.45,trl=0.35;tg=4,tsolo=10,a1s=1.4,a1l=2.0,trs=0.4,trl=0.3;tg=2,tsolo=8,a1s=1.6,a1l=2.0,trs=0.45,trl=0.35;tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3,prs=300,prl=300' > $OUT/hsweep.jsonl 2>&1
echo "session I rc=$?"
