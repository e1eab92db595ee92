#!/bin/bash
# Round-4 session R: pixel timelines (with a 1 ms throughput profile) of R = 2/4/8 shares on the new
# defaults; then the R = 8 solo bar.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6r; mkdir -p $OUT
V=raytrace-we-gpu_amd/lib/variants
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 2 4 8 > $OUT/pt.jsonl 2>&1 &&
timeout -k 10 400 python tools/heavy_sweep.py --parts 8 4 --rounds 2 --sets "default;tsolo=4;tsolo=3;tsolo=4,a1s=1.4;tsolo=4,trs=0.45;tg=2,tsolo=4" > $OUT/hsweep.jsonl 2>&1
echo "session R rc=$?"
