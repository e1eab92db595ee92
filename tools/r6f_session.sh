#!/bin/bash
# Round-4 session F: pixel timelines at R = 8 (round-3 k_trace vs the grouped one, default and
# tg 4 schedules) and the R = 1 wave timeline.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6f; mkdir -p $OUT
V=raytrace-we-gpu_amd/lib/variants
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_r3ptime.so --parts 8 > $OUT/pt_r3.jsonl 2>&1 &&
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 8 > $OUT/pt_head.jsonl 2>&1 &&
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 8 --set "tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3" > $OUT/pt_head_tg4.jsonl 2>&1 &&
timeout -k 10 300 python tools/wave_timeline.py > $OUT/wt_r1.jsonl 2>&1 &&
timeout -k 10 300 python tools/wave_timeline.py --rng per-sample > $OUT/wt_r1_ps.jsonl 2>&1
echo "session F rc=$?"
