#!/bin/bash
# Round-4 session V: dynamic lane-mode priority as the default (ABI 1.4.0 prio_bar1..3): GPU parity,
# pixel timelines R = 4 / 8, an R = 8 / 4 sweep around it (tier-1 priority, bars), and the coop tail
# taking the dynamic priority too (A/B build dtail), early promotion above 2x / 3x the mean pixel (early2/3), tail promotion past 100 segments (tail100).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6v; mkdir -p $OUT
V=raytrace-we-gpu_amd/lib/variants
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -ge 124 ] && exit $rc
[ $rc -ne 0 ] && { tail -5 $OUT/tests.log; exit 1; }
timeout -k 10 300 python tools/pixel_timeline.py $V/librtx_ptime.so --parts 4 8 > $OUT/pt.jsonl 2>&1 || exit $?
timeout -k 10 500 python tools/heavy_sweep.py --parts 8 4 --rounds 2 --sets "default;pb1=0;p1=2;pb1=0.5,pb2=1.0,pb3=2.0;pb1=0.6,pb2=1.0,pb3=1.4;a1s=1.4;trs=0.45;p1=2,trs=0.45" > $OUT/hsweep.jsonl 2>&1 || exit $?
for r in 0 1; do
  timeout -k 10 400 python tools/part_scaling.py raytrace-we-gpu_amd/lib/librtx.so $V/librtx_dtail.so $V/librtx_early2.so $V/librtx_early3.so $V/librtx_tail100.so --parts 1 2 4 8 >> $OUT/parts_ab.jsonl 2>&1 || exit $?
done
echo "session V ok"
