set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
L=raytrace-we-gpu_amd/lib/variants/librtx_ptime.so
timeout -k 10 200 python tools/pixel_timeline.py $L --parts 1 --set "a1=1.5,trL=0.03" > $O/ptime_r1_a15.log 2>&1 || exit $?
timeout -k 10 200 python tools/pixel_timeline.py $L --parts 1 --set "a1=1.3,trL=0.06" > $O/ptime_r1_a13.log 2>&1 || exit $?
timeout -k 10 300 python tools/heavy_sweep.py --parts 1 --rounds 2 --set "trL=0" --set "a1=1.5,trL=0.03" --set "a1=1.5,trL=0.03,p1=1" --set "a1=1.4,trL=0.04" --set "a1=1.3,trL=0.06,p1=2" --set "a1=1.2,trL=0.1" > $O/sweep_r1.log 2>&1 || exit $?
