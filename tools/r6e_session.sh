set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/session.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python tools/heavy_sweep.py --parts 8 4 --rounds 2 --set "coop=8" --set "coop=16" --set "coop=32" --set "coop=64" > $O/sweep_coop.log 2>&1 || exit $?
timeout -k 10 300 python tools/heavy_sweep.py --parts 1 --rounds 2 --set "a1=1.7" --set "a1=1.5" --set "a1=1.4" --set "a1=1.3" --set "coop=32" > $O/sweep_r1.log 2>&1 || exit $?
