#!/bin/bash
# The one GPU-box session runner: every GPU step under its own timeout; a
# crash, abort, or timeout (exit >= 124 or signal) ends the script there.
# Test failures (exit 1/2: pytest failures, Python exceptions) do not stop
# the later measurement steps. Steps are named on the command line and
# parameterised through environment variables (below), so a session is one
# line, e.g.
#   tools/gpu_session.sh R7a tests smoke bench prof prof8 c5b
#   PTLIB=ptime PTPARTS="4 8" HSETS='--sets "default;pb1=0"' tools/gpu_session.sh R7b ptime hsweep
# Usage: tools/gpu_session.sh TAG [steps...]   (default: ubench tests smoke bench prof)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${*:-ubench tests smoke bench prof}
fatal() { echo "STOP: step $1 exited $2" | tee -a "$OUT/session.log"; exit "$2"; }
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name: $*" >> "$OUT/session.log"
    local t0=$(date +%s)
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/session.log"
    # >= 124: timeout (124/137) or killed by a signal (134 abort, 139 segv): stop.
    if [ $rc -ge 124 ]; then fatal "$name" $rc; fi
    return 0
}
for s in $STEPS; do
  case $s in
    ubench) run ubench 120 ./tools/ubench_valu ;;
    issue)  run issue 600 python tools/issue_probe.py ;;
    tests)  run tests 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps 10 --warmup 2 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
                python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --pmc off --parts '' --per-sample 0 ;;
    prof8)  run prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof8" -o run -- \
                python3 bench.py --probe --probe-parts 8 ;;
    c5prof) run c5prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5prof" -o run -- \
                python3 bench.py --probe --spp 16 --grid 159 --max-spheres 100000 --probe-frames 2 ;;
    psprof) run psprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/psprof" -o run -- \
                python3 bench.py --probe --rng per-sample --probe-frames 3 ;;
    gtest)  run gtest 600 python -u -m pytest ${GTESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 \
                --timeout-method thread ;;
    c3b)    run c3b 900 python bench.py --width 3840 --height 2160 --spp 1024 --steps 2 --warmup 1 --cpu-seconds 10 --parts '' ;;
    c5b)    run c5b 900 python bench.py --spp 16 --grid 159 --max-spheres 100000 --steps 3 --warmup 1 --cpu-seconds 10 --parts '' --per-sample ${C5PS:-0} ;;
    c3ps)   run c3ps 900 python bench.py --rng per-sample --width 3840 --height 2160 --spp 1024 --steps 2 --warmup 1 --cpu-seconds 10 --parts '' ;;
    c5lin)  run c5lin 900 python bench.py --spp 16 --grid 159 --max-spheres 100000 --scan linear --steps 1 --warmup 1 --cpu-seconds 10 --parts '' --per-sample 0 ;;
    c2lin)  run c2lin 600 python bench.py --scan linear --steps 5 --warmup 1 --cpu-seconds 10 --parts '' --per-sample 0 ;;
    c5ps)   run c5ps 900 python bench.py --rng per-sample --spp 16 --grid 159 --max-spheres 100000 --steps 3 --warmup 1 --cpu-seconds 10 --parts '' ;;
    variants) run variants 900 python tools/variant_bench.py --rounds ${VROUNDS:-5} --frames 2 ${VARGS:-} ${VNAMES:-} ;;
    ctrlist) run ctrlist 120 rocprofv3 -L ;;
    c2ps)   run c2ps 600 python bench.py --rng per-sample --steps 5 --warmup 1 --cpu-seconds 10 --parts '' ;;
    timeline) run timeline 300 python tools/wave_timeline.py ;;
    vtimeline) for v in ${VTL:-blk64 lpt lpt_blk64}; do
              run timeline_$v 300 python tools/wave_timeline.py raytrace-we-gpu_amd/lib/variants/librtx_$v.so; done ;;
    sprof)  run sprof 300 python tools/section_prof.py raytrace-we-gpu_amd/lib/variants/librtx_prof.so ;;
    parts)  run parts 600 python tools/part_scaling.py ${PARGS:-} ${PLIBS:-} ;;
    hsweep) eval run hsweep 900 python tools/heavy_sweep.py --parts ${HPARTS:-8} --rounds ${HROUNDS:-2} ${HSETS:-} ;;
    psparts) run psparts 600 python tools/part_scaling.py --rng per-sample ;;
    cprof)  run cprof 300 python tools/coop_prof.py raytrace-we-gpu_amd/lib/variants/librtx_cprof.so ;;
    ptime)  run ptime 600 python tools/pixel_timeline.py raytrace-we-gpu_amd/lib/variants/librtx_${PTLIB:-ptime}.so \
                --parts ${PTPARTS:-1 2 8} ;;
    cost)   run cost 600 python tools/cost_analysis.py --out "$OUT/cost.npz" ;;
    c5)     run c5 900 python tools/variant_bench.py --rounds 2 --frames 1 --spp 16 --grid 159 --max-spheres 100000 ${C5V:-} ;;
    diag)   run diag 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
                SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/diag" -o run -- \
                python3 bench.py --probe ;;
    diag2)  run diag2 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM \
                SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/diag2" -o run -- \
                python3 bench.py --probe ;;
    vdiag)  V=raytrace-we-gpu_amd/lib/variants/librtx_${VDIAG:-best}.so
            RTX_LIB=$V run vdiag 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES \
                SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/vdiag" -o run -- \
                python3 bench.py --probe
            RTX_LIB=$V run vdiag2 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
                SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d "$OUT/vdiag2" -o run -- \
                python3 bench.py --probe ;;
    vinsts) for v in ${VNAMES:-best}; do  # VALU/SALU instruction counts per variant (deterministic A/B)
              RTX_LIB=raytrace-we-gpu_amd/lib/variants/librtx_$v.so run vinsts_$v 300 rocprofv3 --pmc SQ_INSTS_VALU \
                  SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$OUT/vinsts_$v" -o run -- \
                  python3 bench.py --probe ${VARGS:-}
              python tools/pmc_sum.py "$OUT/vinsts_$v" "$v" >> "$OUT/vinsts.jsonl"; done ;;
    pmc)    for c in FETCH_SIZE WRITE_SIZE; do
              run pmc_$c 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
                  python3 bench.py --probe ; done ;;
  esac
done
echo "session done" >> "$OUT/session.log"
