#!/bin/bash
# Round-4 session W (final tree): GPU tests, smoke, bench, kernel stats (C2 and an R = 8 share),
# part scaling in both RNG modes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_session.sh R6w tests smoke bench prof parts psparts
OUT=gpurun_out/R6w
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof8 -o run -- python3 tools/part_scaling.py --parts 8 > $OUT/prof8.log 2>&1
echo "prof8 rc=$?" >> $OUT/session.log
