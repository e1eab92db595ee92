#!/bin/bash
# Round-4 session N: where the C2 issue goes (section profile of the chain render) + stall counters of the
# tail (wave timeline) for the record.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6n; mkdir -p $OUT
timeout -k 10 300 python tools/section_prof.py raytrace-we-gpu_amd/lib/variants/librtx_prof.so > $OUT/sprof.jsonl 2>&1
echo "session N rc=$?"
