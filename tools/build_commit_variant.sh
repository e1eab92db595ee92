#!/bin/bash
# Build librtx from another commit's sources as an A/B variant:
#   tools/build_commit_variant.sh <commit> <name> [extra hipcc flags]
# -> raytrace-we-gpu_amd/lib/variants/librtx_<name>.so (variant_bench.py loads it by name).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$1; N=$2; shift 2
T=$(mktemp -d)
git -C "$ROOT" archive "$C" raytrace-we-gpu_amd/csrc include | tar -x -C "$T"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -ffp-contract=off -Wno-unused-function $*"
pids=()
for s in rtx_kernels.hip rtx_api.hip rtx_host.cpp; do
  /opt/rocm/bin/hipcc $F -DRTX_VARIANT="\"commit-$C\"" -c "$T/raytrace-we-gpu_amd/csrc/$s" -o "$T/$s.o" &
  pids+=($!)
done
# a bare `wait` returns 0 even when a compile failed: check each job
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed" >&2; rm -rf "$T"; exit 1; }; done
mkdir -p "$ROOT/raytrace-we-gpu_amd/lib/variants"
/opt/rocm/bin/hipcc $F -shared -o "$ROOT/raytrace-we-gpu_amd/lib/variants/librtx_$N.so" "$T"/*.o
rm -rf "$T"
echo "built librtx_$N.so from $C"
