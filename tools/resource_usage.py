#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of rtx_kernels.hip for
gfx950 (the compiler's kernel-resource-usage remarks), so a kernel change can
be checked for new spills before it goes to the GPU.

    python tools/resource_usage.py [-DRTX_...=... ...]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
SRC = f"{ROOT}/raytrace-we-gpu_amd/csrc/rtx_kernels.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-Wno-unused-function", "--offload-device-only", "-c", SRC, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill",
        "VGPRs Spill", "LDS Size [bytes/block]"]
short = ["vgpr", "agpr", "sgpr", "scratch", "occ", "s_spill", "v_spill", "lds"]
print(f"{'kernel':44s} " + " ".join(f"{s:>7s}" for s in short))
for r in rows:
    n = r["name"].replace("_ZN3rtx12_GLOBAL__N_1", "")
    print(f"{n[:44]:44s} " + " ".join(f"{r.get(k, '-'):>7s}" for k in keys))
