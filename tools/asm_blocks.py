#!/usr/bin/env python3
"""Basic blocks of one kernel in the device asm (make asm) with their
instruction mix: finds the scan loop bodies (v_pk_fma_f32-heavy blocks).

    python tools/asm_blocks.py [asm] [kernel-substring] [min_pk]
"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "raytrace-we-gpu_amd/lib/rtx_kernels.s"
want = sys.argv[2] if len(sys.argv) > 2 else "k_renderILb1ELb0ELb0E"
min_pk = int(sys.argv[3]) if len(sys.argv) > 3 else 16
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and want in l and l.endswith(want.split("E")[0] + l[l.find(want) + len(want):].split(":")[0] + ":") or (l.startswith("_Z") and want in l))
end = next(i for i in range(start, len(lines)) if "-- End function" in lines[i])
blocks, cur, name = [], [], "entry"
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        blocks.append((name, cur))
        name, cur = m.group(1), []
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    cur.append(t.split()[0])
blocks.append((name, cur))
for name, ins in blocks:
    pk = ins.count("v_pk_fma_f32")
    if pk >= min_pk:
        valu = [x for x in ins if x.startswith("v_")]
        other = {}
        for x in valu:
            if x != "v_pk_fma_f32":
                other[x] = other.get(x, 0) + 1
        print(f"{name}: {len(ins)} instrs, VALU {len(valu)} (pk_fma {pk}), "
              f"SALU/SMEM {len([x for x in ins if x.startswith('s_')])}; other VALU {other}")
