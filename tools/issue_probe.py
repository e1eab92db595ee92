#!/usr/bin/env python3
"""issue_probe.py — the VALU issue ceiling in the chip's own cycles (VERDICT
r5 item 5).

Pass 1: tools/ubench_issue under `rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU
SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES`:
per instruction class and occupancy, SIMD-cycles per wave64 VALU instruction
(4 SIMDs x CUs x GRBM_GUI_ACTIVE/8 over SQ_INSTS_VALU; GRBM_GUI_ACTIVE counts
the real clock, summed over the 8 XCDs) and the clock itself (GRBM/8 over the
kernel's duration).
Pass 2: the VALU class counters (FMA/MUL/ADD/INT32/TRANS/CVT) over the
ubench (which class a v_pk_fma_f32 counts as) and over one C2 frame of the
render (bench.py --probe): the render's mix.
Pass 3: the ubench's `mix` kernel replaying that mix (no memory, independent
chains, the render's occupancy): the cycles per VALU instruction that mix
can issue at — the ceiling the render's own rate is compared with.

    python tools/issue_probe.py [--out DIR] [--iters N]
Prints one JSON object.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UB = os.path.join(ROOT, "tools", "ubench_issue")
ISSUE = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]
CLASSES = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32",
           "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_CVT", "SQ_INSTS_SALU"]


def rocprof(counters, cmd, trace=True):
    """Per-dispatch counter rows (and durations with --kernel-trace) of cmd."""
    out = tempfile.mkdtemp(prefix="issue_")
    try:
        args = ["rocprofv3"] + (["--kernel-trace"] if trace else []) + ["--pmc"] + counters + \
               ["--output-format", "csv", "-d", out, "-o", "run", "--"] + cmd
        r = subprocess.run(args, capture_output=True, text=True, timeout=240)
        if r.returncode != 0:
            raise RuntimeError(f"rocprofv3 failed ({r.returncode}): {r.stderr[-800:]}")
        disp = {}
        for path in glob.glob(os.path.join(out, "**", "*counter_collection*.csv"), recursive=True):
            for row in csv.DictReader(open(path)):
                d = disp.setdefault(int(row["Dispatch_Id"]), {"kernel": row["Kernel_Name"]})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        for path in glob.glob(os.path.join(out, "**", "*kernel_trace*.csv"), recursive=True):
            for row in csv.DictReader(open(path)):
                i = int(row["Dispatch_Id"])
                if i in disp:
                    disp[i]["ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        return [disp[k] for k in sorted(disp)], r.stdout
    finally:
        shutil.rmtree(out, ignore_errors=True)


def ub_name(kernel):
    m = re.search(r"k_(\w+?)<(\d+)>", kernel)
    return (m.group(1), int(m.group(2))) if m else (kernel, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=4000)
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    simds = 4 * a.cus
    res = {"method": "SIMD-cycles (4 x CUs x GRBM_GUI_ACTIVE/8: the real clock) per wave64 VALU instruction; "
                     "clock = GRBM_GUI_ACTIVE/8 / kernel duration"}
    # pass 1: issue cost per class / occupancy (the second of each kernel's two launches)
    rows, _ = rocprof(ISSUE, [UB, str(a.iters)])
    last = {}
    for d in rows:
        last[ub_name(d["kernel"])] = d
    ub = []
    for (k, w), d in last.items():
        cyc = d["GRBM_GUI_ACTIVE"] / 8.0
        ub.append({"class": k, "waves_per_simd": w,
                   "cycles_per_valu": round(simds * cyc / max(1.0, d["SQ_INSTS_VALU"]), 3),
                   "salu_per_valu": round(d["SQ_INSTS_SALU"] / max(1.0, d["SQ_INSTS_VALU"]), 3),
                   "valu_busy_quad": round(4.0 * d["SQ_ACTIVE_INST_VALU"] / (simds * cyc), 4),
                   "clock_GHz": round(cyc / d["ns"], 3) if d.get("ns") else None})
    res["ubench"] = ub
    # pass 2: class counters, ubench and one C2 render frame
    rows, _ = rocprof(CLASSES, [UB, str(a.iters)], trace=False)
    cls = {}
    for d in rows:
        cls[ub_name(d["kernel"])] = {c: d.get(c, 0.0) for c in CLASSES}
    res["ubench_classes"] = {f"{k}@{w}": {c.replace("SQ_INSTS_", ""): round(v / max(1.0, x["SQ_INSTS_VALU"]), 4)
                                          for c, v in x.items()} for (k, w), x in cls.items()}
    rows, _ = rocprof(CLASSES, [sys.executable, os.path.join(ROOT, "bench.py"), "--probe"], trace=False)
    tot = {c: 0.0 for c in CLASSES}
    for d in rows:
        if "k_render<true, false, false>" in d["kernel"]:
            for c in CLASSES:
                tot[c] += d.get(c, 0.0)
    v = max(1.0, tot["SQ_INSTS_VALU"])
    res["render_classes"] = {c.replace("SQ_INSTS_", ""): round(tot[c] / v, 4) for c in CLASSES}
    res["render_classes"]["SQ_INSTS_VALU"] = tot["SQ_INSTS_VALU"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
