#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X path tracer on BASELINE.json's config.

Workload (BASELINE.json configs[1]): 1920x1080, RTIOW final
random-sphere scene (WorldDef::random_world with grid -11..11 = 486
spheres), spp 100, depth 50, the reference's chain RNG. One step = one
frame: every rank renders its interleaved row tiles (rtx_render_rows), the
ranks gather to rank 0 over RCCL (torch.distributed "nccl" = RCCL) and
rank 0 de-interleaves into the image. Scene/camera are resident on the
device before timing. Launch:

    python bench.py [--gpus 1] [--steps 10] [--warmup 2]
    python bench.py --gpus N ...        (N > 1: launches its N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

`--gpus N` outside torch.distributed.run (WORLD_SIZE unset) starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child
process and exits with its code; the parent makes no GPU call (it counts the
visible devices in a child of its own). `--spawn` does the same for N = 1
(the one-rank RCCL path).

Rank 0 prints ONE JSON line. `value` = pixels*spp*steps / max-over-ranks
wall time of the timed steps: the frame is split across ranks, so the work
per step is fixed as N grows ("scaling": "strong"). An N > 1
line also carries `dist` (the process group's backend and size as
torch.distributed saw them, the RCCL version, each rank's device and its
per-step render / gather / de-interleave times from HIP events on the
step's stream) and `parity` (rows of the gathered frame, two from every
rank's share, bit for bit against the fp32 oracle after timing).
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
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA peak (spec)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FLOP_PER_TEST = 20        # the reference algorithm's FLOP per ray-sphere test (effective rate)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=100)
    p.add_argument("--depth", type=int, default=50)
    p.add_argument("--grid", type=int, default=11, help="random_world grid half extent (11 -> 486 spheres)")
    p.add_argument("--max-spheres", type=int, default=0)
    p.add_argument("--tile-rows", type=int, default=5)
    p.add_argument("--rng", choices=["chain", "per-sample"], default="chain")
    p.add_argument("--scan", choices=["auto", "linear"], default="auto",
                   help="hit_world's candidate search (rtx_set_scan_mode): auto = layer grid / culled scan, "
                        "linear = every block of every segment (the reference's Hittable_list traversal)")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--pmc", choices=["auto", "off"], default="auto",
                   help="rocprofv3 PMC child passes for HBM traffic (rank 0, N=1)")
    p.add_argument("--per-sample", type=int, default=1,
                   help="also time the per-sample-RNG kernel on the same frame (N=1, chain runs only)")
    p.add_argument("--parts", default="2,4,8",
                   help="N=1: time every part of these R-way row-tile splits on this device ('' = skip)")
    p.add_argument("--gather", action="store_true",
                   help="N=1: run the N-rank path anyway (process group over RCCL, row tiles, one gather, "
                        "de-interleave): a one-GPU rehearsal of it")
    p.add_argument("--spawn", action="store_true",
                   help="launch the ranks through torch.distributed.run as a child process even for N=1 "
                        "(N>1 outside torch.distributed.run always does)")
    p.add_argument("--dump-image", default="", help=argparse.SUPPRESS)  # rank 0 saves the last frame (.npy)
    p.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--probe-parts", type=int, default=0, help=argparse.SUPPRESS)  # --probe: an R-way split
    p.add_argument("--probe-frames", type=int, default=1, help=argparse.SUPPRESS)  # --probe: whole frames
    p.add_argument("--probe-scan", type=int, default=0, help=argparse.SUPPRESS)  # --probe: scan-rate reps
    return p.parse_args()


def scene_and_frame(args):
    import rtx
    cap = args.max_spheres or None
    world = rtx.random_world(args.grid, capacity=cap, depth=args.depth, spp=args.spp)
    frame = rtx.camera_look_at(args.width, args.height, aspect=args.width / args.height)
    frame.rng_mode = 1 if args.rng == "per-sample" else 0
    return world, frame


def probe(args):
    """One frame through the C-ABI, no torch: the process rocprofv3 wraps."""
    import rtx
    world, frame = scene_and_frame(args)
    with rtx.Context(0) as ctx:
        ctx.set_scan_mode(args.scan)
        ctx.upload_world(world)
        ctx.set_frame(frame)
        if args.probe_scan:  # hit_world alone at the render's occupancy (rtx_debug_scan_rate)
            ctx.debug_scan_rate(args.probe_scan)
        elif args.probe_parts > 1:  # every part of an R-way row-tile split, once each
            R, T = args.probe_parts, args.tile_rows
            buf = ctx.alloc((rtx.part_rows(args.height, T, 0, R), args.width, 4))
            for p in range(R):
                ctx.render_rows(T, p, R, buf.ptr)
            ctx.sync()
            buf.free()
        else:
            for _ in range(max(1, args.probe_frames)):
                ctx.render()
            ctx.sync()


def kernel_class(name):
    """The role of one dispatch of an rtx_render_rows launch (rocprof
    Kernel_Name), or None for the HIP runtime's own fills and copies."""
    m = re.search(r"k_render<(true|false), (true|false), (true|false)(?:, (?:true|false))*>", name)
    if m:
        if m.group(2) == "true":
            return "prepass"
        return "render" if m.group(1) == "true" else "render_grid"
    for k in ("k_render_ps", "k_trace", "k_cost_hist", "k_cost_scatter", "k_heavy_split", "k_unpermute",
              "k_render_trivial", "k_deinterleave", "k_debug_scan_rate"):
        if k in name:
            return k
    return None


def _pmc_pass(args, counters, tag, rng=None, extra=()):
    """One rocprofv3 --pmc pass over the --probe child (one frame through
    the C-ABI). Returns {counter: summed value over the launch's rtx
    dispatches, "by_kernel": {role: {counter: value}}}, or raises
    RuntimeError."""
    exe = shutil.which("rocprofv3")
    if not exe:
        raise RuntimeError("rocprofv3 not found")
    base = [sys.executable, os.path.abspath(__file__), "--probe", "--width", str(args.width),
            "--height", str(args.height), "--spp", str(args.spp), "--depth", str(args.depth),
            "--grid", str(args.grid), "--max-spheres", str(args.max_spheres), "--rng", rng or args.rng,
            "--scan", args.scan] + list(extra)
    out = tempfile.mkdtemp(prefix=f"rtx_pmc_{tag}_")
    cmd = [exe, "--pmc"] + list(counters) + ["--output-format", "csv", "-d", out, "-o", "pmc", "--"] + base
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=240)
        vals = {c: 0.0 for c in counters}
        by = {}
        seen = set()
        for path in glob.glob(os.path.join(out, "**", "*counter_collection*.csv"), recursive=True):
            for row in csv.DictReader(open(path)):
                role = kernel_class(row.get("Kernel_Name", ""))
                c = row.get("Counter_Name")
                if role is None or c not in vals:
                    continue
                v = float(row["Counter_Value"])
                vals[c] += v
                by.setdefault(role, {k: 0.0 for k in counters})[c] += v
                if role.startswith("render") or role in ("k_render_ps", "k_debug_scan_rate"):
                    seen.add(c)
        if seen != set(counters):
            raise RuntimeError(f"no render rows for {sorted(set(counters) - seen)}")
        vals["by_kernel"] = by
        return vals
    except subprocess.SubprocessError as e:
        raise RuntimeError(f"rocprofv3 {tag} failed: {type(e).__name__}") from e
    finally:
        shutil.rmtree(out, ignore_errors=True)


def pmc_traffic(args, rng=None):
    """HBM bytes per render launch from rocprofv3 PMC counters, per
    MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in separate passes
    (TCC slots), KB units, FETCH_SIZE x2 on gfx950 for wide coalesced reads.
    Summed over every dispatch of the launch, and split per dispatch role
    (pre-pass, sort, render, k_trace). Returns (bytes, details) or (None,
    reason)."""
    try:
        f = _pmc_pass(args, ["FETCH_SIZE"], "fetch", rng)
        w = _pmc_pass(args, ["WRITE_SIZE"], "write", rng)
    except RuntimeError as e:
        return None, str(e)
    fetch, write = f["FETCH_SIZE"], w["WRITE_SIZE"]
    kb = 2.0 * fetch + write
    roles = sorted(set(f["by_kernel"]) | set(w["by_kernel"]))
    split = {r: {"FETCH_SIZE_KB": round(f["by_kernel"].get(r, {}).get("FETCH_SIZE", 0.0), 1),
                 "WRITE_SIZE_KB": round(w["by_kernel"].get(r, {}).get("WRITE_SIZE", 0.0), 1)} for r in roles}
    return kb * 1024.0, {"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write, "by_dispatch": split,
                         "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024, every rtx dispatch of the launch"}


SQ_COUNTERS = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU",
               "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_FLOPS_FP32_TRANS",
               "GRBM_GUI_ACTIVE"]
# where the waves' cycles go (MI355X_MICROARCH.md PMC table: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
# ~= WAVE_CYCLES, all in quad-cycles)
STALL_COUNTERS = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "GRBM_GUI_ACTIVE"]


# A wave64 fp32 VALU instruction occupies the 32-lane SIMD for 2 cycles when
# several waves issue (one wave alone: 4) — MI355X_MICROARCH.md, cycle
# constants: this is the issue rate behind the 157.3 TF fp32 peak (64 FLOP /
# cycle / SIMD with v_fma_f32). Packed fp32 (v_pk_fma_f32) does twice the
# work in twice the cycles.
VALU_ISSUE_CYCLES = 2.0


def pmc_valu(args, n_cu, launch_ms, rng=None):
    """Executed-work view of the render launch (its own --pmc passes): the FP32
    FLOPs the VALU ran, the VALU issue rate, the lanes each VALU instruction
    had, and where the waves' cycles went. SQ_ACTIVE_INST_* / SQ_WAVE_CYCLES
    count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs
    (MI355X_MICROARCH.md, cycle constants)."""
    try:
        v = _pmc_pass(args, SQ_COUNTERS, "sq", rng)
        w = _pmc_pass(args, STALL_COUNTERS, "stall", rng)
    except RuntimeError as e:
        return {"skipped": str(e)}
    v.pop("by_kernel", None)
    w.pop("by_kernel", None)
    cycles = v["GRBM_GUI_ACTIVE"] / 8.0
    simds = 4 * n_cu
    # the FLOPS counters count per wave-instruction (FMA 2, ...): x64 lanes is
    # rocprof's convention; x the measured lane utilisation counts active lanes
    lane_util = v["SQ_THREAD_CYCLES_VALU"] / (64.0 * v["SQ_ACTIVE_INST_VALU"])
    flops = 64.0 * (v["SQ_INSTS_VALU_FLOPS_FP32"] + v["SQ_INSTS_VALU_FLOPS_FP32_TRANS"])
    tflops = flops / (launch_ms * 1e-3) / 1e12
    ipc = v["SQ_INSTS_VALU"] / (simds * cycles)
    wc = w["SQ_WAVE_CYCLES"]
    return {"executed_tflops": round(tflops, 3), "executed_frac": round(tflops / FP32_PEAK_TFLOPS, 4),
            "executed_tflops_active_lanes": round(tflops * lane_util, 3),
            "executed_flop_per_launch": flops,
            "issue_frac": round(ipc * VALU_ISSUE_CYCLES, 4),
            "valu_busy": round(4.0 * v["SQ_ACTIVE_INST_VALU"] / (simds * cycles), 4),
            "valu_lane_util": round(lane_util, 4),
            "valu_insts_per_simd_cycle": round(ipc, 4),
            "flop_per_valu_inst": round(flops / 64.0 / max(1.0, v["SQ_INSTS_VALU"]), 3),
            "trans_share_of_valu_insts": round(v["SQ_INSTS_VALU_TRANS_F32"] / max(1.0, v["SQ_INSTS_VALU"]), 4),
            "salu_per_valu_inst": round(v["SQ_INSTS_SALU"] / max(1.0, v["SQ_INSTS_VALU"]), 4),
            "wave_cycles": {"resident_waves_per_simd": round(4.0 * wc / (simds * w["GRBM_GUI_ACTIVE"] / 8.0), 3),
                            "issuing": round(w["SQ_ACTIVE_INST_ANY"] / wc, 4),
                            "issuing_valu": round(w["SQ_ACTIVE_INST_VALU"] / wc, 4),
                            "issuing_salu_smem": round(w["SQ_ACTIVE_INST_SCA"] / wc, 4),
                            "issuing_lds": round(w["SQ_ACTIVE_INST_LDS"] / wc, 4),
                            "issuing_vmem": round(w["SQ_ACTIVE_INST_VMEM"] / wc, 4),
                            "stalled_on_issue": round(w["SQ_WAIT_INST_ANY"] / wc, 4),
                            "waiting_on_waitcnt": round(w["SQ_WAIT_ANY"] / wc, 4)},
            "formula": "executed = 64 * (SQ_INSTS_VALU_FLOPS_FP32 + _TRANS) / launch time (the FP32 FLOPs "
                       "the VALU ran, prefilter, exact tests and shading included; _active_lanes scales by "
                       "valu_lane_util); issue_frac = 2 * SQ_INSTS_VALU / (4*CUs * GRBM_GUI_ACTIVE/8): VALU "
                       "issue cycles at the SIMD-32's 2 cycles per wave64 instruction (the rate of the fp32 "
                       "peak) over the SIMD-cycles; valu_busy = 4*SQ_ACTIVE_INST_VALU / (4*CUs * GRBM_GUI_ACTIVE/8) "
                       "(rocprof VALUBusy, quad-cycle accounting: ~1 when every wave-cycle of VALU work is "
                       "counted at 4 cycles, can read above 1 because two waves' instructions overlap); "
                       "valu_lane_util = SQ_THREAD_CYCLES_VALU / (64*SQ_ACTIVE_INST_VALU); wave_cycles: "
                       "SQ_ACTIVE_INST_* / SQ_WAIT_INST_ANY (ready, not issued) / SQ_WAIT_ANY (s_waitcnt, "
                       "barrier) over SQ_WAVE_CYCLES (its own pass)",
            "counters": v, "stall_counters": w, "cus": n_cu}


UBENCH = os.path.join(ROOT, "tools", "ubench_issue")


def issue_ceiling(args, executed, n_cu):
    """The VALU issue ceiling at the render's occupancy,
    in the chip's own cycles: tools/ubench_issue issues independent
    v_fma_f32 (and v_pk_fma_f32, integer, transcendental) streams at 1, 2, 5
    and 8 waves per SIMD, one rocprofv3 pass gives SQ_INSTS_VALU and
    GRBM_GUI_ACTIVE per kernel; cycles per VALU instruction = 4 * CUs *
    GRBM_GUI_ACTIVE/8 / SQ_INSTS_VALU (the real clock, DVFS included). No
    instruction class of the render's mix issues faster than an independent
    v_fma_f32 stream at the same occupancy, so the fma stream at the render's
    resident waves (rounded up: the generous side) is a rate the render
    cannot beat; render_frac_of_ceiling = its cycles / the render's."""
    if not executed or "counters" not in executed:
        return {"skipped": "needs the N=1 PMC passes"}
    if not os.path.exists(UBENCH):
        return {"skipped": f"{os.path.relpath(UBENCH, ROOT)} not built (make)"}
    exe = shutil.which("rocprofv3")
    out = tempfile.mkdtemp(prefix="rtx_ubench_")
    try:
        cmd = [exe, "--pmc", "SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE", "--output-format", "csv", "-d", out,
               "-o", "ub", "--", UBENCH, "4000"]
        subprocess.run(cmd, check=True, capture_output=True, timeout=240)
        disp = {}
        for path in glob.glob(os.path.join(out, "**", "*counter_collection*.csv"), recursive=True):
            for row in csv.DictReader(open(path)):
                d = disp.setdefault(int(row["Dispatch_Id"]), {"kernel": row["Kernel_Name"]})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    except (subprocess.SubprocessError, OSError, KeyError, ValueError) as e:
        return {"skipped": f"ubench pass failed: {type(e).__name__}"}
    finally:
        shutil.rmtree(out, ignore_errors=True)
    simds = 4 * n_cu
    rates = {}
    for i in sorted(disp):  # the second launch of each kernel overwrites the first
        m = re.search(r"k_(\w+?)<(\d+)>", disp[i]["kernel"])
        if m and disp[i].get("SQ_INSTS_VALU"):
            rates[f"{m.group(1)}@{m.group(2)}"] = round(
                simds * disp[i]["GRBM_GUI_ACTIVE"] / 8.0 / disp[i]["SQ_INSTS_VALU"], 3)
    rc = executed["counters"]
    render_cpv = simds * rc["GRBM_GUI_ACTIVE"] / 8.0 / rc["SQ_INSTS_VALU"]
    occ = executed.get("wave_cycles", {}).get("resident_waves_per_simd") or 5.0
    fma = {int(k.split("@")[1]): v for k, v in rates.items() if k.startswith("fma@")}
    w = min([x for x in fma if x >= occ] or [max(fma)]) if fma else None
    ceil_cpv = fma.get(w) if w else None
    return {"probe": "tools/ubench_issue: independent VALU streams per class and occupancy, one rocprofv3 pass; "
                     "cycles per VALU instruction in the chip's own clock (GRBM_GUI_ACTIVE)",
            "cycles_per_valu_by_class": rates,
            "render_resident_waves_per_simd": occ, "ceiling_class": f"fma@{w}" if w else None,
            "ceiling_cycles_per_valu": ceil_cpv,
            "render_cycles_per_valu": round(render_cpv, 3),
            "render_frac_of_ceiling": round(ceil_cpv / render_cpv, 4) if ceil_cpv else None}


def roofline_of(executed, launch_ms, tests_per_launch):
    """The compute roofline of one launch. `frac` is the EXECUTED FP32 FLOP
    rate over the FP32 peak (PMC counters over the live launch time: <= 1 by
    construction); `issue_frac` is the VALU issue cycles (2 per wave64
    instruction on the 32-lane SIMD, the rate of that peak) over the
    SIMD-cycles (<= 1 by construction); `executed.wave_cycles` says where the
    waves' cycles go (issuing, ready but not issued, waiting on s_waitcnt).
    The reference-algorithm rate — 20 FLOP for every ray-sphere test of
    every segment — is reported
    as `effective_tflops`: an effective-work rate, not a roofline fraction
    (the prefilter executes 5-7 FLOP per test plus exact tests of the few
    flagged spheres, so it can exceed what the ALUs run)."""
    eff = FLOP_PER_TEST * tests_per_launch / (launch_ms * 1e-3) / 1e12
    r = {"bound": "fp32-valu",
         "roof": "fp32 vector ALU, 157.3 TF = 1,024 SIMD-32s x 64 FLOP/cycle x 2.4 GHz, i.e. one wave64 v_fma_f32 "
                 "per SIMD every 2 cycles (the kernel issues no MFMA)",
         "achieved": None, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": None,
         "frac_kind": "executed FP32 FLOP/s / FP32 peak",
         "issue_frac": None}
    if executed and "executed_tflops" in executed:
        r.update(achieved=executed["executed_tflops"], frac=executed["executed_frac"],
                 issue_frac=executed["issue_frac"])
    else:
        r["frac_kind"] += " (needs the N=1 PMC passes: not run here)"
    r.update(effective_tflops=round(eff, 3),
             effective_note="20 FLOP x (segments x spheres) per launch / launch time: the reference algorithm's "
                            "work rate (every sphere tested per segment), not a fraction of any roof; large "
                            "scenes skip most spheres (culled scan), so there it exceeds the peak")
    return r


def cpu_baseline(args, world, frame, gpu_image, budget_s):
    """The fp32 oracle (port of the reference path) on the host cores, on a
    bounded sample of the same frame: whole rows at full spp, spread over
    the image, until the time budget is spent. Those rows are also compared
    bit for bit with the GPU frame."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    visible = len(os.sched_getaffinity(0))
    # the box's CPU share: OMP_NUM_THREADS is set to it on the GPU box
    # (16); sched_getaffinity shows every CPU of the host there
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or visible
    threads = max(1, min(visible, share))
    H = args.height
    order = [(7 + 37 * k) % H for k in range(H)]  # 37 is coprime to 1080: every row once
    done, t0, mism = [], time.perf_counter(), 0
    while done == [] or (time.perf_counter() - t0 < budget_s and len(done) < H):
        batch = order[len(done):len(done) + threads]
        if not batch:
            break
        rows, _ = oracle.render_rows(world, frame, np.array(batch, np.uint32), nthreads=threads)
        if gpu_image is not None:
            g = gpu_image[batch]
            same = (g.view(np.uint32) == rows.view(np.uint32)) | (np.isnan(g) & np.isnan(rows))
            mism += int((~same).sum())
        done += batch
    dt = time.perf_counter() - t0
    samples = len(done) * args.width * args.spp
    # single-thread rate on a few of the same rows (report 1 thread too)
    few = [H // 8, 3 * H // 8, 5 * H // 8, 7 * H // 8]
    t1 = time.perf_counter()
    oracle.render_rows(world, frame, np.array(few, np.uint32), nthreads=1)
    dt1 = time.perf_counter() - t1
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "cores_note": f"threads used = min(CPUs in sched_getaffinity ({visible}), OMP_NUM_THREADS "
                          f"= the box's CPU share ({share}))",
            "sample": f"{len(done)} full rows (x{args.width} px, spp {args.spp}) of the same frame, "
                      f"spread over the image, fp32 oracle (oracle/rtx_oracle.c), {threads} threads, "
                      f"{dt:.1f} s",
            "single_thread": {"value": len(few) * args.width * args.spp / dt1 / 1e6, "unit": "Msamples/s",
                              "sample": f"{len(few)} rows, 1 thread, {dt1:.1f} s"},
            "host": host_cpu()}, {"rows_checked": len(done), "values_differing": mism, "bit_exact": mism == 0}


def part_scaling(ctx, args, world, frame, t1_ms, dev, parts=(2, 4, 8), frames=2, check_rows=8):
    """The 1/2/4/8-GPU split rehearsed on this one device (N = 1 only): an
    R-GPU frame gives rank p the rows rtx_render_rows(T, p, R) renders, so
    timing every part of an R-way split here gives each rank's kernel time
    and the critical path max_p t_p of the R-GPU frame (before its gather).
    efficiency = t(1) / (R * max_p t_p), t(1) = the headline's launch time.
    After timing, `check_rows` rows of each R's critical part are compared
    bit for bit with the fp32 oracle (the checker, never the timed path)."""
    import numpy as np
    import torch
    import rtx
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    W, H, T = args.width, args.height, args.tile_rows
    threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16))
    buf = torch.empty((rtx.part_rows(H, T, 0, 1), W, 4), dtype=torch.float32, device=dev)
    out = {"t1_ms": round(t1_ms, 3), "frames_per_part": frames, "tile_rows": T,
           "note": "each part of an R-way row-tile split timed on this one MI355X (HIP events around "
                   "rtx_render_rows); critical_ms = max over parts; efficiency = t1 / (R * critical)"}
    for R in parts:
        times, segs = [], []
        for p in range(R):
            ctx.render_rows(T, p, R, buf.data_ptr())  # warm (and the schedule's buffers)
            torch.cuda.synchronize()
            ctx.stats_reset()
            for _ in range(frames):
                ctx.render_rows(T, p, R, buf.data_ptr())
            torch.cuda.synchronize()
            st = ctx.stats()
            times.append(st.kernel_ms / max(1, st.launches))
            segs.append(int(st.segments // max(1, st.launches)))
        crit = max(times)
        pc = times.index(crit)
        # parity of the critical part: its last frame is not in buf any more
        # unless it was the last part timed, so render it once more
        ctx.render_rows(T, pc, R, buf.data_ptr())
        torch.cuda.synchronize()
        ids = rtx.part_row_ids(H, T, pc, R)
        local = sorted(set(int(i) for i in np.linspace(0, len(ids) - 1, check_rows)))
        got = buf[local].cpu().numpy()
        want, _ = oracle.render_rows(world, frame, ids[local], nthreads=threads)
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        out[str(R)] = {"critical_ms": round(crit, 3), "efficiency": round(t1_ms / (R * crit), 4),
                       "mean_ms": round(sum(times) / R, 3), "part_ms": [round(t, 3) for t in times],
                       "part_segments": segs,
                       "parity": {"part": pc, "rows_checked": len(local), "values_differing": int((~same).sum()),
                                  "bit_exact": bool(same.all())}}
    del buf
    return out


def per_sample_parity(world, frame, img, rows):
    """Checker for the per-sample line: a few rows of the per-sample frame
    against the fp32 oracle in the same RNG mode (bit for bit)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16))
    want, _ = oracle.render_rows(world, frame, np.array(rows, np.uint32), nthreads=threads)
    got = img[rows]
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    return {"rows_checked": len(rows), "values_differing": int((~same).sum()), "bit_exact": bool(same.all())}


def host_cpu():
    """The box's CPU: logical CPUs visible and the model name."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "model": model}


def launch_desc(n_spheres, spp, nparts, rng, scan_mode="auto"):
    """What one rtx_render_rows launch runs for this configuration
    (rtx_kernels.hip launch_render / launch_ps)."""
    if spp < 8 and rng == "chain":
        return "rtx_render_rows launch = k_render<false> (exact grid, one lane per pixel)"
    large = ((n_spheres + 7) // 8) * 8 > 1024  # kScanPfMin: the kPF kernels
    if scan_mode == "linear":
        scan = ("linear scan: every 8-sphere block of the scene for every segment, in index order "
                + ("(streamed through a per-wave LDS tile of 64 blocks), candidate lists of 24" if large
                   else "(scalar loads), resolve from the block's LDS copy of the scene"))
    else:
        scan = ("culled scan over a spatially ordered copy of the scene (bounds over 512, 64 and 8 spheres, then "
                "spheres; the coop tiers split the same hierarchy over a ray's lanes), candidate lists of 24"
                if large else "scalar-loaded scan of the flat layer's blocks the wave's slab walks mark (layer grid) "
                              "and of every other block, resolve from the block's LDS copy of the scene")
    if rng == "per-sample":
        return f"k_render_ps (one lane per pixel-sample, in-order fold per pixel; {scan.split(' (')[0]})"
    whole = nparts == 1
    if large:
        pre = ("k_render<true,true,kPF> 1-spp cost pre-pass on persistent lanes (sample 0, resumed from"
               + ("; a pixel past 24 segments stops with a saturated key and restarts in the render)" if whole
                  else ")"))
    else:
        pre = ("k_render<false,true> 2-spp exact-grid cost pre-pass (samples 0-1, resumed from"
               + ("; a pixel past 16 segments stops and restarts in the render)" if whole else ")"))
    return (f"rtx_render_rows launch = {pre} + k_cost_hist + k_heavy_split + k_cost_scatter + "
            f"k_render<true> (cost-ordered persistent lanes"
            + (" — queue in 16x16 pixel tiles, 64-slot private runs per wave —" if whole and not large else "")
            + f" at a wave priority from their projected remaining "
            f"chains, {scan}, heavy-pixel coop tiers, promotion)"
            + (" [+ k_trace on the aux stream for a row-split share]" if not large and not whole else ""))


def build_provenance(rtx):
    """The loaded library and whether it was built from this tree's sources
    (rtx_build_info's hash vs tools/src_sha.py over the same files)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from src_sha import src_sha16
    info = rtx.build_info()
    tree = src_sha16(ROOT)
    return {"lib": os.path.relpath(rtx.LIB_PATH, ROOT), "lib_src_sha16": info.get("src_sha16"),
            "tree_src_sha16": tree, "variant": info.get("variant", "product"),
            "built_from_this_tree": info.get("src_sha16") == tree and info.get("variant", "product") == "product",
            "arch": info.get("arch")}


# ---------------------------------------------------------------------------
# Rank launcher: `bench.py --gpus N` outside torch.distributed.run
# ---------------------------------------------------------------------------
def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch_command(n: int, script: str, script_args, port: int, python: str = sys.executable):
    """The child command that runs `script` as n ranks of one node:
    torch.distributed.run, rendezvous on 127.0.0.1 (the container hostname
    may not resolve)."""
    return [python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", script] + list(script_args)


def rank_launch_env(base=None) -> dict:
    """The ranks' environment: the caller's, with dmabuf IPC kept (the host
    driver supports only that; RCCL fails without it) and a marker so a rank
    never launches again."""
    env = dict(os.environ if base is None else base)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    env["RTX_BENCH_RANKS_LAUNCHED"] = "1"
    return env


def visible_gpus(timeout: float = 300.0) -> int:
    """HIP devices visible to a fresh process, counted in a child so this one
    never touches the GPU (it is about to start the ranks)."""
    code = "import torch; print(torch.cuda.device_count())"
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)
        return int(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError):
        return 0


def launch_ranks(n: int, script: str, script_args, timeout=None) -> int:
    """Run `script` as n ranks (torch.distributed.run in a child process) and
    return its exit code; the ranks' stdout and stderr are this process's."""
    cmd = rank_launch_command(n, script, script_args, free_port())
    try:
        return subprocess.run(cmd, env=rank_launch_env(), timeout=timeout).returncode
    except subprocess.TimeoutExpired:
        return 124


def spawn_main(args, argv) -> int:
    """`bench.py --gpus N` (N > 1, or --spawn) outside torch.distributed.run:
    start the N ranks as a fresh child and exit with its code. Fewer than N
    visible devices is an error, not a smaller run."""
    n = max(1, args.gpus)
    have = visible_gpus()
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} visible HIP devices, found {have} "
              f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', 'unset')})", file=sys.stderr)
        return 3
    rest = [a for a in argv if a != "--spawn"]
    if n == 1 and "--gather" not in rest:
        rest.append("--gather")  # one rank still runs the process group and the RCCL gather
    return launch_ranks(n, os.path.abspath(__file__), rest)


def parity_rows(H, T, R, per_part=2):
    """`per_part` rows from every rank's share of an R-way row-tile split
    (its first row, then evenly spaced), ascending."""
    import numpy as np
    import rtx
    rows = []
    for p in range(R):
        ids = rtx.part_row_ids(H, T, p, R)
        rows += [int(ids[int(k)]) for k in np.linspace(0, len(ids) - 1, per_part + 1)[:-1]]
    return sorted(set(rows))


def gathered_parity(world, frame, image, H, T, R, per_part=2):
    """Rows of the gathered frame against the fp32 oracle (bit for bit):
    `per_part` rows from every rank's share, so every rank's rows and the
    de-interleave are checked."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    rows = parity_rows(H, T, R, per_part)
    threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16))
    want, _ = oracle.render_rows(world, frame, np.array(rows, np.uint32), nthreads=threads)
    got = image[rows]
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    return {"rows": rows, "rows_checked": len(rows), "ranks_covered": R, "values_differing": int((~same).sum()),
            "bit_exact": bool(same.all()), "checker": "fp32 oracle (oracle/rtx_oracle.c), after timing"}


def main():
    args = parse()
    if args.probe:
        probe(args)
        return
    if "WORLD_SIZE" not in os.environ and not os.environ.get("RTX_BENCH_RANKS_LAUNCHED") \
            and (args.gpus > 1 or args.spawn):
        sys.exit(spawn_main(args, sys.argv[1:]))
    import numpy as np
    import torch
    import torch.distributed as dist
    import rtx

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        if world_size == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1: WORLD_SIZE is 1 in a launched rank")
        args.gpus = world_size
    torch.cuda.set_device(local_rank)
    collective = world_size > 1 or args.gather
    if collective:
        if world_size == 1:  # --gather outside torch.distributed.run: a one-rank group
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    world, frame = scene_and_frame(args)
    W, H, T, R = args.width, args.height, args.tile_rows, world_size
    # One stream for everything of a step: the render (librtx), torch's
    # buffer fills, the RCCL gather (it waits on the current stream) and the
    # de-interleave all order on it.
    stream = torch.cuda.Stream(device=local_rank)
    torch.cuda.set_stream(stream)
    ctx = rtx.Context(local_rank, stream=stream.cuda_stream)
    ctx.set_scan_mode(args.scan)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    dev = torch.device("cuda", local_rank)
    if not collective:
        image = torch.empty((H, W, 4), dtype=torch.float32, device=dev)

        def step():
            ctx.render_rows(1, 0, 1, image.data_ptr())
    else:
        from rtx.dist import FrameGather
        fg = FrameGather(W, H, T, rank, R, device=dev, collective=True,
                         render_part=lambda send, part, nparts: ctx.render_rows(T, part, nparts, send.data_ptr()),
                         deinterleave=lambda g, img: ctx.deinterleave(g.data_ptr(), W, H, T, R, img.data_ptr()))
        image = fg.image
        # per-step phase times of this rank: HIP events on the step's stream
        # (the gather's completion is ordered on it: torch waits the RCCL
        # stream into the current one), recorded in the timed steps only
        phase_events, recording = [], [False]

        def mark(name):
            if recording[0]:
                if name == "start":
                    phase_events.append({})
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                phase_events[-1][name] = ev
        fg.mark = mark

        def step():
            fg.step()

    def barrier():
        if collective:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.stats_reset()
    barrier()
    if collective:
        recording[0] = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if collective:
        recording[0] = False
    barrier()
    elapsed_local = elapsed
    if collective:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = ctx.stats()
    dist_info = None
    if collective:
        def phase_ms(a, b):
            v = [e[a].elapsed_time(e[b]) for e in phase_events if a in e and b in e]
            return round(sum(v) / len(v), 4) if v else None
        props = torch.cuda.get_device_properties(local_rank)
        mine = {"rank": rank, "local_rank": local_rank, "device": props.name,
                "pci_bus_id": getattr(props, "pci_bus_id", None), "rows": fg.rows,
                "render_ms": phase_ms("start", "rendered"), "gather_ms": phase_ms("rendered", "gathered"),
                "deinterleave_ms": phase_ms("gathered", "done"), "step_ms": phase_ms("start", "done"),
                "wall_ms_per_step": round(elapsed_local / args.steps * 1e3, 4),
                "kernel_ms": round(st.kernel_ms / max(1, st.launches), 4),
                "segments_per_launch": int(st.segments // max(1, st.launches))}
        per_rank = [None] * world_size
        dist.all_gather_object(per_rank, mine)
        nccl_v = torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else None
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "rccl_version": ".".join(str(x) for x in nccl_v) if isinstance(nccl_v, tuple) else nccl_v,
                     "launcher": "bench.py self-launch (torch.distributed.run child)"
                                 if os.environ.get("RTX_BENCH_RANKS_LAUNCHED") else
                                 ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "direct"),
                     "per_rank": per_rank,
                     "note": "render = rtx_render_rows into the rank's send buffer; gather = one RCCL gather to "
                             "rank 0 (torch.distributed 'nccl'); deinterleave = rtx_deinterleave_rows on rank 0; "
                             "each the mean over the timed steps of HIP events on the step's stream"}
    if args.dump_image and rank == 0:
        np.save(args.dump_image, image.cpu().numpy())

    if rank == 0:
        samples = W * H * args.spp * args.steps
        value = samples / elapsed / 1e6
        launch_ms = st.kernel_ms / max(1, st.launches)
        tests_per_launch = st.sphere_tests / max(1, st.launches)
        rows0 = rtx.part_rows(H, T, 0, R) if R > 1 else H
        alg_bytes = rows0 * W * 16 + world.count * 32  # framebuffer + scene
        n_cu = torch.cuda.get_device_properties(local_rank).multi_processor_count
        traffic, pmc_note, executed = (None, "skipped (PMC passes run at N=1 with --pmc auto)", None)
        ceiling = None
        if args.pmc == "auto" and R == 1:
            traffic, pmc_note = pmc_traffic(args)
            executed = pmc_valu(args, n_cu, launch_ms)
            ceiling = issue_ceiling(args, executed, n_cu)
        host_img = image.cpu().numpy()
        cpu, parity = (None, None)
        if R == 1 and args.cpu_seconds > 0:
            cpu, parity = cpu_baseline(args, world, frame, host_img, args.cpu_seconds)
        if collective and parity is None:  # the gathered frame: rows of every rank's share
            parity = gathered_parity(world, frame, host_img, H, T, R)
        # the 1/2/4/8-GPU split rehearsed on this device (BASELINE.json metric:
        # "1/2/4/8-GPU scaling"); the real N-GPU runs are the driver's
        parts = None
        if R == 1 and args.parts:
            parts = part_scaling(ctx, args, world, frame, launch_ms, dev,
                                 parts=[int(x) for x in args.parts.split(",") if x])
        # The north star's kernel shape — one lane per (pixel, sample) — on the
        # same frame with per-(pixel, sample) seeds (rtx_frame.rng_mode 1,
        # DESIGN.md §3a): reported beside the headline, which stays the
        # reference's chain RNG. N = 1 only.
        per_sample = None
        if R == 1 and args.rng == "chain" and args.per_sample:
            frame.rng_mode = 1
            ctx.set_frame(frame)
            ctx.render_rows(1, 0, 1, image.data_ptr())
            torch.cuda.synchronize()
            ctx.stats_reset()
            n_ps = max(1, min(args.steps, 5))
            t_ps = time.perf_counter()
            for _ in range(n_ps):
                ctx.render_rows(1, 0, 1, image.data_ptr())
            torch.cuda.synchronize()
            t_ps = (time.perf_counter() - t_ps) / n_ps
            st_ps = ctx.stats()
            ps_ms = st_ps.kernel_ms / max(1, st_ps.launches)
            ps_exec = pmc_valu(args, n_cu, ps_ms, rng="per-sample") if args.pmc == "auto" else None
            ps_traffic, ps_pmc = pmc_traffic(args, rng="per-sample") if args.pmc == "auto" else (None, "skipped")
            per_sample = {"value": round(W * H * args.spp / t_ps / 1e6, 3), "unit": "Msamples/s",
                          "ms_per_step": round(t_ps * 1e3, 3), "steps": n_ps, "kernel_ms": round(ps_ms, 4),
                          "roofline": roofline_of(ps_exec, ps_ms, st_ps.sphere_tests / max(1, st_ps.launches)),
                          "executed": ps_exec,
                          "traffic": None if ps_traffic is None else round(ps_traffic), "pmc": ps_pmc,
                          "measured_hbm_GBs": None if ps_traffic is None else round(ps_traffic / (ps_ms * 1e-3) / 1e9, 3),
                          "kernel": launch_desc(world.count, args.spp, R, "per-sample", args.scan)}
            if args.cpu_seconds > 0:
                rows_ps = [int(r) for r in np.linspace(5, H - 6, 16)]  # 16 rows spread over the image
                per_sample["parity"] = per_sample_parity(world, frame, image.cpu().numpy(), rows_ps)
            frame.rng_mode = 0
            ctx.set_frame(frame)
        roof = roofline_of(executed, launch_ms, tests_per_launch)
        roof.update(traffic=None if traffic is None else round(traffic),
                    kernel=launch_desc(world.count, args.spp, R, args.rng, args.scan), kernel_ms=round(launch_ms, 4),
                    sphere_tests_per_launch=tests_per_launch,
                    segments_per_sample=round(st.segments / max(1, st.samples), 4),
                    pmc=pmc_note, executed=executed, issue_ceiling=ceiling)
        line = {
            "metric": "Msamples/sec (pixels x spp) at 1920x1080 spp=100 depth=50",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": R,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic RTIOW random_world scene, MSVC-rand LCG)",
            "config": {"workload": f"RTIOW final scene {W}x{H}, spp {args.spp}, depth {args.depth}, "
                                   f"{world.count} spheres, {args.rng} RNG"
                                   + (", linear scan" if args.scan == "linear" else ""),
                       "width": W, "height": H, "spp": args.spp, "depth": args.depth,
                       "spheres": world.count, "rng": args.rng, "scan": args.scan, "tile_rows": T,
                       "parallelism": f"row-tiles x{R}" + (" + RCCL gather" if collective else "")},
            "roofline": roof,
            "roofline_hbm": {"bound": "hbm", "achieved": round(alg_bytes / (launch_ms * 1e-3) / 1e9, 3),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(alg_bytes / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 7),
                             "achieved_kind": "algorithmic bytes (framebuffer + scene) / launch time",
                             "algorithmic_bytes_per_launch": alg_bytes,
                             "traffic": None if traffic is None else round(traffic),
                             "measured": None if traffic is None else round(traffic / (launch_ms * 1e-3) / 1e9, 3),
                             "measured_frac": None if traffic is None
                             else round(traffic / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                             "measured_kind": "rocprofv3 PMC traffic per launch / launch time"},
            "part_scaling": parts,
            "dist": dist_info,
            "cpu_baseline": cpu,
            "parity": parity,
            "per_sample_rng": per_sample,
            "build": build_provenance(rtx),
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if collective:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
