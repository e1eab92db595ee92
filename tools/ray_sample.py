#!/usr/bin/env python3
"""Sample the rays of lane-mode wave iterations (diagnostic).

Needs the `rays` variant (Makefile: -DRTX_DIAG_RAYS=4099): every 4099th
lane-mode iteration of each wave appends its 64 lanes' (origin, direction,
live, queue slot) to the wave_times buffer (rtx_diag.h Diag::rays). Writes
the records as an .npz for offline analysis of the scan's per-block pass
rates (tools/block_cull_sim.py).

    python tools/ray_sample.py OUT.npz [lib]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402

out = sys.argv[1]
lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "raytrace-we-gpu_amd/lib/variants/librtx_rays.so")
grid = int(os.environ.get("RTX_RAYS_GRID", "11"))
world = rtx.random_world(grid, capacity=int(os.environ.get("RTX_RAYS_CAP", "0")) or None, depth=50,
                         spp=int(os.environ.get("RTX_RAYS_SPP", "100")))
frame = rtx.camera_look_at(1920, 1080, aspect=1920 / 1080)
c = rtx.Context(0, lib=rtx.load_library(lib))
c.upload_world(world)
c.set_frame(frame)
MAXREC = 6000
cap = 32 + 128 * MAXREC  # pairs: 2 * cap words >= 64 + 256 * MAXREC
c.arm_wave_times(cap)
c.render()
c.sync()
v = c.wave_times(cap).reshape(-1)
nrec = int(v[0])
keep = min(nrec, MAXREC)
rec = v[64:64 + 256 * keep].reshape(keep, 64, 4)
lo = (rec & 0xffffffff).astype(np.uint32).view(np.float32)
hi = (rec >> 32).astype(np.uint32).view(np.float32)
o = np.stack([lo[..., 0], hi[..., 0], lo[..., 1]], -1)
d = np.stack([hi[..., 1], lo[..., 2], hi[..., 2]], -1)
live = (rec[..., 3] & 1).astype(bool)
slot = (rec[..., 3] >> 32).astype(np.uint32)
np.savez_compressed(out, o=o, d=d, live=live, slot=slot, spheres=world.spheres, grid=grid)
print({"records": nrec, "kept": keep, "live_frac": float(live.mean()), "out": out})
