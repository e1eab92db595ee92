#!/usr/bin/env python3
"""Per-pixel segment counts of the C2 frame at several sample counts
(rtx_debug_pixel_cost with spp = 1, 2, 4, 8 and the full 100), saved as one
compressed .npz, so that cost keys (the scheduling pre-pass's estimate of a
pixel's chain) can be compared offline with the chains they predict. With the
reference's chain RNG the first k samples of a pixel are the same whatever the
spp, so the spp-k map is what a k-spp pre-pass sees.

    python tools/cost_maps.py OUT.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import numpy as np  # noqa: E402
import rtx  # noqa: E402

W, H = 1920, 1080
world = rtx.random_world(11, depth=50, spp=100)
frame = rtx.camera_look_at(W, H, aspect=W / H)
ctx = rtx.Context(0)
ctx.upload_world(world)
ctx.set_frame(frame)
maps = {f"spp{k}": ctx.debug_pixel_cost(k).astype(np.uint16) for k in (1, 2, 4, 8)}
maps["spp100"] = ctx.debug_pixel_cost(0).astype(np.uint16)
np.savez_compressed(sys.argv[1], **maps)
print({k: int(v.astype(np.int64).sum()) for k, v in maps.items()})
ctx.close()
