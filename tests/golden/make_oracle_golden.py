#!/usr/bin/env python3
"""Write tests/golden/c1_oracle_rows.npz: rows of the C1 frame (400x225,
test_world, Camera.h camera, spp 20, depth 12) rendered by the fp32 oracle.

This is a regression pin of OUR restatement (the reference's GPU shader
cannot run here — D3D11/HLSL — so no reference image exists); the geometry
underneath is pinned to the reference by make_golden.py's vectors.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "raytrace-we-gpu_amd")]
import oracle as orc  # noqa: E402
import rtx  # noqa: E402

world = rtx.test_world(depth=12, spp=20)
frame = rtx.camera_simple(400, 225)
rows = np.arange(0, 225, 25).astype(np.uint32)
img, segs = orc.render_rows(world, frame, rows, nthreads=8)
np.savez_compressed(os.path.join(HERE, "c1_oracle_rows.npz"), rows=rows, pixels=img)
print("wrote c1_oracle_rows.npz", img.shape, "segments", segs)
