"""Child process of test_gpu_parity.py::test_frame_gather_on_torch_default_stream.

torch must own the process's HIP runtime before librtx loads,
so this runs in its own interpreter: torch first, then rtx. It drives the
multi-GPU frame assembly (rtx.dist.FrameGather) with every buffer a torch
tensor on torch's DEFAULT stream (handle 0 = HIP's null stream) and the
library told to launch there, and checks the image bit for bit against the
context's own-stream render. Prints "ok" or raises."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402
from rtx.dist import FrameGather  # noqa: E402

torch.cuda.set_device(0)
assert torch.cuda.current_stream().cuda_stream == 0  # the default stream is the null stream
W, H, T = 160, 90, 5
world = rtx.random_world(11, depth=50, spp=12)
frame = rtx.camera_look_at(W, H, aspect=W / H)
with rtx.Context(0) as ref:
    ref.upload_world(world)
    ref.set_frame(frame)
    want = ref.render_image()
ctx = rtx.Context(0, stream=torch.cuda.current_stream().cuda_stream)
ctx.upload_world(world)
ctx.set_frame(frame)
dev = torch.device("cuda", 0)
for nparts in (1, 3):
    # one process plays every part: render each part into its send buffer,
    # stack them as the gather would, de-interleave on the GPU
    parts = [FrameGather(W, H, T, p, nparts, device=dev,
                         render_part=lambda send, part, n: ctx.render_rows(T, part, n, send.data_ptr()))
             for p in range(nparts)]
    gathered = torch.zeros((nparts, parts[0].max_rows, W, 4), dtype=torch.float32, device=dev)
    for p, fg in enumerate(parts):
        fg.send.fill_(float("nan"))  # torch work on the default stream, then the render over it
        fg.render_part(fg.send, p, nparts)
        gathered[p].copy_(fg.send)
    image = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    ctx.deinterleave(gathered.data_ptr(), W, H, T, nparts, image.data_ptr())
    got = image.cpu().numpy()  # synchronises the default stream only
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    if not same.all():
        raise SystemExit(f"{nparts} parts: {(~same).sum()} values differ from the own-stream render")
ctx.close()
print("ok")
