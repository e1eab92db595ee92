"""Multi-GPU frame assembly: interleaved row tiles + ONE gather per frame.

SURVEY §8e: pixels are independent and the RNG seed depends only on the
global pixel (ShaderCompute.hlsl:295), so a frame splits across R ranks
with no data-path exchange. Rows are cut into `tile_rows`-row tiles dealt
round-robin (tile k -> rank k % R) so sky-heavy and sphere-heavy rows
balance; each rank renders its rows contiguously into a send buffer padded
to the largest part; one `torch.distributed.gather` (RCCL over xGMI with the
"nccl" backend, gloo on CPU) brings them to the root, which de-interleaves
them into the image (rtx_deinterleave_rows on the GPU).

The class is generic over two callables so the same host logic runs on
MI355X ranks (librtx) and in CPU gloo tests (oracle + numpy).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np


def part_rows(height: int, tile_rows: int, part: int, nparts: int) -> int:
    """Rows owned by `part` (same arithmetic as rtx_part_rows)."""
    if tile_rows == 0 or nparts == 0 or part >= nparts:
        return 0
    y = np.arange(height)
    return int(((y // tile_rows) % nparts == part).sum())


def part_row_ids(height: int, tile_rows: int, part: int, nparts: int) -> np.ndarray:
    y = np.arange(height, dtype=np.int64)
    return y[(y // tile_rows) % nparts == part].astype(np.uint32)


def deinterleave_host(gathered: np.ndarray, height: int, tile_rows: int, nparts: int) -> np.ndarray:
    """Host statement of rtx_deinterleave_rows: [R][max_rows][W][...] -> [H][W][...]."""
    out = np.empty((height,) + gathered.shape[2:], gathered.dtype)
    for p in range(nparts):
        ids = part_row_ids(height, tile_rows, p, nparts)
        out[ids] = gathered[p, :len(ids)]
    return out


class FrameGather:
    """Per-rank state for one frame size: send buffer, root's gather buffer
    and image, plus the step (render own rows -> gather -> de-interleave)."""

    def __init__(self, width: int, height: int, tile_rows: int, rank: int, world_size: int,
                 render_part: Callable, deinterleave: Optional[Callable] = None,
                 device=None, root: int = 0, collective: bool = False):
        import torch
        self.W, self.H, self.T, self.rank, self.R, self.root = width, height, tile_rows, rank, world_size, root
        self.max_rows = part_rows(height, tile_rows, 0, world_size)  # part 0 is the largest
        self.rows = part_rows(height, tile_rows, rank, world_size)
        kw = dict(dtype=torch.float32, device=device)
        self.send = torch.zeros((self.max_rows, width, 4), **kw)
        self.gathered = torch.zeros((world_size, self.max_rows, width, 4), **kw) if rank == root else None
        self.image = torch.zeros((height, width, 4), **kw) if rank == root else None
        self.render_part = render_part
        self.deinterleave = deinterleave
        # collective: gather through the process group even with one rank (a
        # one-GPU rehearsal of the N-rank path: RCCL's gather on the render's
        # buffers, the same stream order)
        self.collective = collective or world_size > 1
        # optional phase marks: mark("start" | "rendered" | "gathered" | "done")
        # at the step's phase boundaries (bench.py records HIP events there)
        self.mark: Optional[Callable] = None

    def _mark(self, name):
        if self.mark is not None:
            self.mark(name)

    def step(self):
        import torch.distributed as dist
        self._mark("start")
        self.render_part(self.send, self.rank, self.R)
        self._mark("rendered")
        if self.collective:
            gl = list(self.gathered.unbind(0)) if self.rank == self.root else None
            dist.gather(self.send, gather_list=gl, dst=self.root)
        elif self.rank == self.root:
            self.gathered[0].copy_(self.send)
        self._mark("gathered")
        if self.rank == self.root:
            if self.deinterleave is not None:
                self.deinterleave(self.gathered, self.image)
            else:
                self.image.copy_(self._deinterleave_torch())
        self._mark("done")
        return self.image

    def _deinterleave_torch(self):
        import torch
        img = deinterleave_host(self.gathered.cpu().numpy(), self.H, self.T, self.R)
        return torch.from_numpy(img).to(self.image.device)
