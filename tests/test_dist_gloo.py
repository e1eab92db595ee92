"""The N>1 path on CPU: world_size 2 (and 3) gloo ranks run the same host
logic as the MI355X ranks (rtx/dist.py: interleaved row tiles, one gather,
de-interleave), with the oracle standing in for the kernel. The gathered
frame must be bit-identical to a single-process render."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world_size, port, W, H, T, spp, out_path):
    sys.path[:0] = [os.path.join(ROOT, "raytrace-we-gpu_amd"), os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import oracle
    import rtx
    from rtx.dist import FrameGather, part_row_ids

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    world = rtx.random_world(4, depth=20, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)

    def render_part(send, part, nparts):  # the oracle stands in for rtx_render_rows
        ids = part_row_ids(H, T, part, nparts)
        rows, _ = oracle.render_rows(world, frame, ids, nthreads=1)
        send[:len(ids)] = torch.from_numpy(rows)

    fg = FrameGather(W, H, T, rank, world_size, render_part)
    img = fg.step()
    if rank == 0:
        np.save(out_path, img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size,T", [(2, 5), (3, 4)])
def test_gloo_gather_bit_identical(tmp_path, oracle, rtx, world_size, T):
    import torch.multiprocessing as mp
    W, H, spp = 48, 27, 2
    out = str(tmp_path / "img.npy")
    mp.spawn(_rank_main, args=(world_size, _free_port(), W, H, T, spp, out), nprocs=world_size, join=True)
    got = np.load(out)
    world = rtx.random_world(4, depth=20, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    want, _ = oracle.render_rows(world, frame, np.arange(H), nthreads=2)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_host_deinterleave_matches_partition(rtx):
    from rtx.dist import deinterleave_host, part_row_ids, part_rows
    H, T, R, W = 53, 4, 3, 2
    img = np.random.default_rng(0).normal(size=(H, W)).astype(np.float32)
    g = np.zeros((R, part_rows(H, T, 0, R), W), np.float32)
    for p in range(R):
        ids = part_row_ids(H, T, p, R)
        assert part_rows(H, T, p, R) == rtx.part_rows(H, T, p, R)
        g[p, :len(ids)] = img[ids]
    np.testing.assert_array_equal(deinterleave_host(g, H, T, R), img)
