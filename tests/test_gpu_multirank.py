"""The N>1 path with the real kernel (no test ran rtx_render_rows
under a multi-rank gather): world_size 2 and 3 ranks — separate processes,
each with its own librtx context on the box's one MI355X — render their
interleaved row tiles with rtx_render_rows, gather them to rank 0 with
torch.distributed (gloo: two ranks cannot share one GPU under RCCL), and
rank 0 de-interleaves on the GPU with rtx_deinterleave_rows (rtx/dist.py
FrameGather, the same host logic bench.py runs over RCCL). The assembled
frame must be bit-identical to the one-process frame and to the oracle's
rows."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world_size, port, W, H, T, spp, out_path):
    # torch before librtx: one HIP runtime in the process (DESIGN.md §6 caveat)
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
    import rtx
    from rtx.dist import FrameGather, part_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    world = rtx.random_world(11, depth=50, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    ctx = rtx.Context(0)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    dev = ctx.alloc((part_rows(H, T, 0, world_size), W, 4))

    def render_part(send, part, nparts):  # the kernel: this rank's rows on the GPU
        ctx.render_rows(T, part, nparts, dev.ptr)
        ctx.sync()
        send.copy_(torch.from_numpy(dev.numpy()))

    def deinterleave(gathered, image):  # rank 0: rtx_deinterleave_rows on the GPU
        g = ctx.alloc(tuple(gathered.shape))
        g.upload(gathered.numpy())
        img = ctx.alloc(tuple(image.shape))
        ctx.deinterleave(g.ptr, W, H, T, world_size, img.ptr)
        ctx.sync()
        image.copy_(torch.from_numpy(img.numpy()))
        g.free()
        img.free()

    fg = FrameGather(W, H, T, rank, world_size, render_part, deinterleave)
    img = fg.step()
    if rank == 0:
        np.save(out_path, img.numpy())
    dist.barrier()
    dev.free()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size,T", [(2, 5), (3, 4)])
def test_multirank_gather_with_the_kernel(tmp_path, gpu_ctx, oracle, rtx, world_size, T):
    W, H, spp = 320, 180, 12
    out = str(tmp_path / "img.npy")
    port = _free_port()
    spawn = mp.get_context("spawn")
    procs = [spawn.Process(target=_rank_main, args=(r, world_size, port, W, H, T, spp, out))
             for r in range(world_size)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = np.load(out)
    world = rtx.random_world(11, depth=50, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(frame)
    whole = gpu_ctx.render_image()
    same = (got.view(np.uint32) == whole.view(np.uint32)) | (np.isnan(got) & np.isnan(whole))
    assert same.all(), f"{int((~same).sum())} values differ from the one-process frame"
    rows = np.linspace(1, H - 2, 8).astype(np.uint32)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(got[rows].view(np.uint32), want.view(np.uint32))


def test_bench_rccl_path_one_rank(tmp_path, oracle, rtx):
    """bench.py's N-rank path (process group over RCCL — torch.distributed
    "nccl" —, the render into the rank's row-tile send buffer, ONE RCCL gather,
    rtx_deinterleave_rows, all ordered on one torch stream handed to librtx)
    run with one rank on the box's GPU (`--gather`): the driver's 8-GPU run is
    the only other place it executes. The line must carry the RCCL
    parallelism and the gathered frame must equal the oracle's rows."""
    import json
    import subprocess
    W, H, spp = 320, 180, 16
    img_path = str(tmp_path / "img.npy")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--gather", "--width", str(W),
           "--height", str(H), "--spp", str(spp), "--steps", "2", "--warmup", "1", "--pmc", "off",
           "--cpu-seconds", "0", "--parts", "", "--per-sample", "0", "--dump-image", img_path]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["config"]["parallelism"] == "row-tiles x1 + RCCL gather"
    got = np.load(img_path)
    world = rtx.random_world(11, depth=50, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    rows = np.linspace(1, H - 2, 8).astype(np.uint32)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(got[rows].view(np.uint32), want.view(np.uint32))


def test_bench_spawn_one_rank(tmp_path, oracle, rtx):
    """`bench.py --gpus 1 --spawn`: the self-launch the driver's `--gpus N`
    run takes — bench.py starts torch.distributed.run as a
    child, the rank runs the RCCL path — and the N-rank line's schema: the
    process group as torch.distributed saw it, the RCCL version, the rank's
    device and per-step render / gather / de-interleave times, and the
    gathered frame's rows bit-exact against the oracle."""
    import json
    import subprocess
    W, H, spp = 320, 180, 16
    img_path = str(tmp_path / "img.npy")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--spawn", "--width", str(W),
           "--height", str(H), "--spp", str(spp), "--steps", "3", "--warmup", "1", "--pmc", "off",
           "--cpu-seconds", "0", "--parts", "", "--per-sample", "0", "--dump-image", img_path]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["config"]["parallelism"] == "row-tiles x1 + RCCL gather"
    d = line["dist"]
    assert d["backend"] == "nccl" and d["world_size"] == 1 and d["rccl_version"]
    assert d["launcher"].startswith("bench.py self-launch")
    (pr,) = d["per_rank"]
    assert pr["rank"] == 0 and pr["rows"] == H
    for k in ("render_ms", "gather_ms", "deinterleave_ms", "step_ms"):
        assert pr[k] is not None and pr[k] >= 0, k
    assert pr["render_ms"] <= pr["step_ms"]
    p = line["parity"]
    assert p["bit_exact"] and p["rows_checked"] == 2 and p["values_differing"] == 0
    got = np.load(img_path)
    world = rtx.random_world(11, depth=50, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    rows = np.linspace(1, H - 2, 8).astype(np.uint32)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(got[rows].view(np.uint32), want.view(np.uint32))
