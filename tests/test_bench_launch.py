"""bench.py's rank launcher on CPU: `bench.py --gpus N`
outside torch.distributed.run starts its N ranks itself, as a fresh
`python -m torch.distributed.run` child, and never touches the GPU first.

* the child command and environment (rendezvous on 127.0.0.1, dmabuf IPC
  kept, the no-relaunch marker);
* fewer visible devices than N is a clear non-zero exit (this container has
  no GPU, so `--gpus 2` must refuse);
* the launcher itself, end to end, on 2 and 3 gloo ranks with the oracle
  standing in for the kernel (tests/dist_rank_helper.py): every rank sees
  the world size and env it should, runs FrameGather's phases in order, and
  the gathered frame equals the single-process oracle frame bit for bit.
The GPU side (`bench.py --gpus 1 --spawn`, the one-rank RCCL line) is
tests/test_gpu_multirank.py::test_bench_spawn_one_rank.
"""
import importlib.util
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_command_and_env(bench):
    cmd = bench.rank_launch_command(8, "/x/bench.py", ["--gpus", "8", "--steps", "3"], 29511, python="py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["/x/bench.py", "--gpus", "8", "--steps", "3"][-4:] and "/x/bench.py" in cmd
    env = bench.rank_launch_env({"HSA_ENABLE_IPC_MODE_LEGACY": "1", "PATH": "/bin"})
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["RTX_BENCH_RANKS_LAUNCHED"] == "1"
    assert env["PATH"] == "/bin"


def test_spawn_refuses_without_enough_devices():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, (r.returncode, r.stderr[-1000:])
    assert "needs 2 visible HIP devices, found 0" in r.stderr
    assert not r.stdout.strip()  # no bench line


@pytest.mark.parametrize("n,T", [(2, 5), (3, 4)])
def test_launched_ranks_gather_bit_identical(tmp_path, bench, oracle, rtx, n, T):
    W, H, spp = 40, 23, 2
    rc = bench.launch_ranks(n, os.path.join(ROOT, "tests", "dist_rank_helper.py"),
                            [str(tmp_path), str(W), str(H), str(T), str(spp)], timeout=240)
    assert rc == 0
    ranks = json.load(open(tmp_path / "ranks.json"))
    assert [r["rank"] for r in ranks] == list(range(n))
    assert all(r["world_size"] == n and r["local_rank"] == r["rank"] for r in ranks)
    assert all(r["ipc_legacy"] == "0" and r["launched"] == "1" and r["master_addr"] == "127.0.0.1"
               for r in ranks)
    assert all(r["marks"] == ["start", "rendered", "gathered", "done"] for r in ranks)
    got = np.load(tmp_path / "img.npy")
    world = rtx.random_world(4, depth=20, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    want, _ = oracle.render_rows(world, frame, np.arange(H), nthreads=2)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_gathered_parity_rows_cover_every_rank(bench, rtx):
    """The N>1 line's parity rows: two from every rank's share."""
    for H, T, R in [(1080, 5, 8), (1080, 5, 4), (1080, 5, 2), (180, 5, 1), (23, 4, 3)]:
        rows = bench.parity_rows(H, T, R)
        owners = {(r // T) % R for r in rows}
        assert owners == set(range(R)) and len(rows) == 2 * R and rows == sorted(rows)
        assert all(0 <= r < H for r in rows)


def test_kernel_class_names_every_render_instance(bench):
    """The PMC passes attribute counters by rocprof kernel name: every
    k_render template instance (3 to 5 bool parameters) must map to its role,
    or the bench line loses its executed-FLOP and issue fields."""
    for n in (3, 4, 5):
        rest = ", ".join(["false"] * (n - 1))
        assert bench.kernel_class(f"void rtx::k_render<true, {rest}>(rtx::KParams)") == "render"
        assert bench.kernel_class(f"void rtx::k_render<false, {rest}>(rtx::KParams)") == "render_grid"
        assert bench.kernel_class(f"void rtx::k_render<false, true, {', '.join(['true'] * (n - 2))}>(x)") == "prepass"
    assert bench.kernel_class("void rtx::k_render_ps<true, false, false>(rtx::KParams)") == "k_render_ps"
    assert bench.kernel_class("__amd_rocclr_fillBufferAligned") is None
