"""GPU parity tests: the HIP path (librtx.so, through the C-ABI) against the
CPU oracle. The bar is bit-exact: the kernel and the oracle execute the
same IEEE-754 fp32 operation sequence, so every pixel,
every hit record and every math-function output must have identical bits
(NaNs compare equal to NaNs). Against the reference's fp64 geometry the
stated fp32 tolerance of tests/tolerance.py applies.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from cases import grazing_rays, lambert_cases
from conftest import GOLDEN
from golden_cases import case_ids, load_case
from tolerance import check_hits_against_fp64

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    assert a.shape == b.shape
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return same


def assert_bits_equal(a, b, what=""):
    same = bits_equal(a, b)
    if not same.all():
        bad = np.argwhere(~same)
        raise AssertionError(f"{what}: {(~same).sum()} of {same.size} values differ; first at "
                             f"{bad[:5].tolist()}: gpu {np.asarray(a)[tuple(bad[0])]} vs oracle "
                             f"{np.asarray(b)[tuple(bad[0])]}")


# ---------------------------------------------------------------------------
# function-level parity
# ---------------------------------------------------------------------------
def _math_inputs(fn):
    rng = np.random.default_rng(sum(map(ord, fn)))
    if fn == "sqrt":
        return np.concatenate([rng.uniform(0, 10, 4000), 10.0 ** rng.uniform(-44, 38, 4000),
                               [0.0, -0.0, np.inf, -1.0, np.nan, 1e-45]]).astype(np.float32), None
    if fn == "div":
        a = np.concatenate([rng.normal(size=4000), 10.0 ** rng.uniform(-30, 30, 4000)])
        b = np.concatenate([rng.normal(size=4000), 10.0 ** rng.uniform(-30, 30, 4000)])
        return a.astype(np.float32), b.astype(np.float32)
    if fn in ("sin", "cos"):
        return np.concatenate([rng.uniform(0, 2 * np.pi, 6000), rng.uniform(-20, 20, 2000),
                               [0.0, np.float32(6.28318530718), np.pi / 2]]).astype(np.float32), None
    if fn == "log2":
        return np.concatenate([rng.uniform(0, 4, 3000), 10.0 ** rng.uniform(-44, 38, 5000),
                               [1.0, 2.0, 0.5, 1e-45, 1.17549435e-38]]).astype(np.float32), None
    if fn == "exp2":
        return np.concatenate([rng.uniform(-2, 2, 3000), rng.uniform(-160, 135, 5000),
                               [0.0, -126.0, -149.0, -150.0, 127.5, 128.0, np.nan]]).astype(np.float32), None
    if fn == "pow":
        a = np.concatenate([rng.uniform(0, 1, 3000), rng.uniform(0, 3, 3000), [0.0, 1.0, -1.0, np.inf, np.nan, 1e-40]])
        b = np.concatenate([np.full(3000, 1 / 3), rng.choice([0.454545454545, 5.0, 2.0], 3000), np.full(6, 1 / 3)])
        return a.astype(np.float32), b.astype(np.float32)
    if fn == "basehash":
        u = rng.integers(0, 2**32, size=(2, 8000), dtype=np.uint64).astype(np.uint32)
        return u[0].view(np.float32), u[1].view(np.float32)
    # hash1/2/3, rius: seeds
    return np.concatenate([rng.uniform(0, 1, 6000), rng.uniform(0, 40, 2000)]).astype(np.float32), None


@pytest.mark.parametrize("fn", ["sqrt", "div", "sin", "cos", "log2", "exp2", "pow", "basehash",
                                "hash1", "hash2", "hash3", "rius"])
def test_device_math_bit_exact(gpu_ctx, oracle, fn):
    a, b = _math_inputs(fn)
    got = gpu_ctx.debug_math(fn, a, b)
    want = oracle.math(fn, a, b)
    assert_bits_equal(got, want, fn)


# ---------------------------------------------------------------------------
# hit_world parity against the reference's golden vectors
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name,k", case_ids())
def test_hit_world_golden(gpu_ctx, oracle, rtx, name, k):
    """hit_world on the GPU against the reference's compiled Hittable_list::hit
    (tests/golden: test_world, the 326- and 486-sphere scenes, grazing rays
    over the 486-sphere scene, the 100k-sphere C5 scene): bit for bit equal
    to the fp32 twin, and within the stated fp32 tolerance of the reference
    (grazing: ill-conditioned rays exempt from the identity, tests/tolerance.py)."""
    c = load_case(name, k, lambda ext, cap: rtx.random_world(ext, capacity=cap).spheres)
    n = len(c["spheres"])
    world = rtx.World(c["spheres"], np.zeros(n, np.float32), np.zeros((n, 4), np.float32), 1, 1)
    gpu_ctx.upload_world(world)
    rays = c["rays"].astype(np.float32)
    got = gpu_ctx.debug_hit_world(rays, c["t_min"], c["t_max"])
    assert_bits_equal(got, oracle.hit_world_f32(world, rays, c["t_min"], c["t_max"]), "hit_world vs fp32 twin")
    check_hits_against_fp64(c["spheres"], c["rays"], got, c["expected"], c["t_min"], c["t_max"],
                            allow_ill=c["allow_ill"])


def test_hit_world_ties_and_padding(gpu_ctx, oracle, rtx):
    """Exact-t ties: the later sphere wins (strict `t_max < root`, ShaderCompute.hlsl:171).
    Counts not a multiple of the device padding (8) exercise the padded copies."""
    rng = np.random.default_rng(7)
    for n in (1, 2, 7, 9, 13):
        sph = np.concatenate([rng.uniform(-3, 3, (n, 3)), rng.uniform(0.2, 1.0, (n, 1))], 1).astype(np.float32)
        sph[n // 2] = sph[0]  # duplicate -> ties
        sph[-1] = sph[0] if n > 2 else sph[-1]
        world = rtx.World(sph, np.zeros(n, np.float32), np.zeros((n, 4), np.float32), 1, 1)
        gpu_ctx.upload_world(world)
        o = rng.uniform(-6, 6, (500, 3))
        d = (sph[rng.integers(0, n, 500), :3] - o) + rng.normal(scale=0.2, size=(500, 3))
        rays = np.concatenate([o, d], 1).astype(np.float32)
        got = gpu_ctx.debug_hit_world(rays)
        want = oracle.hit_world_f32(world, rays)
        assert_bits_equal(got, want, f"n={n}")
        if n > 2:
            hit0 = want[:, 9] >= 0
            assert not np.any(np.isin(want[hit0, 9], [0])), "tie must go to the later duplicate"


def test_hit_world_t_range_contract(gpu_ctx, oracle, rtx):
    """rtx_debug_hit_world's t range: t_min must be finite and > 0 (the
    resolve orders roots by their bits), t_max < t_min means no hit, a tiny
    positive t_min is bit-exact against the oracle."""
    world = rtx.random_world(11, depth=1, spp=1)
    gpu_ctx.upload_world(world)
    rng = np.random.default_rng(21)
    rays = grazing_rays(world.spheres, 3000, rng)
    for bad in (0.0, -0.0, -1.0, float("nan"), float("inf")):
        with pytest.raises(rtx.RtxError, match="t_min"):
            gpu_ctx.debug_hit_world(rays, t_min=bad)
    with pytest.raises(rtx.RtxError, match="NaN"):
        gpu_ctx.debug_hit_world(rays, t_max=float("nan"))
    none = gpu_ctx.debug_hit_world(rays, t_min=2.0, t_max=1.0)
    assert (none[:, 0] == 0).all() and (none[:, 9] == -1).all()
    for t_min, t_max in ((1e-30, float("inf")), (1e-3, 7.5), (3.0, 3.0)):
        got = gpu_ctx.debug_hit_world(rays, t_min=t_min, t_max=t_max)
        assert_bits_equal(got, oracle.hit_world_f32(world, rays, t_min, t_max), f"t in [{t_min}, {t_max}]")


@pytest.mark.parametrize("which", ["c5_100k", "ties"])
def test_hit_world_wrapped_scan_starts(gpu_ctx, oracle, rtx, which):
    """The large-scene kernels start a segment's scan where their workgroup's
    other waves are (pack start) and wrap round ([b0, nblk) then [0, b0)):
    the resolution rule must give the in-order answer from every start —
    rtx_debug_hit_world_from at start blocks 0, 1, mid, nblk - 1 and beyond,
    on the 100k-sphere golden case and on a scene of duplicated spheres
    whose ties straddle the wrap point; and the culled scan (spatial order)
    on both."""
    if which == "c5_100k":
        c = load_case("hit_c5_100k.npz", 0, lambda ext, cap: rtx.random_world(ext, capacity=cap).spheres)
        sph, rays, t_min = c["spheres"], c["rays"].astype(np.float32), c["t_min"]
    else:
        rng = np.random.default_rng(17)
        base = np.concatenate([rng.uniform(-8, 8, (700, 1)), rng.uniform(-1, 2, (700, 1)),
                               rng.uniform(-8, 8, (700, 1)), rng.uniform(0.2, 0.9, (700, 1))], 1)
        sph = np.concatenate([base, base[::-1]]).astype(np.float32)  # every sphere twice, far apart in index
        o = rng.uniform(-10, 10, (6000, 3))
        d = (sph[rng.integers(0, len(sph), 6000), :3] - o) + rng.normal(scale=0.1, size=(6000, 3))
        rays, t_min = np.concatenate([o, d], 1).astype(np.float32), 0.001
    n = len(sph)
    world = rtx.World(sph, np.zeros(n, np.float32), np.zeros((n, 4), np.float32), 1, 1)
    gpu_ctx.upload_world(world)
    want = oracle.hit_world_f32(world, rays, t_min)
    nblk = (n + 7) // 8
    for start in (0, 1, nblk // 2, nblk - 1, nblk + 3, rtx.DEBUG_CULLED):
        got = gpu_ctx.debug_hit_world(rays, t_min=t_min, start_block=start)
        assert_bits_equal(got, want, f"{which}: scan from block {start} of {nblk}")
    if which == "ties":
        hit = want[:, 9] >= 0
        assert (want[hit, 9] >= n // 2).all(), "a tie must go to the later duplicate"


@pytest.mark.parametrize("scan", ["plain", "culled"])
def test_hit_world_grazing_rays(gpu_ctx, oracle, rtx, scan):
    """Rays whose line passes within 1e-9..1e-2 (relative) of a sphere's
    silhouette, on either side, plus near-vertical rays and rays near the x
    axis (the prefilter basis's degenerate direction), tiny and huge
    direction lengths (some outside the prefilter's safe range) and origins
    far down the line: the kernel's prefiltered scan (rtx_prefilter.h) must
    return the reference scan's records bit for bit — the plain scan (the
    486-sphere scene) and the culled one (block bounds first, spatial order,
    position map; a 2,504-sphere random scene)."""
    rng = np.random.default_rng(11)
    world = rtx.random_world(11 if scan == "plain" else 25, depth=1, spp=1)
    rays = grazing_rays(world.spheres, 30000, rng, xaxis_frac=0.05)
    gpu_ctx.upload_world(world)
    got = gpu_ctx.debug_hit_world(rays, start_block=rtx.DEBUG_CULLED if scan == "culled" else None)
    want = oracle.hit_world_f32(world, rays)
    assert_bits_equal(got, want, f"grazing rays, {scan} scan")
    assert (want[:, 0] == 1).mean() > 0.3


@pytest.mark.parametrize("walk", ["bfs", "lane"])
@pytest.mark.parametrize("q", [1, 2, 5, 8, 17, 32, 64])
def test_hit_world_culled_coop(gpu_ctx, oracle, rtx, q, walk):
    """The culled scan split over a wave's lanes (hit_world_groups_culled: the
    large-scene frame tail, heavy tiers and promoted pixels), q rays per wave
    (64 lanes per ray at q = 1 down to 2 at q = 32; q > 32 in two chunks), in
    both walks: k_render's (one ray per wave breadth first) and the per-lane
    walk k_render_ps runs at every q: grazing rays
    over a 2,504-sphere scene (its flat layer's radii 0.05..0.6), aimed and random rays over a scene of
    duplicated spheres (ties), bit for bit against the oracle."""
    coop = rtx.DEBUG_CULLED_COOP if walk == "bfs" else rtx.DEBUG_CULLED_COOP_LANE
    rng = np.random.default_rng(100 + q)
    world = rtx.random_world(25, depth=1, spp=1)
    layer = world.spheres[:, 1] == np.float32(0.2)  # the flat layer, with radii 0.05..0.6 instead of 0.2
    world.spheres[layer, 3] = rng.uniform(0.05, 0.6, layer.sum()).astype(np.float32)
    rays = grazing_rays(world.spheres, 4000, rng, xaxis_frac=0.05)
    gpu_ctx.upload_world(world)
    got = gpu_ctx.debug_hit_world(rays, start_block=coop(q))
    assert_bits_equal(got, oracle.hit_world_f32(world, rays), f"culled coop {walk} q={q}, grazing")
    base = np.concatenate([rng.uniform(-20, 20, (900, 1)), rng.uniform(0, 2, (900, 1)),
                           rng.uniform(-20, 20, (900, 1)), rng.uniform(0.2, 0.9, (900, 1))], 1)
    sph = np.concatenate([base, base[::-1]]).astype(np.float32)
    n = len(sph)
    dup = rtx.World(sph, np.zeros(n, np.float32), np.zeros((n, 4), np.float32), 1, 1)
    gpu_ctx.upload_world(dup)
    o = rng.uniform(-22, 22, (3000, 3))
    d = (sph[rng.integers(0, n, 3000), :3] - o) + rng.normal(scale=0.1, size=(3000, 3))
    rays = np.concatenate([np.concatenate([o, d], 1), rng.normal(size=(1000, 6)) * 10]).astype(np.float32)
    want = oracle.hit_world_f32(dup, rays, 0.001)
    got = gpu_ctx.debug_hit_world(rays, t_min=0.001, start_block=coop(q))
    assert_bits_equal(got, want, f"culled coop {walk} q={q}, ties")
    hit = want[:, 9] >= 0
    assert (want[hit, 9] >= n // 2).all(), "a tie must go to the later duplicate"


def surface_rays(sph, count, rng):
    """Rays starting on (or within 1e-7..1e-2 of) a sphere's surface: half
    leaving it radially (the tight case of the culled scan's half test: the
    hit at t ~ 0, the sphere's bounds behind the origin), half in random
    directions; direction lengths 1e-2..1e2."""
    idx = rng.integers(0, len(sph), count)
    c, r = sph[idx, :3].astype(np.float64), sph[idx, 3:4].astype(np.float64)
    nrm = rng.normal(size=(count, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    delta = np.where(rng.random((count, 1)) < 0.3, 0.0,
                     10.0 ** rng.uniform(-7, -2, (count, 1)) * rng.choice([-1.0, 1.0], (count, 1)))
    o = c + r * (1.0 + delta) * nrm
    radial = rng.random((count, 1)) < 0.5
    d = np.where(radial, nrm + 1e-4 * rng.normal(size=(count, 3)) * (rng.random((count, 1)) < 0.5),
                 rng.normal(size=(count, 3)))
    d *= 10.0 ** rng.uniform(-2, 2, (count, 1))
    return np.concatenate([o, d], 1).astype(np.float32)


@pytest.mark.parametrize("mode", ["lane", "coop1", "coop8", "coop1_lane"])
def test_hit_world_culled_half_test(gpu_ctx, oracle, rtx, mode):
    """The culled scan's half test (a bound wholly behind the origin fails;
    rtx_prefilter.h HalfTest) at its tight case — rays leaving a sphere's
    surface, whose reference roots sit at t ~ 0 — at t_min 1e-6, 1e-3 and
    0.5 (the API takes t_min > 0; the kernel's guard for t_min < 0 is
    covered by tests/prefilter_check.cpp's t_min 0 cases), lane mode and the
    coop (one ray per wave: breadth first; eight: the per-lane walk), bit for
    bit against the oracle."""
    rng = np.random.default_rng({"lane": 7, "coop1": 8, "coop8": 9, "coop1_lane": 10}[mode])
    world = rtx.random_world(25, depth=1, spp=1)
    layer = world.spheres[:, 1] == np.float32(0.2)
    world.spheres[layer, 3] = rng.uniform(0.05, 0.6, layer.sum()).astype(np.float32)
    gpu_ctx.upload_world(world)
    rays = np.concatenate([surface_rays(world.spheres, 5000, rng), grazing_rays(world.spheres, 1000, rng)])
    start = {"lane": rtx.DEBUG_CULLED, "coop1": rtx.DEBUG_CULLED_COOP(1), "coop8": rtx.DEBUG_CULLED_COOP(8),
             "coop1_lane": rtx.DEBUG_CULLED_COOP_LANE(1)}[mode]
    for t_min in (1e-6, 0.001, 0.5):
        want = oracle.hit_world_f32(world, rays, t_min)
        got = gpu_ctx.debug_hit_world(rays, t_min=t_min, start_block=start)
        assert_bits_equal(got, want, f"culled half test, {mode}, t_min={t_min}")
        assert (want[:, 9] >= 0).mean() > 0.3


@pytest.mark.parametrize("layout", ["all_flat", "no_flat"])
def test_hit_world_culled_scan_sections(gpu_ctx, oracle, rtx, layout):
    """The culled layout's edge cases: a scene that is one flat layer but for
    the ground sphere (the flat section after one padded block), and one with
    no two centres at the same height (no flat section, nothing stretched)."""
    rng = np.random.default_rng(5 if layout == "all_flat" else 6)
    n = 3000
    ext = 11.0 * np.sqrt(n / 486.0)
    y = np.full((n - 1, 1), 0.2) if layout == "all_flat" else rng.uniform(0, 3, (n - 1, 1))
    small = np.concatenate([rng.uniform(-ext, ext, (n - 1, 1)), y, rng.uniform(-ext, ext, (n - 1, 1)),
                            rng.uniform(0.05, 0.5, (n - 1, 1))], 1)
    sph = np.concatenate([[[0, -1000, 0, 1000]], small]).astype(np.float32)
    world = rtx.World(sph, np.zeros(n, np.float32), np.zeros((n, 4), np.float32), 1, 1)
    gpu_ctx.upload_world(world)
    o = rng.uniform(-ext, ext, (5000, 3)) * np.array([1, 0.2, 1]) + np.array([0, 4, 0])
    d = (sph[rng.integers(1, n, 5000), :3] - o) + rng.normal(scale=0.2, size=(5000, 3))
    rays = np.concatenate([np.concatenate([o, d], 1), grazing_rays(sph[1:], 5000, rng, xaxis_frac=0.05)])
    rays = rays.astype(np.float32)
    want = oracle.hit_world_f32(world, rays)
    for start, what in ((rtx.DEBUG_CULLED, "lane"), (rtx.DEBUG_CULLED_COOP(1), "coop 1"),
                        (rtx.DEBUG_CULLED_COOP(8), "coop 8"), (rtx.DEBUG_CULLED_COOP_LANE(1), "coop 1, per-lane walk")):
        assert_bits_equal(gpu_ctx.debug_hit_world(rays, start_block=start), want, f"{layout}, {what}")
    assert (want[:, 0] == 1).mean() > 0.4


@pytest.mark.parametrize("n", [1025, 1100, 1500, 4100, 12000])
def test_hit_world_culled_scan(gpu_ctx, oracle, rtx, n):
    """The culled scan (DESIGN.md §3e "culled scan") on scenes across its size
    range: random spheres at mixed heights, a flat run at one height (the 5-op
    bound test), a few large spheres (their own section) and duplicated
    spheres whose ties must still go to the later index though the layout
    reorders them; rays aimed at spheres, random ones and grazing ones, at
    two t_min's."""
    rng = np.random.default_rng(n)
    k = n // 3
    ext = 11.0 * np.sqrt(n / 486.0)  # the RTIOW density
    # the flat run (one centre height) with radii 0.05..0.6: its bounds live in the stretched space
    flat = np.concatenate([rng.uniform(-ext, ext, (k, 1)), np.full((k, 1), 0.2), rng.uniform(-ext, ext, (k, 1)),
                           rng.uniform(0.05, 0.6, (k, 1))], 1)
    big = np.array([[0, -1000, 0, 1000], [0, 1, 0, 1.0], [-4, 1, 0, 1.0], [4, 1, 0, 1.0]])
    m = n - k - len(big) - 8
    other = np.concatenate([rng.uniform(-ext, ext, (m, 1)), rng.uniform(0, 3, (m, 1)), rng.uniform(-ext, ext, (m, 1)),
                            rng.uniform(0.1, 0.5, (m, 1))], 1)
    sph = np.concatenate([big[:1], other, flat, big[1:]]).astype(np.float32)
    dup_src = rng.choice(len(sph) - 1, 8, replace=False) + 1
    sph = np.concatenate([sph, sph[dup_src]]).astype(np.float32)  # the copies come later: they win ties
    assert len(sph) == n
    world = rtx.World(sph, np.zeros(n, np.float32), np.zeros((n, 4), np.float32), 1, 1)
    gpu_ctx.upload_world(world)
    o = rng.uniform(-ext - 3, ext + 3, (6000, 3)) * np.array([1, 0.3, 1]) + np.array([0, 8, 0])
    d = (sph[rng.integers(1, n, 6000), :3] - o) + rng.normal(scale=0.15, size=(6000, 3))
    rays = np.concatenate([np.concatenate([o, d], 1), grazing_rays(sph, 6000, rng, xaxis_frac=0.05),
                           np.concatenate([rng.uniform(-ext, ext, (3000, 3)), rng.normal(size=(3000, 3))], 1)])
    rays = rays.astype(np.float32)
    for t_min in (0.001, 0.5):
        want = oracle.hit_world_f32(world, rays, t_min)
        got = gpu_ctx.debug_hit_world(rays, t_min=t_min, start_block=rtx.DEBUG_CULLED)
        assert_bits_equal(got, want, f"n={n} culled scan, t_min={t_min}")
        hit = want[:, 9] >= 0
        assert hit.mean() > 0.3
        assert not np.isin(want[hit, 9], dup_src).any(), "a tie must go to the later duplicate"


# ---------------------------------------------------------------------------
# whole-frame parity
# ---------------------------------------------------------------------------
def render_gpu(ctx, world, frame):
    ctx.upload_world(world)
    ctx.set_frame(frame)
    ctx.stats_reset()
    img = ctx.render_image()
    return img, ctx.stats()


def test_c1_full_frame_bit_exact(gpu_ctx, oracle, rtx):
    """C1: 400x225 test_world, Camera.h, spp 20, depth 12 — every pixel bit-exact,
    and equal to the committed golden rows of the oracle."""
    world = rtx.test_world(depth=12, spp=20)
    frame = rtx.camera_simple(400, 225)
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(225), nthreads=8)
    assert_bits_equal(img, want, "C1 image")
    assert st.segments == segs
    gold = np.load(os.path.join(GOLDEN, "c1_oracle_rows.npz"))
    assert_bits_equal(img[gold["rows"]], gold["pixels"], "C1 golden rows")


@pytest.mark.parametrize("ext,w,h,spp,depth,rng_mode", [
    (11, 192, 108, 6, 50, 0),
    (9, 160, 90, 4, 50, 0),
    (11, 96, 54, 5, 50, 1),
    (3, 33, 17, 3, 7, 0),
])
def test_random_world_frames_bit_exact(gpu_ctx, oracle, rtx, ext, w, h, spp, depth, rng_mode):
    world = rtx.random_world(ext, depth=depth, spp=spp)
    frame = rtx.camera_look_at(w, h, aspect=w / h)
    frame.rng_mode = rng_mode
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(h), nthreads=8)
    assert_bits_equal(img, want, f"random_world({ext}) {w}x{h}")
    assert st.segments == segs
    assert st.sphere_tests == segs * world.count


def test_lambert_guard_device(gpu_ctx, oracle):
    """RTX_FN_LAMBERT_DIR[_GUARD]: the kernel's diffuse direction equals the
    oracle's bit for bit; zero directions give NaN unguarded, the normal guarded."""
    p, nrm, rius, nz = lambert_cases()
    for guard in (False, True):
        got = gpu_ctx.debug_lambert_dir(p, nrm, rius, guard)
        want = oracle.lambert_dir(p, nrm, rius, guard)
        assert_bits_equal(got[:-nz], want[:-nz], f"lambert guard={guard}")
        if guard:
            assert_bits_equal(got[-nz:], nrm[-nz:], "guarded zero directions")
        else:
            assert np.isnan(got[-nz:]).all()


def test_lambert_guard_frame_bit_exact(gpu_ctx, oracle, rtx):
    world = rtx.random_world(9, depth=20, spp=3)
    frame = rtx.camera_look_at(96, 54, aspect=96 / 54)
    frame.flags = rtx.FRAME_LAMBERT_GUARD
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(54), nthreads=8)
    assert_bits_equal(img, want, "lambert-guard frame")
    assert st.segments == segs
    bad = rtx.camera_look_at(96, 54, aspect=96 / 54)
    bad.flags = 2
    with pytest.raises(rtx.RtxError):
        gpu_ctx.set_frame(bad)


@pytest.mark.parametrize("spp,depth", [(1, 25), (8, 25)])
def test_ps_world_bit_exact(gpu_ctx, oracle, rtx, spp, depth):
    """f-4: the pixel-shader prototype's 7-sphere scene (Shader_RT.fx:300-335)
    at its own depth 25, through the compute path, every pixel bit-exact."""
    world = rtx.ps_world(depth=depth, spp=spp)
    frame = rtx.camera_look_at(320, 180)
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(180), nthreads=8)
    assert_bits_equal(img, want, f"ps_world spp {spp}")
    assert st.segments == segs

def test_c2_full_size_row_subset(gpu_ctx, oracle, rtx):
    """C2 at full size: 1920x1080, RTIOW final scene (486 spheres), spp 100,
    depth 50. The oracle renders every 24th row (45 rows, 8.6 M samples);
    those rows must be bit-identical in the GPU frame."""
    world = rtx.random_world(11, depth=50, spp=100)
    frame = rtx.camera_look_at(1920, 1080)
    img, st = render_gpu(gpu_ctx, world, frame)
    rows = np.arange(7, 1080, 24)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img[rows], want, "C2 rows")
    assert np.isfinite(img).all()
    assert st.samples == 1920 * 1080 * 100


def test_c3_full_size_rows(gpu_ctx, oracle, rtx):
    """C3 at full size: 3840x2160, RTIOW final scene (486 spheres), spp 1024,
    depth 50 (BASELINE configs[2]). 8 full rows spread over the image must be
    bit-identical to the oracle's; the frame's segment count (the scheduled
    render's own counter) must equal the per-pixel counts of an independent
    exact-grid pass (rtx_debug_pixel_cost), whose sums over those rows equal
    the oracle's."""
    W, H = 3840, 2160
    world = rtx.random_world(11, depth=50, spp=1024)
    frame = rtx.camera_look_at(W, H)
    img, st = render_gpu(gpu_ctx, world, frame)
    assert st.samples == W * H * 1024
    rows = np.linspace(11, H - 11, 8).astype(np.uint32)
    want, segs = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img[rows], want, "C3 rows")
    assert np.isfinite(img).all()
    cost = gpu_ctx.debug_pixel_cost(0)
    assert int(cost.sum(dtype=np.uint64)) == st.segments
    assert int(cost[rows].sum(dtype=np.uint64)) == segs


def test_c5_exact_grid_100k_spheres(gpu_ctx, oracle, rtx):
    """100,000 spheres (C5's scene) at spp 2 < kLptMinSpp: the exact-grid
    kernel k_render<false> with the double-buffered (kPF) scan."""
    world = rtx.random_world(159, capacity=100000, depth=50, spp=2)
    frame = rtx.camera_look_at(48, 27, aspect=48 / 27)
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(27), nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img, want, "100k spheres")
    assert st.segments == segs


def test_c5_scheduled_path_100k_spheres(gpu_ctx, oracle, rtx):
    """C5 on the bench's path (BASELINE configs[4]: 100k spheres, spp 16):
    spp >= kLptMinSpp takes the cost pre-pass and resumed state, the
    persistent cost-ordered render with the kPF scan and its 24-entry lists
    (RTX_CAND_PF), and, on a frame this small, the heavy-pixel coop tiers
    reading the spheres from HBM. Every pixel bit-exact, same segments."""
    world = rtx.random_world(159, capacity=100000, depth=50, spp=16)
    frame = rtx.camera_look_at(64, 36, aspect=64 / 36)
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(36), nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img, want, "C5 scheduled path")
    assert st.segments == segs
    assert st.samples == 64 * 36 * 16


def test_c5_full_width_rows(gpu_ctx, oracle, rtx):
    """C5 at full size (BASELINE configs[4]: 100k spheres, 1920x1080, spp 16,
    depth 50) on the bench's schedule: the kPF scan with its pack start,
    lane mode with 24-entry lists, the 1-spp persistent pre-pass, the tail
    coop reading the scene from HBM. Eight full 1920-px rows spread over the
    image (sky, horizon, the far and near field, the big spheres) bit-exact
    against the oracle; the frame's segment count (the scheduled render's own
    counter) equal to the per-pixel counts of an independent exact-grid pass
    (rtx_debug_pixel_cost), whose sums over those rows equal the oracle's."""
    W, H = 1920, 1080
    world = rtx.random_world(159, capacity=100000, depth=50, spp=16)
    frame = rtx.camera_look_at(W, H)
    img, st = render_gpu(gpu_ctx, world, frame)
    assert st.samples == W * H * 16
    rows = np.unique(np.concatenate([np.linspace(4, H - 5, 6), [317, 771]])).astype(np.uint32)
    want, segs = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img[rows], want, "C5 rows")
    assert np.isfinite(img).all()
    cost = gpu_ctx.debug_pixel_cost(0)
    assert int(cost.sum(dtype=np.uint64)) == st.segments
    assert int(cost[rows].sum(dtype=np.uint64)) == segs


def test_per_sample_c5_full_width_rows(gpu_ctx, oracle, rtx):
    """C5 at full size in per-sample RNG mode (rng_mode 1: 1920x1080, 100k
    spheres, spp 16, depth 50) — the path where round 3's illegal-address
    fault hit ("Faults"): k_render_ps with the kPF SGPR scan
    (no per-wave LDS tile in this kernel) and its group-coop tail reading the
    scene from HBM. Eight full rows (spread over the image) bit-exact against
    the oracle in the same RNG mode; the frame's segment count equal to an
    independent exact-grid pass's per-pixel counts (rtx_debug_pixel_cost, per-sample seeds too),
    whose sums over those rows equal the oracle's."""
    W, H = 1920, 1080
    world = rtx.random_world(159, capacity=100000, depth=50, spp=16)
    frame = rtx.camera_look_at(W, H)
    frame.rng_mode = 1
    img, st = render_gpu(gpu_ctx, world, frame)
    assert st.samples == W * H * 16
    rows = np.unique(np.concatenate([np.linspace(9, H - 9, 6), [211, 866]])).astype(np.uint32)
    want, segs = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img[rows], want, "per-sample C5 rows")
    assert np.isfinite(img).all()
    cost = gpu_ctx.debug_pixel_cost(0)
    assert int(cost.sum(dtype=np.uint64)) == st.segments
    assert int(cost[rows].sum(dtype=np.uint64)) == segs


def test_edge_cases(gpu_ctx, oracle, rtx):
    """Empty scene (all sky), spp 0 (0/0 = NaN, as accColor /= 0), depth 0
    (black), unknown material code (no scatter -> black), 1x1 frame."""
    base = rtx.random_world(2, depth=10, spp=3)
    empty = rtx.World(np.zeros((0, 4), np.float32), np.zeros(0, np.float32), np.zeros((0, 4), np.float32), 5, 3)
    odd = rtx.World(base.spheres.copy(), base.mat_types.copy(), base.mat_values.copy(), 10, 3)
    odd.mat_types[::3] = 7.0
    odd.mat_types[1::5] = 0.5
    cases = [(empty, 20, 10), (rtx.World(base.spheres, base.mat_types, base.mat_values, 10, 0), 9, 5),
             (rtx.World(base.spheres, base.mat_types, base.mat_values, 0, 3), 9, 5), (odd, 31, 9),
             (base, 1, 1)]
    for world, w, h in cases:
        frame = rtx.camera_look_at(w, h, aspect=max(w / h, 0.1))
        img, _ = render_gpu(gpu_ctx, world, frame)
        want, _ = oracle.render_rows(world, frame, np.arange(h))
        assert_bits_equal(img, want, f"edge case n={world.count} spp={world.spp} depth={world.depth}")
    img, _ = render_gpu(gpu_ctx, rtx.World(base.spheres, base.mat_types, base.mat_values, 10, 0),
                        rtx.camera_look_at(4, 2))
    assert np.isnan(img[..., :3]).all() and (img[..., 3] == 1).all()


def test_determinism(gpu_ctx, rtx):
    world = rtx.random_world(11, depth=50, spp=4)
    frame = rtx.camera_look_at(320, 180)
    a, _ = render_gpu(gpu_ctx, world, frame)
    b, _ = render_gpu(gpu_ctx, world, frame)
    assert_bits_equal(a, b, "two renders")


def test_lpt_schedule_and_pixel_cost(gpu_ctx, oracle, rtx):
    """spp >= 8 takes the cost-ordered persistent path (1-spp pre-pass +
    counting sort): the frame and segment count equal the oracle's, and the
    per-pixel segment counts (rtx_debug_pixel_cost) equal the oracle's
    per-row totals and sum to the frame's count."""
    W, H = 128, 72
    world = rtx.random_world(11, depth=50, spp=9)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(H), nthreads=8)
    assert_bits_equal(img, want, "LPT frame")
    assert st.segments == segs
    cost = gpu_ctx.debug_pixel_cost(0)
    assert cost.shape == (H, W) and int(cost.sum()) == segs
    for y in (0, 31, H - 1):
        _, row_segs = oracle.render_rows(world, frame, [y])
        assert int(cost[y].sum()) == row_segs
    one = gpu_ctx.debug_pixel_cost(1)
    assert (one >= 1).all() and (one <= 50).all()
    # the pre-pass does not disturb the framebuffer or the stats
    assert_bits_equal(gpu_ctx.download(), img, "framebuffer after cost pass")
    assert gpu_ctx.stats().segments == segs


# ---------------------------------------------------------------------------
# per-sample RNG: one lane per (pixel, sample) (k_render_ps)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("ext,w,h,spp,depth", [
    (11, 96, 54, 100, 50),   # batches of 40 pixels
    (11, 64, 36, 1, 50),     # one sample per pixel: 64-pixel batches, lanes wait for folds
    (11, 33, 17, 7, 3),      # ragged last batch, shallow paths
    (4, 3, 2, 5000, 20),     # spp > 4096: one pixel per batch, scratch sized by spp
    (20, 48, 27, 9, 50),     # > kScanPfMin spheres: the kPF scan
])
def test_per_sample_kernel_bit_exact(gpu_ctx, oracle, rtx, ext, w, h, spp, depth):
    """rng_mode 1 takes k_render_ps: lanes trace single samples of a batch
    of pixels, each pixel's sample colours are folded in sample order; the
    frame and its segment count equal the oracle's (pixel by pixel, samples
    in order, one seed per (pixel, sample))."""
    world = rtx.random_world(ext, depth=depth, spp=spp)
    frame = rtx.camera_look_at(w, h, aspect=w / h)
    frame.rng_mode = 1
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(h), nthreads=8)
    assert_bits_equal(img, want, f"per-sample {w}x{h} spp {spp}")
    assert st.segments == segs
    assert st.samples == w * h * spp


def test_per_sample_options_and_parts(gpu_ctx, oracle, rtx):
    """k_render_ps with thin lens, frame_index, the Lambert guard, a 5-way
    row split and progressive accumulation: bit-exact in every case."""
    W, H, spp = 80, 45, 12
    world = rtx.random_world(11, depth=50, spp=spp)

    def fr():
        f = rtx.camera_look_at(W, H, aspect=W / H)
        f.rng_mode = 1
        return f
    lens = rtx.set_aperture(fr(), 0.4)
    idx = fr()
    idx.frame_index = 5
    guard = fr()
    guard.flags = rtx.FRAME_LAMBERT_GUARD
    for name, f in (("thin lens", lens), ("frame_index", idx), ("lambert guard", guard)):
        img, st = render_gpu(gpu_ctx, world, f)
        want, segs = oracle.render_rows(world, f, np.arange(H), nthreads=8)
        assert_bits_equal(img, want, f"per-sample {name}")
        assert st.segments == segs
    f = fr()
    gpu_ctx.set_frame(f)
    buf = gpu_ctx.alloc((H, W, 4))
    for part in range(5):
        rows = rtx.part_row_ids(H, 4, part, 5)
        gpu_ctx.render_rows(4, part, 5, buf.ptr)
        got = buf.numpy().reshape(-1)[: len(rows) * W * 4].reshape(len(rows), W, 4)
        want, _ = oracle.render_rows(world, f, rows, nthreads=8)
        assert_bits_equal(got, want, f"per-sample part {part} of 5")
    buf.free()
    total = np.zeros((H, W, 3), np.float32)
    for k in range(2):
        gpu_ctx.accumulate(reset=(k == 0))
        g = fr()
        g.frame_index = k
        lin, _ = oracle.render_rows_linear(world, g, np.arange(H), nthreads=8)
        total = total + lin[..., :3]
    mean = (total / np.float32(2 * spp)).astype(np.float32)
    want = oracle.math("pow", mean.ravel(), np.full(mean.size, 0.454545454545, np.float32)).reshape(mean.shape)
    assert_bits_equal(gpu_ctx.download()[..., :3], want, "per-sample accumulation")


def test_per_sample_c2_rows(gpu_ctx, oracle, rtx):
    """The C2 frame (1920x1080, 486 spheres, spp 100, depth 50) in per-sample
    mode: 24 rows bit-exact against the oracle, and one rank's share of an
    8-way split bit-exact too."""
    world = rtx.random_world(11, depth=50, spp=100)
    frame = rtx.camera_look_at(1920, 1080)
    frame.rng_mode = 1
    img, st = render_gpu(gpu_ctx, world, frame)
    assert st.samples == 1920 * 1080 * 100
    rows = np.arange(13, 1080, 45)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img[rows], want, "per-sample C2 rows")
    ids = rtx.part_row_ids(1080, 5, 6, 8)
    buf = gpu_ctx.alloc((len(ids), 1920, 4))
    gpu_ctx.render_rows(5, 6, 8, buf.ptr)
    got = buf.numpy()
    buf.free()
    assert_bits_equal(got, img[ids], "per-sample part 6 of 8 vs the whole frame")


# ---------------------------------------------------------------------------
# row-tile partitions (the multi-GPU data path) on one device
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("nparts,tile_rows", [(2, 8), (3, 5), (8, 5), (8, 1), (5, 64)])
def test_partitions_reassemble_bit_identical(gpu_ctx, rtx, nparts, tile_rows):
    """Each part renders its interleaved row tiles into its own buffer; the
    gathered buffers de-interleave (rtx_deinterleave_rows) into exactly the
    single-device image — the R-rank frame is bit-identical for every R.
    (Device buffers come from rtx_alloc: no second HIP runtime via torch.)"""
    W, H = 200, 117
    world = rtx.random_world(11, depth=50, spp=3)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    full, _ = render_gpu(gpu_ctx, world, frame)
    max_rows = rtx.part_rows(H, tile_rows, 0, nparts)
    gathered = gpu_ctx.alloc((nparts, max_rows, W, 4))
    gathered.upload(np.zeros((nparts, max_rows, W, 4), np.float32))
    image = gpu_ctx.alloc((H, W, 4))
    part_bytes = max_rows * W * 16
    for p in range(nparts):
        rows = rtx.part_rows(H, tile_rows, p, nparts)
        assert rows == len(rtx.part_row_ids(H, tile_rows, p, nparts))
        gpu_ctx.render_rows(tile_rows, p, nparts, gathered.ptr + p * part_bytes)
    g = gathered.numpy()
    for p in range(nparts):
        ids = rtx.part_row_ids(H, tile_rows, p, nparts)
        assert_bits_equal(g[p, :len(ids)], full[ids], f"part {p} rows")
    gpu_ctx.deinterleave(gathered.ptr, W, H, tile_rows, nparts, image.ptr)
    assert_bits_equal(image.numpy(), full, f"{nparts} parts x {tile_rows}-row tiles")
    gathered.free()
    image.free()


def test_tiled_queue_whole_frame_equals_split(gpu_ctx, oracle, rtx):
    """The cost queue's orders: a whole 1920x1080 frame
    enumerates its queue in 16 x 16 pixel tiles with 64-slot private runs, a
    2-way share in tiles with runs of 16, an 8-way share row by row without
    runs. Every pixel's chain is its own, so all three must give the same
    image: the whole frame equals both split frames reassembled, bit for bit
    over every pixel (the frame's partial tiles at the bottom edge included),
    with equal segment counts, and rows of it equal the oracle's."""
    W, H, T = 1920, 1080, 5
    world = rtx.random_world(11, depth=50, spp=12)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    full, st = render_gpu(gpu_ctx, world, frame)
    for nparts in (2, 8):
        max_rows = rtx.part_rows(H, T, 0, nparts)
        gathered = gpu_ctx.alloc((nparts, max_rows, W, 4))
        image = gpu_ctx.alloc((H, W, 4))
        segs = 0
        for p in range(nparts):
            gpu_ctx.stats_reset()
            gpu_ctx.render_rows(T, p, nparts, gathered.ptr + p * max_rows * W * 16)
            segs += gpu_ctx.stats().segments
        gpu_ctx.deinterleave(gathered.ptr, W, H, T, nparts, image.ptr)
        assert_bits_equal(image.numpy(), full, f"whole frame vs {nparts} parts")
        assert segs == st.segments
        gathered.free()
        image.free()
    rows = np.array([0, 533, 1077, 1079], np.uint32)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(full[rows], want, "whole-frame rows")


@pytest.mark.parametrize("nparts,part", [(8, 3), (4, 0), (2, 1)])
def test_rank_share_of_c2_bit_exact(gpu_ctx, oracle, rtx, nparts, part):
    """One rank's share of the C2 frame (rtx_render_rows with R parts): a
    small share takes the heavy-pixel tiers (group-coop waves, k_heavy_split)
    and the hot-wave priority; its rows must still equal the oracle's."""
    W, H, T = 1920, 1080, 5
    world = rtx.random_world(11, depth=50, spp=100)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(frame)
    ids = rtx.part_row_ids(H, T, part, nparts)
    buf = gpu_ctx.alloc((len(ids), W, 4))
    gpu_ctx.stats_reset()
    gpu_ctx.render_rows(T, part, nparts, buf.ptr)
    st = gpu_ctx.stats()
    got = buf.numpy()
    buf.free()
    pick = np.linspace(0, len(ids) - 1, 6).astype(int)
    want, _ = oracle.render_rows(world, frame, ids[pick], nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(got[pick], want, f"part {part}/{nparts} rows")
    assert st.samples == len(ids) * W * 100


# ---------------------------------------------------------------------------
# §8f rows: thin lens (f-3) and progressive accumulation (f-2)
# ---------------------------------------------------------------------------
def test_thin_lens_bit_exact(gpu_ctx, oracle, rtx):
    """Defocus: lens offset from random_in_unit_disk (ShaderCompute.hlsl:50-57)
    applied as in Shader_RT.fx:288-298; bit-exact vs the oracle."""
    world = rtx.random_world(11, depth=50, spp=4)
    frame = rtx.set_aperture(rtx.camera_look_at(160, 90, aspect=160 / 90), 0.4)
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(90), nthreads=8)
    assert_bits_equal(img, want, "thin lens")
    assert st.segments == segs


@pytest.mark.parametrize("mode", ["chain", "per_sample_rng", "thin_lens", "frame_index", "lambert_guard"])
def test_scheduled_path_with_frame_options(gpu_ctx, oracle, rtx, mode):
    """spp >= 8 takes the cost pre-pass + ordered persistent render, which
    resumes every pixel after the pre-pass's sample 0 (acc, seed); each frame
    option must survive that hand-off bit for bit."""
    world = rtx.random_world(11, depth=50, spp=10)
    frame = rtx.camera_look_at(160, 90, aspect=160 / 90)
    if mode == "per_sample_rng":
        frame.rng_mode = 1
    elif mode == "thin_lens":
        frame = rtx.set_aperture(frame, 0.4)
    elif mode == "frame_index":
        frame.frame_index = 3
    elif mode == "lambert_guard":
        frame.flags = rtx.FRAME_LAMBERT_GUARD
    img, st = render_gpu(gpu_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(90), nthreads=8)
    assert_bits_equal(img, want, f"scheduled path, {mode}")
    assert st.segments == segs


def test_scheduled_path_edge_cases(gpu_ctx, oracle, rtx):
    """The scheduled path (spp >= 8) on tiny frames, an all-sky scene, depth
    1 and a ragged final tile of a split: pre-pass, heavy split, resume."""
    base = rtx.random_world(4, depth=6, spp=9)
    empty = rtx.World(np.zeros((0, 4), np.float32), np.zeros(0, np.float32), np.zeros((0, 4), np.float32), 5, 12)
    shallow = rtx.World(base.spheres, base.mat_types, base.mat_values, 1, 8)
    for world, w, h in [(base, 1, 1), (base, 3, 2), (empty, 17, 9), (shallow, 40, 23), (base, 65, 3)]:
        frame = rtx.camera_look_at(w, h, aspect=max(w / h, 0.1))
        img, st = render_gpu(gpu_ctx, world, frame)
        want, segs = oracle.render_rows(world, frame, np.arange(h))
        assert_bits_equal(img, want, f"scheduled edge n={world.count} {w}x{h} spp={world.spp}")
        assert st.segments == segs
    # a split whose last tile is ragged: 23 rows in 4-row tiles over 3 parts
    world, W, H, T, R = base, 40, 23, 4, 3
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(rtx.camera_look_at(W, H, aspect=W / H))
    buf = gpu_ctx.alloc((H, W, 4))
    for part in range(R):
        rows = rtx.part_row_ids(H, T, part, R)
        gpu_ctx.render_rows(T, part, R, buf.ptr)
        gpu_ctx.sync()
        got = buf.numpy().reshape(-1)[: len(rows) * W * 4].reshape(len(rows), W, 4)
        want, _ = oracle.render_rows(world, rtx.camera_look_at(W, H, aspect=W / H), rows)
        assert_bits_equal(got, want, f"ragged split part {part}")
    buf.free()


STRESS_LIB = os.path.join(os.path.dirname(GOLDEN), "..", "raytrace-we-gpu_amd", "lib", "variants",
                          "librtx_stress.so")


@pytest.fixture(scope="module")
def stress_ctx(rtx):
    """The stress build (make all): candidate lists of 1 entry and 2
    sphere-major pairs, so resolve rounds, list overflows and the exact
    sequential fallbacks run all the time."""
    if not os.path.exists(STRESS_LIB):
        pytest.skip("stress build missing: make all")
    ctx = rtx.Context(0, lib=rtx.load_library(STRESS_LIB))
    yield ctx
    ctx.close()


@pytest.mark.parametrize("nparts,part", [(1, 0), (2, 1), (4, 2), (8, 5)])
def test_overflow_and_fallback_paths_bit_exact(stress_ctx, oracle, rtx, nparts, part):
    """Every share size (lane mode, tiers 1 and 2, tail coop) with every
    overflow forced: the rows equal the oracle's bit for bit."""
    world = rtx.random_world(11, depth=50, spp=12)
    W, H, T = 320, 180, 5
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    stress_ctx.upload_world(world)
    stress_ctx.set_frame(frame)
    rows = rtx.part_row_ids(H, T, part, nparts)
    buf = stress_ctx.alloc((H, W, 4))
    stress_ctx.render_rows(T, part, nparts, buf.ptr)
    stress_ctx.sync()
    got = buf.numpy().reshape(-1)[: len(rows) * W * 4].reshape(len(rows), W, 4)
    buf.free()
    want, _ = oracle.render_rows(world, frame, rows, nthreads=8)
    assert_bits_equal(got, want, f"stress build, part {part} of {nparts}")


def test_per_sample_stress_build(stress_ctx, oracle, rtx):
    """k_render_ps with every candidate list overflowing (stress build)."""
    world = rtx.random_world(11, depth=50, spp=6)
    frame = rtx.camera_look_at(64, 36, aspect=64 / 36)
    frame.rng_mode = 1
    img, st = render_gpu(stress_ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(36), nthreads=8)
    assert_bits_equal(img, want, "per-sample, stress build")
    assert st.segments == segs


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
def test_double_buffered_scan_bit_exact(request, oracle, rtx, ctx_name):
    """Scenes above kScanPfMin (1024 padded spheres) take the kernels whose
    scan double-buffers each 8-sphere block in SGPRs (RTX_SCAN_PF): the
    scheduled path (pre-pass + persistent render, spp >= 8) and hit_world
    on random rays. With the stress build every candidate fills the list,
    so the scan leaves early after nearly every flagged block."""
    ctx = request.getfixturevalue(ctx_name)
    world = rtx.random_world(20, depth=50, spp=8)
    assert world.count > 1024
    frame = rtx.camera_look_at(96, 54, aspect=96 / 54)
    img, st = render_gpu(ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(54), nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img, want, f"{ctx_name}: {world.count} spheres")
    assert st.segments == segs
    rng = np.random.default_rng(11)
    o = np.concatenate([rng.uniform(-20, 20, (4000, 1)), rng.uniform(0.1, 6, (4000, 1)),
                        rng.uniform(-20, 20, (4000, 1))], 1)
    d = rng.normal(size=(4000, 3))
    d[:, 1] = -np.abs(d[:, 1]) * 0.3
    rays = np.concatenate([o, d], 1).astype(np.float32)
    got = ctx.debug_hit_world(rays)
    assert_bits_equal(got, oracle.hit_world_f32(world, rays), f"{ctx_name}: hit_world")


def test_scan_kernel_choice_boundary(gpu_ctx, oracle, rtx):
    """n = 1024 (plain scan) and 1025 (n_pad 1032: kPF scan) on the same
    rays, random spheres with duplicates (ties), small frames through the
    scheduled path: bit-exact on both sides of kScanPfMin."""
    rng = np.random.default_rng(5)
    for n in (1024, 1025):
        sph = np.concatenate([rng.uniform(-12, 12, (n, 1)), rng.uniform(-1, 3, (n, 1)),
                              rng.uniform(-12, 12, (n, 1)), rng.uniform(0.1, 0.6, (n, 1))], 1).astype(np.float32)
        sph[n - 1] = sph[3]
        mt = rng.integers(0, 3, n).astype(np.float32)
        mv = np.concatenate([rng.uniform(0.2, 1.0, (n, 3)), rng.uniform(1.2, 1.6, (n, 1))], 1).astype(np.float32)
        world = rtx.World(sph, mt, mv, 20, 8)
        gpu_ctx.upload_world(world)
        o = np.concatenate([rng.uniform(-14, 14, (3000, 1)), rng.uniform(0, 5, (3000, 1)),
                            rng.uniform(-14, 14, (3000, 1))], 1)
        d = rng.normal(size=(3000, 3))
        rays = np.concatenate([o, d], 1).astype(np.float32)
        assert_bits_equal(gpu_ctx.debug_hit_world(rays), oracle.hit_world_f32(world, rays), f"n={n} hit_world")
        frame = rtx.camera_look_at(64, 36, aspect=64 / 36)
        img, st = render_gpu(gpu_ctx, world, frame)
        want, segs = oracle.render_rows(world, frame, np.arange(36), nthreads=min(16, os.cpu_count() or 1))
        assert_bits_equal(img, want, f"n={n} frame")
        assert st.segments == segs


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
@pytest.mark.parametrize("ext", [11, 20])
def test_flat_block_runs_bit_exact(request, oracle, rtx, ctx_name, ext):
    """The scan's 6-op test on the scene's longest run of flat blocks (all 8
    centres at one height, rtx_prefilter.h line_test_q_flat) and the 7-op
    test elsewhere: a RTIOW scene broken into several runs — two blocks with
    mixed heights, one flat block at another height, a mixed last block —
    on both scan kernels (486 and 1,600 spheres) and the stress build (scan
    rounds that stop and resume inside and across runs)."""
    ctx = request.getfixturevalue(ctx_name)
    world = rtx.random_world(ext, depth=50, spp=8)
    s = world.spheres
    s[100:108, 1] = np.float32(0.35)  # blocks 12 and 13 become mixed
    s[200:208, 1] = np.float32(0.35)  # block 25: flat at another height
    s[-1, 1] = np.float32(0.5)        # the last block (padded with copies of n-1) mixed
    rng = np.random.default_rng(3)
    rays = np.concatenate([grazing_rays(s, 12000, rng, ext_frac=0.02),
                           np.concatenate([rng.uniform(-12, 12, (4000, 1)), rng.uniform(0.05, 3, (4000, 1)),
                                           rng.uniform(-12, 12, (4000, 1)), rng.normal(size=(4000, 3))], 1)
                           .astype(np.float32)])
    ctx.upload_world(world)
    assert_bits_equal(ctx.debug_hit_world(rays), oracle.hit_world_f32(world, rays), f"{ctx_name} n={world.count}")
    frame = rtx.camera_look_at(64, 36, aspect=64 / 36)
    img, st = render_gpu(ctx, world, frame)
    want, segs = oracle.render_rows(world, frame, np.arange(36), nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img, want, f"{ctx_name} n={world.count} frame")
    assert st.segments == segs


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
@pytest.mark.parametrize("coop", [24, 64])
def test_sphere_major_chunks_bit_exact(request, oracle, rtx, ctx_name, coop):
    """Queue exhausted: waves with up to `coop` pixels left trace them with
    the sphere-major group coop in chunks of 8 rays, two rays per packed test
    (rtx_set_schedule tail_coop_max). An 8-way share of a 320x180 frame
    (fewer pixels than lanes: every wave starts in the tail) and the whole
    frame, against the oracle; on the stress build every chunk overflows its
    pair list and takes the exact sequential path."""
    ctx = request.getfixturevalue(ctx_name)
    ctx.set_schedule(tail_coop_max=coop)
    assert ctx.get_schedule().tail_coop_max == coop
    world = rtx.random_world(11, depth=50, spp=10)
    W, H, T = 320, 180, 5
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    for nparts, part in ((8, 3), (1, 0)):
        rows = rtx.part_row_ids(H, T, part, nparts)
        buf = ctx.alloc((H, W, 4))
        ctx.render_rows(T, part, nparts, buf.ptr)
        ctx.sync()
        got = buf.numpy().reshape(-1)[: len(rows) * W * 4].reshape(len(rows), W, 4)
        buf.free()
        want, _ = oracle.render_rows(world, frame, rows, nthreads=8)
        assert_bits_equal(got, want, f"{ctx_name} coop={coop} part {part} of {nparts}")
    ctx.set_schedule()  # back to the defaults
    assert ctx.get_schedule().tail_coop_max == rtx.schedule_defaults().tail_coop_max


def test_schedule_validation_and_extremes(gpu_ctx, oracle, rtx):
    """rtx_set_schedule refuses out-of-range fields and keeps the previous
    schedule; extreme but valid schedules (every pixel of a small part in
    tier 1, no tiers, one wave in ten launched, tail coop of one ray) change
    only the time: the rows stay bit-exact."""
    d = rtx.schedule_defaults()
    for field, bad in (("tier1_bar", 0.0), ("tier2_bar_small", float("nan")), ("small_share", -1.0),
                       ("hot_fraction", 1.5), ("occupancy_low", 0.0), ("occupancy_normal", 1.01),
                       ("tail_coop_max", 0), ("tail_coop_max", 65), ("tail_coop_max_large", 0), ("tail_coop_max_large", 65), ("tier1_priority", 4), ("trace_group", 0), ("trace_group", 3), ("trace_group", 16), ("trace_solo_bar", 0.0), ("prepass_cap_split", 5000), ("trace_low", 0.6), ("trace_small", -0.1), ("promote_low", -1.0), ("promote_big_scene", -1.0), ("refill_chunk", 5000),
                       ("prio_bar1", -1.0), ("prio_bar1", 2.0), ("prio_bar2", 0.2), ("prio_bar3", float("nan")),
                       ("reserved", 1)):
        with pytest.raises(rtx.RtxError):
            gpu_ctx.set_schedule(**{field: bad})
        assert gpu_ctx.get_schedule().as_dict() == d.as_dict()
    world = rtx.random_world(11, depth=50, spp=9)
    W, H, T = 160, 90, 5
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(frame)
    extremes = [dict(tier1_bar=0.01, tier1_bar_small=0.01, tier1_bar_low=0.01),
                dict(tier1_bar=1e6, tier1_bar_small=1e6, tier1_bar_low=1e6, tier2_bar_small=1e6,
                     tier2_bar_medium=1e6),
                dict(occupancy_small=0.1, occupancy_low=0.1, occupancy_normal=0.1, hot_fraction=1.0),
                dict(tail_coop_max=1, hot_fraction=0.0),
                dict(tier1_priority=0, tier2_priority=1, hot_priority=2, tier2_bar=0.5),
                dict(trace_small=0.0, trace_low=0.0, trace_medium=0.0, trace_large=0.0, tier1_bar=0.01,
                     tier1_bar_small=0.01, tier1_bar_low=0.01),
                dict(trace_small=0.5, trace_low=0.5, trace_medium=0.5, trace_large=0.5, tier1_bar=0.01,
                     tier1_bar_small=0.01, tier1_bar_low=0.01),
                dict(trace_small=0.5, trace_low=0.5, trace_medium=0.5, trace_large=0.5, tier1_bar=0.01,
                     tier1_bar_small=0.01, tier1_bar_low=0.01, trace_group=4, trace_solo_bar=0.5),
                dict(prio_bar1=0.0),  # the static hot slots
                dict(prio_bar1=1e-3, prio_bar2=1e-3, prio_bar3=1e-3),  # every lane-mode wave at priority 3
                dict(prio_bar1=1e30, prio_bar2=1e30, prio_bar3=1e30)]  # ... at 0
    for ex in extremes:
        gpu_ctx.set_schedule()
        gpu_ctx.set_schedule(**ex)
        for nparts, part in ((1, 0), (4, 1)):
            rows = rtx.part_row_ids(H, T, part, nparts)
            buf = gpu_ctx.alloc((len(rows), W, 4))
            gpu_ctx.render_rows(T, part, nparts, buf.ptr)
            got = buf.numpy()
            buf.free()
            want, _ = oracle.render_rows(world, frame, rows, nthreads=8)
            assert_bits_equal(got, want, f"schedule {ex}, part {part} of {nparts}")
    gpu_ctx.set_schedule()


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
def test_trace_kernel_and_promotion_bit_exact(request, oracle, rtx, ctx_name):
    """Tier 1 in k_trace beside k_render, and promotion: once its queue is
    empty a lane hands its pixel to k_trace at a sample boundary (threshold 1
    projected segment: nearly every pixel still in flight is handed over,
    the 65,536-entry queue overflows on the whole frame and lanes keep the
    rest). k_trace with 1, 2, 4 and 8 pixels per wave (trace_group), the
    heaviest alone (trace_solo_bar). Whole frames and row-tile shares of
    every size class, against the oracle bit for bit, and the frame's
    segment count."""
    ctx = request.getfixturevalue(ctx_name)
    world = rtx.random_world(11, depth=50, spp=12)
    W, H, T = 320, 180, 5
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    want_all, segs_all = oracle.render_rows(world, frame, np.arange(H), nthreads=8)
    for sched in (dict(trace_small=0.3, trace_low=0.3, trace_medium=0.3, trace_large=0.3, tier1_bar=1.2,
                       tier1_bar_small=1.5, tier1_bar_low=1.5),
                  dict(trace_small=0.3, trace_low=0.3, trace_medium=0.3, trace_large=0.3, promote_small=1,
                       promote_low=1, promote_medium=1, promote_large=1),
                  dict(trace_small=0.05, trace_low=0.05, trace_medium=0.05, trace_large=0.05, promote_small=50,
                       promote_low=50, promote_medium=50, promote_large=50, tier1_bar=1.3),
                  # several tier-1 pixels per k_trace wave (groups of 32 / 16 / 4 lanes), the heaviest
                  # alone (trace_solo_bar), regrouping as tier 1 runs out, promotion served by groups
                  dict(trace_small=0.3, trace_low=0.3, trace_medium=0.3, trace_large=0.3, tier1_bar=1.2,
                       tier1_bar_small=1.2, tier1_bar_low=1.2, trace_group=2, trace_solo_bar=4.0),
                  dict(trace_small=0.1, trace_low=0.1, trace_medium=0.1, trace_large=0.1, tier1_bar=0.8,
                       tier1_bar_small=0.8, tier1_bar_low=0.8, trace_group=4, promote_small=20, promote_low=20,
                       promote_medium=20, promote_large=20),
                  dict(trace_small=0.05, trace_low=0.05, trace_medium=0.05, trace_large=0.05, tier1_bar=1.0,
                       tier1_bar_small=1.0, tier1_bar_low=1.0, trace_group=4, trace_solo_bar=2.5,
                       promote_small=1, promote_low=1, promote_medium=1, promote_large=1),
                  # groups of 8 lanes (8 pixels per wave), promotion served by them
                  dict(trace_small=0.2, trace_low=0.2, trace_medium=0.2, trace_large=0.2, tier1_bar=1.0,
                       tier1_bar_small=1.0, tier1_bar_low=1.0, trace_group=8, trace_solo_bar=3.0,
                       promote_small=30, promote_low=30, promote_medium=30, promote_large=30),
                  # a row-split share's pre-pass stops pixels past 6 segments: they restart from
                  # sample 0 in tier 1 (k_trace), their neighbours' keys count the cap
                  dict(trace_small=0.25, trace_low=0.2, trace_group=2, prepass_cap_split=6, promote_small=100,
                       promote_low=100)):
        ctx.set_schedule()
        ctx.set_schedule(**sched)
        for nparts, part in ((1, 0), (2, 1), (4, 3), (8, 2)):
            rows = rtx.part_row_ids(H, T, part, nparts)
            buf = ctx.alloc((len(rows), W, 4))
            ctx.stats_reset()
            ctx.render_rows(T, part, nparts, buf.ptr)
            st = ctx.stats()
            got = buf.numpy()
            buf.free()
            assert_bits_equal(got, want_all[rows], f"{ctx_name} {sched} part {part} of {nparts}")
            if nparts == 1:
                assert st.segments == segs_all
    ctx.set_schedule()


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
def test_promotion_across_the_chip(request, oracle, rtx, ctx_name):
    """Promotion with every workgroup of the chip taking part: a
    1280x720 frame (2.8 pixels per resident lane: a "medium" part) with
    promote_* 1 — nearly every pixel still in flight once the queue is empty
    is handed over, the 65,536-entry queue overflows — and k_trace beside the
    render (trace_* 0.3, the combination whose exit used to depend on both
    kernels running together). Entries cross XCDs (the queue is one array;
    producers and servers sit on all 8). The launch must complete (no
    RTX_ERR_INCOMPLETE from rtx_get_stats), rows bit-exact, and the segment
    count equal to an independent exact-grid pass's. Through the stress build
    the promotion valve is 20 ms: the launch completes only if
    the tracing waves' heartbeat counts as progress while no pixel finishes
    (a 2 ms valve fired here in R7e while only full waves, which had not
    seen the queue exhausted and did not beat yet, were tracing; a 20 ms one
    fired once in R8x, profiles/R8x_gtest_valve_fire.log: since round 6 the
    valve's clock runs only while the server itself runs, the entry wait has
    its own clock and bit, and a firing reports what the server saw)."""
    gpu_ctx = request.getfixturevalue(ctx_name)
    W, H, T = 1280, 720, 5
    world = rtx.random_world(11, depth=50, spp=12)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(frame)
    rows = np.linspace(2, H - 3, 6).astype(np.uint32)
    want, segs_rows = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    cost = gpu_ctx.debug_pixel_cost(0)
    assert int(cost[rows].sum(dtype=np.uint64)) == segs_rows
    for sched in (dict(promote_small=1, promote_low=1, promote_medium=1, promote_large=1),
                  dict(promote_small=1, promote_low=1, promote_medium=1, promote_large=1, trace_small=0.3,
                       trace_low=0.3, trace_medium=0.3, trace_large=0.3, tier1_bar=1.2, tier1_bar_small=1.5,
                       tier1_bar_low=1.5)):
        gpu_ctx.set_schedule()
        gpu_ctx.set_schedule(**sched)
        for nparts, part in ((1, 0), (2, 1)):
            ids = rtx.part_row_ids(H, T, part, nparts)
            buf = gpu_ctx.alloc((len(ids), W, 4))
            gpu_ctx.stats_reset()
            gpu_ctx.render_rows(T, part, nparts, buf.ptr)
            st = gpu_ctx.stats()  # raises RtxError (RTX_ERR_INCOMPLETE) if pixels were left unwritten
            got = buf.numpy()
            buf.free()
            assert st.segments == int(cost[ids].sum(dtype=np.uint64)), f"{sched} part {part} of {nparts}"
            mine = np.isin(rows, ids)
            pos = np.searchsorted(ids, rows[mine])
            assert_bits_equal(got[pos], want[mine], f"{sched} part {part} of {nparts}")
    gpu_ctx.set_schedule()


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
def test_promotion_large_scene_bit_exact(request, oracle, rtx, ctx_name):
    """Promotion in the large-scene (kPF) kernels, where the promoted pixel's
    whole-wave trace reads the scene from `pre`/`cen` in HBM and the lane-mode
    scan streams it through the per-wave LDS tile: 1,600 spheres (grid 20),
    promote_big_scene 1 (nearly every pixel in flight once the queue is empty
    is handed over; the queue overflows and lanes keep the rest) and the
    default 60, whole frame and a 4-way share, bit for bit against the oracle,
    and the frame's segment count."""
    ctx = request.getfixturevalue(ctx_name)
    world = rtx.random_world(20, depth=50, spp=6)
    assert world.count > 1024  # the kPF kernels
    W, H, T = 192, 108, 3
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    want_all, segs_all = oracle.render_rows(world, frame, np.arange(H), nthreads=8)
    for thr in (1.0, 60.0):
        ctx.set_schedule()
        ctx.set_schedule(promote_big_scene=thr, medium_share=0.01, low_share=0.005, small_share=0.001)
        for nparts, part in ((1, 0), (4, 1)):
            rows = rtx.part_row_ids(H, T, part, nparts)
            buf = ctx.alloc((len(rows), W, 4))
            ctx.stats_reset()
            ctx.render_rows(T, part, nparts, buf.ptr)
            st = ctx.stats()
            got = buf.numpy()
            buf.free()
            assert_bits_equal(got, want_all[rows], f"{ctx_name} promote {thr} part {part} of {nparts}")
            if nparts == 1:
                assert st.segments == segs_all
    ctx.set_schedule()


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
def test_refill_chunk_bit_exact(request, oracle, rtx, ctx_name):
    """Private queue runs per wave (rtx_schedule.refill_chunk): with the share
    classes moved down (medium_share 0.01) a 320x180 frame and its row shares
    count as "large" parts, so every refill takes slots from the wave's run —
    runs of 1 (off), 3, 16 and 500 slots (the last larger than the part, so
    the last-eighth rule and the queue's end are crossed inside one run).
    Bit for bit against the oracle, and the whole frame's segment count."""
    ctx = request.getfixturevalue(ctx_name)
    world = rtx.random_world(11, depth=50, spp=12)
    W, H, T = 320, 180, 5
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    want_all, segs_all = oracle.render_rows(world, frame, np.arange(H), nthreads=8)
    for chunk in (0, 3, 16, 500):
        ctx.set_schedule()
        ctx.set_schedule(medium_share=0.01, low_share=0.005, small_share=0.001, refill_chunk=chunk)
        for nparts, part in ((1, 0), (2, 1), (8, 5)):
            rows = rtx.part_row_ids(H, T, part, nparts)
            buf = ctx.alloc((len(rows), W, 4))
            ctx.stats_reset()
            ctx.render_rows(T, part, nparts, buf.ptr)
            st = ctx.stats()
            got = buf.numpy()
            buf.free()
            assert_bits_equal(got, want_all[rows], f"{ctx_name} chunk {chunk} part {part} of {nparts}")
            if nparts == 1:
                assert st.segments == segs_all
    ctx.set_schedule()


def test_progressive_accumulation_bit_exact(gpu_ctx, oracle, rtx):
    """rtx_accumulate: frame k uses frame_index k; the linear sums add up in
    fp32 frame by frame; the framebuffer is toGamma(sum / (k * spp))."""
    W, H, spp = 64, 36, 2
    world = rtx.random_world(11, depth=20, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(frame)
    total = np.zeros((H, W, 4), np.float32)
    for k in range(3):
        assert gpu_ctx.accumulate(reset=(k == 0)) == k + 1
        f = rtx.camera_look_at(W, H, aspect=W / H)
        f.frame_index = k
        lin, _ = oracle.render_rows_linear(world, f, np.arange(H), nthreads=8)
        total[..., :3] = total[..., :3] + lin[..., :3]
        mean = (total[..., :3] / np.float32((k + 1) * spp)).astype(np.float32)
        want = np.ones((H, W, 4), np.float32)
        want[..., :3] = oracle.math("pow", mean.ravel(), np.full(mean.size, 0.454545454545, np.float32)).reshape(mean.shape)
        assert_bits_equal(gpu_ctx.download(), want, f"accumulated frame {k + 1}")
    # frame 1 of the accumulation is the plain reference frame
    assert gpu_ctx.accumulate(reset=True) == 1
    plain, _ = render_gpu(gpu_ctx, world, frame)
    gpu_ctx.set_frame(frame)
    gpu_ctx.accumulate(reset=True)
    assert_bits_equal(gpu_ctx.download(), plain, "1-frame accumulation == plain frame")


def test_accumulate_after_resize(gpu_ctx, oracle, rtx):
    """Accumulate at one size, set a larger frame, render it (the framebuffer
    grows), then accumulate again: the accumulator restarts at the new size
    (it is sized by its own pixel count, not the framebuffer's)."""
    world = rtx.random_world(11, depth=20, spp=2)
    gpu_ctx.upload_world(world)
    small = rtx.camera_look_at(32, 18, aspect=32 / 18)
    gpu_ctx.set_frame(small)
    assert gpu_ctx.accumulate(reset=True) == 1
    assert gpu_ctx.accumulate() == 2
    big = rtx.camera_look_at(96, 54, aspect=96 / 54)
    gpu_ctx.set_frame(big)
    gpu_ctx.render()
    assert gpu_ctx.accumulate() == 1  # restarted: a new size
    want, _ = oracle.render_rows(world, big, np.arange(54), nthreads=8)
    assert_bits_equal(gpu_ctx.download(), want, "first accumulated frame after a resize")


def test_frame_gather_on_torch_default_stream():
    """The multi-GPU frame assembly with torch tensors on torch's default
    (null) stream: librtx launches there (rtx_set_stream(NULL)), so torch's
    buffer fills, the renders, the copies and the de-interleave are ordered;
    the image equals the own-stream render bit for bit (child process:
    torch must load before librtx)."""
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "torch_stream_check.py")
    out = subprocess.run([sys.executable, script], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout[-2000:] + out.stderr[-2000:]


def test_cli_writes_reference_frame(tmp_path, oracle, rtx):
    """rtx_cli (the headless DxCSApp driver) renders the frame the oracle renders;
    its PFM stores rows bottom-to-top like the framebuffer, its PPM the 8-bit
    image top row first."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "raytrace-we-gpu_amd", "bin", "rtx_cli")
    pfm, ppm = str(tmp_path / "f.pfm"), str(tmp_path / "f.ppm")
    out = subprocess.run([cli, "--width", "64", "--height", "36", "--spp", "3", "--depth", "50",
                          "--scene", "rtiow11", "--frames", "1", "--pfm", pfm, "--ppm", ppm],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    with open(pfm, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        assert float(f.readline()) < 0  # little endian
        img = np.frombuffer(f.read(), "<f4").reshape(h, w, 3)
    world = rtx.random_world(11, depth=50, spp=3)
    frame = rtx.camera_look_at(64, 36, aspect=64 / 36)
    want, _ = oracle.render_rows(world, frame, np.arange(36), nthreads=4)
    assert_bits_equal(img, want[..., :3], "rtx_cli PFM")
    with open(ppm, "rb") as f:  # 8-bit, top row first, clamped, x 255.999 (Color.h:6-11)
        assert f.readline().strip() == b"P6" and f.readline().split() == [b"64", b"36"]
        assert f.readline().strip() == b"255"
        img8 = np.frombuffer(f.read(), np.uint8).reshape(36, 64, 3)
    v = np.nan_to_num(want[::-1, :, :3], nan=0.0)
    np.testing.assert_array_equal(img8, (np.float32(255.999) * np.clip(v, 0, 1).astype(np.float32)).astype(np.uint8))


def test_reference_frame_through_cbuffer_bytes(tmp_path, oracle, rtx):
    """The drop-in on the reference's own bytes: rtx_cli
    --reference-frame fills WorldDef (18,448 B) and PerFrame (112 B) as
    DxCSApp does (DxCSApp.cpp:39-61, 72-134, 481-496), hands them to
    rtx_world_from_worlddef / rtx_frame_from_perframe, and renders the frame
    as shipped: 1024x576, spp 60, depth 50, 326 spheres (:133, :179,
    :330-331, Dispatch :524). Eight full rows bit-exact against the oracle's
    render of the same scene and camera."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "raytrace-we-gpu_amd", "bin", "rtx_cli")
    pfm = str(tmp_path / "ref.pfm")
    out = subprocess.run([cli, "--reference-frame", "--frames", "1", "--pfm", pfm],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rep = __import__("json").loads(out.stdout.strip().splitlines()[-1])
    assert (rep["width"], rep["height"], rep["spp"], rep["depth"], rep["spheres"], rep["cbuffers"]) == \
        (1024, 576, 60, 50, 326, True)
    with open(pfm, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        assert (w, h) == (1024, 576) and float(f.readline()) < 0
        img = np.frombuffer(f.read(), "<f4").reshape(h, w, 3)
    world = rtx.random_world(9, depth=50, spp=60)
    frame = rtx.camera_look_at(1024, 576, aspect=16.0 / 9.0)
    rows = np.linspace(3, 572, 8).astype(np.uint32)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    assert_bits_equal(img[rows], want[..., :3], "reference frame rows")
    assert np.isfinite(img).all()


def test_upload_rejects_out_of_range_scene(gpu_ctx, rtx):
    """Scene values must be finite with |v| <= 1e15 (the all-miss test's
    exactness bound, rtx_api.hip); the context stays usable afterwards."""
    w = rtx.random_world(2, depth=4, spp=1)
    bad = rtx.World(w.spheres.copy(), w.mat_types, w.mat_values, 4, 1)
    bad.spheres[3, 0] = np.inf
    with pytest.raises(rtx.RtxError, match="1e15"):
        gpu_ctx.upload_world(bad)
    bad.spheres[3, 0] = 2e15
    with pytest.raises(rtx.RtxError):
        gpu_ctx.upload_world(bad)
    gpu_ctx.upload_world(w)


def test_debug_scan_rate_probe(gpu_ctx, rtx):
    """rtx_debug_scan_rate (the bench's issue-ceiling probe) runs the render's
    hit_world at full occupancy and reports waves x reps; scenes beyond the
    render's LDS copy (> 640 spheres) are refused, not run."""
    W, H = 320, 180
    world = rtx.random_world(11, depth=50, spp=16)
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    gpu_ctx.upload_world(world)
    gpu_ctx.set_frame(frame)
    ms1, ws1 = gpu_ctx.debug_scan_rate(4)
    ms2, ws2 = gpu_ctx.debug_scan_rate(8)
    assert ms1 > 0.0 and ms2 > 0.0
    assert ws1 > 0 and ws2 == 2 * ws1 and ws1 % 4 == 0
    big = rtx.random_world(20, depth=50, spp=16)  # 1,600 spheres
    gpu_ctx.upload_world(big)
    with pytest.raises(rtx.RtxError):
        gpu_ctx.debug_scan_rate(1)


@pytest.mark.parametrize("ctx_name", ["gpu_ctx", "stress_ctx"])
@pytest.mark.parametrize("grid,spp", [(11, 12), (20, 6)])
def test_scan_modes_bit_exact(request, oracle, rtx, ctx_name, grid, spp):
    """rtx_set_scan_mode: the same frame through the default search (the layer
    grid at 486 spheres, the culled scan at 1,600) and through the linear
    scan (every block of every segment, the reference's Hittable_list order
    of work; the large scene streams it through the per-wave LDS tile):
    both bit for bit against the oracle, with equal segment counts, whole
    frame and a 3-way share. The context goes back to the default mode."""
    ctx = request.getfixturevalue(ctx_name)
    world = rtx.random_world(grid, depth=50, spp=spp)
    W, H, T = 256, 144, 4
    frame = rtx.camera_look_at(W, H, aspect=W / H)
    rows = np.linspace(1, H - 2, 6).astype(np.uint32)
    want, _ = oracle.render_rows(world, frame, rows, nthreads=min(16, os.cpu_count() or 1))
    try:
        for mode in ("linear", "auto"):
            ctx.set_scan_mode(mode)
            ctx.upload_world(world)
            ctx.set_frame(frame)
            ctx.stats_reset()
            img = ctx.render_image()
            segs = ctx.stats().segments
            assert_bits_equal(img[rows], want, f"{ctx_name} grid {grid} {mode}")
            if mode == "linear":
                ref_img, ref_segs = img, segs
            else:
                assert segs == ref_segs
                assert_bits_equal(img, ref_img, f"{ctx_name} grid {grid}: auto vs linear")
            ids = rtx.part_row_ids(H, T, 1, 3)
            buf = ctx.alloc((len(ids), W, 4))
            ctx.render_rows(T, 1, 3, buf.ptr)
            got = buf.numpy()
            buf.free()
            assert_bits_equal(got, ref_img[ids], f"{ctx_name} grid {grid} {mode}: share 1 of 3")
    finally:
        ctx.set_scan_mode("auto")
