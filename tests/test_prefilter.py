"""The scan prefilter's exactness claim, checked on the CPU.

raytrace-we-gpu_amd/csrc/rtx_prefilter.h replaces the reference's per-sphere
discriminant test (ShaderCompute.hlsl:158-166) in the kernel's scan by a
cheaper, inflated line-distance test, and resolves every flagged sphere with
the reference's own operations. The result is bit-identical only if the
prefilter flags every sphere whose reference fp32 discriminant is >= 0 (or
NaN). tests/prefilter_check.cpp evaluates both, with the header's own code,
on adversarial near-tangent cases and must find no miss; likewise for the
culled scan's block bounds (a block is skipped only if no lane's line passes
its bound, or its bound is wholly behind every lane's origin). The GPU side of the same claims is
test_gpu_parity.py::test_hit_world_grazing_rays (both scans).
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "prefilter_check.cpp")


def test_prefilter_never_drops_a_reference_candidate(tmp_path):
    exe = str(tmp_path / "prefilter_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-o", exe, SRC], check=True)
    out = subprocess.run([exe, "4000000"], capture_output=True, text=True, timeout=120)
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and rep["missed"] == 0, out.stderr
    assert rep["reference_candidates"] > 1_000_000  # the near-tangent set is exercised
    # the rounding errors use a small share of the margin (rigorous bound: <= 0.38)
    assert rep["max_margin_used"] < 0.38, rep
    # the culled scan's block bounds (rtx_prefilter.h cull_bound): no reference
    # candidate's block is skipped; the tightest lines use the geometric part
    # of R_b, 1 / (1 + k) = 0.97 of it, never the rounding margins
    assert rep["block_missed"] == 0 and rep["block_reference_candidates"] > 500_000, rep
    assert rep["block_max_used"] < 0.98, rep
    # the half-space part (rtx_prefilter.h HalfTest): no sphere the reference
    # accepts (a root >= t_min) is behind a failed half test; the rays that
    # leave a sphere straight away from its bound reach 1 / (1 + k) of K, and
    # the test does cull reference candidates whose roots are behind
    assert rep["half_missed"] == 0 and rep["block_reference_accepted"] > 300_000, rep
    assert 0.9 < rep["half_max_used"] < 0.98, rep
    assert rep["half_culled"] > 100_000, rep
    # the same test per sphere (RTX_CULL_HALF_SPHERES, an option: measured
    # slower), on the single-sphere cases, a fifth of them starting on the sphere
    assert rep["sphere_half_missed"] == 0 and rep["sphere_reference_accepted"] > 500_000, rep
    assert rep["sphere_half_max_used"] < 1.0 and rep["sphere_half_culled"] > 100_000, rep


GRID_SRC = os.path.join(ROOT, "tests", "grid_check.cpp")


def _build_grid_check(tmp_path, header_dir):
    exe = str(tmp_path / "grid_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-I", header_dir, "-o", exe, GRID_SRC],
                   check=True)
    return exe


def test_layer_grid_never_skips_an_accepted_sphere(tmp_path):
    """The layer grid (rtx_grid.h): a block of the flat run is left out of a
    wave's scan only if no lane's walk marks it; tests/grid_check.cpp checks,
    on RTIOW and random layers and adversarial rays (near-tangent at every
    slope down to grazing the layer, through cell corners, along the axes,
    leaving a sphere's surface), that every sphere the reference accepts is
    in a marked block. The checker itself must catch a grid built without
    the margins (rho = r, no fattening)."""
    exe = _build_grid_check(tmp_path, ROOT)
    out = subprocess.run([exe, "300", "4000"], capture_output=True, text=True, timeout=120)
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and rep["missed"] == 0, out.stderr
    assert rep["accepted_spheres"] > 3_000_000 and rep["grid_applied"] > 900_000, rep
    assert rep["every_block"] < 0.01 * rep["grid_applied"], rep  # the walk rarely gives up
    # the far cut (the walk stops far_m / |d| past the best root so far: the
    # winner's own root, ties included)
    assert rep["far_missed"] == 0 and rep["far_checked"] > 500_000, rep
    # sensitivity: the same checker over a grid without the margins misses
    bad = tmp_path / "bad" / "raytrace-we-gpu_amd" / "csrc"
    bad.mkdir(parents=True)
    src = open(os.path.join(ROOT, "raytrace-we-gpu_amd", "csrc", "rtx_grid.h")).read()
    src = src.replace("constexpr double kGridFatCells = 1.0 / 256.0;", "constexpr double kGridFatCells = 0.0;")
    src = src.replace(" + 27.0 * u * c2 + B) * (1.0 + 4.0 * u) * (1.0 + 1e-12)", ") * (1.0 - 1e-7)")
    assert src.count("(1.0 - 1e-7)") == 1
    (bad / "rtx_grid.h").write_text(src)
    (bad / "rtx_prefilter.h").write_text(open(os.path.join(ROOT, "raytrace-we-gpu_amd", "csrc",
                                                           "rtx_prefilter.h")).read())
    btests = tmp_path / "bad" / "tests"
    btests.mkdir()
    (btests / "grid_check.cpp").write_text(open(GRID_SRC).read())
    bexe = str(tmp_path / "grid_check_bad")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-o", bexe, str(btests / "grid_check.cpp")],
                   check=True)
    bout = subprocess.run([bexe, "300", "4000"], capture_output=True, text=True, timeout=120)
    assert bout.returncode == 1 and json.loads(bout.stdout.strip().splitlines()[-1])["missed"] > 0
