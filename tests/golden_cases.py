"""Golden hit_world fixtures produced by the reference's compiled CPU library
(tests/golden/make_golden.py): one loader for the CPU and GPU tests.

Each case: spheres (float32, as the producers make them), rays (float64,
float32-representable), t_min, t_max, the reference's records, and whether
ill-conditioned rays may disagree with fp64 (tests/tolerance.py)."""
import json
import os

import numpy as np

from cases import scene_digest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
JSON_FIXTURES = ("hit_test_world.json", "hit_rtiow9.json")
NPZ_FIXTURES = ("hit_rtiow11.npz", "hit_grazing11.npz", "hit_c5_100k.npz")


def case_ids():
    ids = []
    for name in JSON_FIXTURES:
        d = json.load(open(os.path.join(GOLDEN, name)))
        ids += [(name, k) for k in range(len(d["cases"]))]
    return ids + [(name, 0) for name in NPZ_FIXTURES]


def load_case(name, k, random_world):
    """`random_world(ext, capacity)` -> spheres [n, 4] float32 (the oracle's or
    librtx's producer) rebuilds scenes that fixtures name by digest."""
    path = os.path.join(GOLDEN, name)
    if name.endswith(".json"):
        d = json.load(open(path))
        c = d["cases"][k]
        return dict(spheres=np.array(d["spheres"], np.float32), rays=np.array(d["rays"], np.float64),
                    t_min=c["t_min"], t_max=np.inf if c["t_max"] is None else c["t_max"],
                    expected=np.array(c["expected"], np.float64), allow_ill=False)
    z = np.load(path, allow_pickle=False)
    if "spheres" in z.files:
        sph = z["spheres"].astype(np.float32)
    else:
        sph = np.asarray(random_world(int(z["grid"]), int(z["count"])), np.float32)
        if scene_digest(sph) != bytes(z["digest"]).hex():
            raise AssertionError(f"{name}: scene producer no longer reproduces the fixture's scene")
    return dict(spheres=sph, rays=z["rays"], t_min=float(z["t_min"]), t_max=np.inf, expected=z["expected"],
                allow_ill=name == "hit_grazing11.npz")
