#!/usr/bin/env python3
"""Regenerate the golden vectors in tests/golden/ from the REFERENCE's own
CPU geometry library.

oracle/_ref/ref_golden is built by oracle/Makefile from
/root/reference/{Sphere,Hittable_list,Camera}.cpp (compiled in place) plus
our driver oracle/ref_golden.cpp. This script feeds it deterministic,
fp32-representable inputs and stores inputs + the reference's outputs as
JSON. Only this build container has /root/reference; the GPU box and the
CPU test suite read the committed JSON.

    python3 tests/golden/make_golden.py        (after `make -C oracle`)

Fixtures (all doubles exact; t_max null = +inf):
  camera_simple_400x225.json  Camera(400,225).get_ray(u,v)      (Camera.h:23-26)
  hit_test_world.json         Hittable_list::hit over test_world (Hittable_list.cpp:3-20)
  hit_rtiow9.json             Hittable_list::hit over random_world(9), 326 spheres
  hit_rtiow11.npz             ... over random_world(11), 486 spheres (the bench scene, C2/C3):
                              camera rays + secondary rays + grazing rays (tests/cases.py)
  hit_c5_100k.npz             ... over random_world(159) truncated to 100,000 spheres (C5): camera
                              and secondary rays; the scene is named by generator + sha256 digest
                              (tests/cases.py scene_digest), not stored
npz fixtures hold float64 arrays only (np.load(..., allow_pickle=False)).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as orc  # noqa: E402
from cases import camera_rays, grazing_rays, scene_digest  # noqa: E402


def fmt(x: float) -> str:
    return "%.17g" % x


def run_ref(spheres, rays, t_min, t_max, cam_wh=(1, 1), uv=np.zeros((0, 2))):
    lines = [str(len(spheres))]
    lines += [" ".join(fmt(v) for v in s) for s in spheres]
    lines.append("%d %s %s" % (len(rays), fmt(t_min), "inf" if t_max is None else fmt(t_max)))
    lines += [" ".join(fmt(v) for v in r) for r in rays]
    lines.append("%d %d %d" % (len(uv), cam_wh[0], cam_wh[1]))
    lines += [" ".join(fmt(v) for v in p) for p in uv]
    out = orc.run_ref_golden("\n".join(lines) + "\n").split("\n")
    hits = [[float(v) for v in out[i].split()] for i in range(len(rays))]
    cams = [[float(v) for v in out[len(rays) + i].split()] for i in range(len(uv))]
    return hits, cams


def f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


def random_rays(rng, n, lo, hi, normalize):
    o = rng.uniform(lo, hi, size=(n, 3))
    d = rng.normal(size=(n, 3))
    if normalize:
        d /= np.linalg.norm(d, axis=1, keepdims=True)
    else:
        d *= rng.uniform(0.5, 3.0, size=(n, 1))
    return f32(np.concatenate([o, d], axis=1))


def main():
    rng = np.random.default_rng(20251015)
    os.makedirs(HERE, exist_ok=True)

    # 1. Camera.h rays (u, v on a grid + random).
    uu, vv = np.meshgrid(np.linspace(0, 1, 9), np.linspace(0, 1, 7))
    uv = np.concatenate([np.stack([uu.ravel(), vv.ravel()], 1), rng.uniform(0, 1, (40, 2))])
    uv = f32(uv)
    _, cams = run_ref([], [], 0.001, None, (400, 225), uv)
    json.dump({"source": "Camera(400,225).get_ray(u,v), Camera.h:9-26 (compiled reference)",
               "width": 400, "height": 225, "uv": uv.tolist(), "rays": cams},
              open(os.path.join(HERE, "camera_simple_400x225.json"), "w"))

    # 2. test_world: primary rays of Camera(400,225) + random rays.
    sph, _, _ = orc.test_world()
    sph = f32(sph)
    cam_rays = f32(cams)  # fp32-representable copies of the camera rays
    rays = np.concatenate([cam_rays, random_rays(rng, 200, [-2, -0.6, -3], [2, 1.5, 1], True),
                           random_rays(rng, 60, [-2, -0.6, -3], [2, 1.5, 1], False)])
    blocks = []
    for t_min, t_max in [(0.001, None), (0.001, 1.5), (0.5, None)]:
        hits, _ = run_ref(sph.tolist(), rays.tolist(), t_min, t_max)
        blocks.append({"t_min": t_min, "t_max": t_max, "expected": hits})
    json.dump({"source": "Hittable_list::hit + Sphere::hit (compiled reference); scene = "
                         "WorldDef::test_world (DxCSApp.cpp:136-157)",
               "spheres": sph.tolist(), "rays": rays.tolist(), "cases": blocks},
              open(os.path.join(HERE, "hit_test_world.json"), "w"))

    # 3. random_world(9): DxCSApp camera rays + secondary rays from the ground.
    sph9, _, _ = orc.random_world(9)
    sph9 = f32(sph9)
    fr = orc.camera_look_at(1920, 1080)
    org = np.array(fr.origin[:3], np.float64)
    hor, ver, llc = (np.array(v[:3], np.float64) for v in (fr.horizontal, fr.vertical, fr.lower_left))
    st = rng.uniform(0, 1, (250, 2))
    d = llc + st[:, :1] * hor + st[:, 1:] * ver - org
    prim = f32(np.concatenate([np.repeat(org[None], 250, 0), d], 1))
    sec = random_rays(rng, 250, [-11, 0.0, -11], [11, 1.2, 11], True)
    rays9 = np.concatenate([prim, sec])
    hits, _ = run_ref(sph9.tolist(), rays9.tolist(), 0.001, None)
    json.dump({"source": "Hittable_list::hit + Sphere::hit (compiled reference); scene = "
                         "WorldDef::random_world grid -9..9 (DxCSApp.cpp:72-134), 326 spheres",
               "spheres": sph9.tolist(), "rays": rays9.tolist(),
               "cases": [{"t_min": 0.001, "t_max": None, "expected": hits}]},
              open(os.path.join(HERE, "hit_rtiow9.json"), "w"))

    # 4. random_world(11) (486 spheres): primary + secondary + grazing rays.
    sph11, _, _ = orc.random_world(11)
    rng11 = np.random.default_rng(486)
    fr = orc.camera_look_at(1920, 1080)
    prim = camera_rays(fr, 300, rng11)
    sec = random_rays(rng11, 300, [-13, 0.0, -13], [13, 1.5, 13], True)
    graz = grazing_rays(sph11, 2000, rng11, ext_frac=0.0).astype(np.float64)
    sph11 = f32(sph11)
    for name, rays in (("hit_rtiow11.npz", np.concatenate([prim, sec])), ("hit_grazing11.npz", graz)):
        hits, _ = run_ref(sph11.tolist(), rays.tolist(), 0.001, None)
        np.savez_compressed(os.path.join(HERE, name), spheres=sph11, rays=rays,
                            expected=np.array(hits, np.float64), t_min=np.float64(0.001))

    # 5. the C5 scene: random_world(159) truncated to 100,000 spheres.
    sph5, _, _ = orc.random_world(159, 100000)
    rng5 = np.random.default_rng(100000)
    prim5 = camera_rays(fr, 200, rng5)
    sec5 = random_rays(rng5, 200, [-30, 0.0, -30], [30, 1.5, 30], True)
    rays5 = np.concatenate([prim5, sec5])
    hits, _ = run_ref(f32(sph5).tolist(), rays5.tolist(), 0.001, None)
    np.savez_compressed(os.path.join(HERE, "hit_c5_100k.npz"), rays=rays5, expected=np.array(hits, np.float64),
                        t_min=np.float64(0.001), grid=np.float64(159), count=np.float64(len(sph5)),
                        digest=np.frombuffer(bytes.fromhex(scene_digest(sph5)), np.uint8))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
