"""CPU check of the oracle's mesh area emitter (no GPU): Mesh::sample_position (mesh.cpp:765-816)
against the same flat box emitting as six rectangles (rectangle.cpp:164-178).  Both are unbiased
estimators of one image, so the per-view mean radiance must agree within noise.  The GPU is pinned
to this oracle bit for bit by tests/test_gpu_parity.py::test_mesh_area_emitters."""
import os

import numpy as np

from conftest import SCENES

SEEDS = 6


def _view_means(amvpt_mod, oracle, name, seed0):
    out = []
    for seed in range(seed0, seed0 + SEEDS):
        s = amvpt_mod.load_file(os.path.join(SCENES, name), res=16, spp=32)
        sd, vd, p = s.describe(0, seed, 0)
        film, _, _ = oracle.render(sd, vd, p, threads=8)
        rgb = film[..., :3] / np.maximum(film[..., 3:4], 1e-20)
        out.append([rgb[y:y + 16, x:x + 16].mean() for y in (0, 16) for x in (0, 16)])
    return np.array(out)


def test_oracle_mesh_light_matches_rectangle_lights(amvpt_mod, oracle):
    a = _view_means(amvpt_mod, oracle, "cbox_meshlight.xml", 0)
    b = _view_means(amvpt_mod, oracle, "cbox_cubelight_rects.xml", 100)
    z = np.abs(a.mean(0) - b.mean(0)) / np.sqrt(a.var(0, ddof=1) / SEEDS + b.var(0, ddof=1) / SEEDS)
    print("per-view means", a.mean(0), b.mean(0), "z", z)
    assert np.isfinite(a).all() and np.isfinite(b).all()
    assert z.max() < 4.5, z
