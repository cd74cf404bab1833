"""Pin the CPU oracle to the reference's own known-answer data (CPU only).

Golden values come from tests/golden/reference_kats.json (extracted from the
reference's tests by tests/golden/make_golden.py) and from the published
PCG32 reference output (pcg32 is Dr.Jit's, an un-vendored submodule of the
reference: drjit/include/drjit/random.h, O'Neill's pcg32 "pcg32-demo" stream).
Each test names the reference test it mirrors.
"""
import ctypes
import json
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_kats.json")


@pytest.fixture(scope="module")
def kats():
    with open(GOLDEN) as f:
        return json.load(f)


def _vec(L, fn, *args, n=3):
    out = (ctypes.c_float * n)()
    getattr(L, fn)(*args, out)
    return np.array(out[:], dtype=np.float32)


# ---------------------------------------------------------------- random numbers

def test_tea_float32_golden(oracle, kats):
    """src/core/tests/test_random.py:test01_tea_float32 (exact equality, as the reference asserts)."""
    L = oracle.lib()
    for c in kats["sample_tea_float32"]["cases"]:
        got = L.oracle_tea_float32(c["v0"], c["v1"], c["rounds"])
        assert np.float32(got) == np.float32(c["expected"]), c


def test_tea_float64_golden(oracle, kats):
    """src/core/tests/test_random.py:test02_tea_float64."""
    L = oracle.lib()
    for c in kats["sample_tea_float64"]["cases"]:
        assert L.oracle_tea_float64(c["v0"], c["v1"], c["rounds"]) == c["expected"], c


def test_pcg32_published_stream(oracle):
    """PCG32 (Dr.Jit PCG32::seed(initstate=42, initseq=54)) against the published pcg32-demo output."""
    out = (ctypes.c_uint32 * 6)()
    oracle.lib().oracle_pcg32_u32(42, 54, 6, out)
    assert list(out) == [0xa15c02b7, 0x7b47f409, 0xba1d3330, 0x83d2f293, 0xbfa4784b, 0xcbed606e]


def test_independent_sampler_is_tea_seeded_pcg32(oracle):
    """samplers/tests/test_independent.py:test02_sample_vs_pcg32: sampler.next_1d == PCG32(tea(seed, lane))."""
    L = oracle.lib()
    for seed, lane in ((0, 0), (7, 12345), (1234, 2 ** 31 + 5)):
        v0, v1 = ctypes.c_uint32(), ctypes.c_uint32()
        L.oracle_tea(seed, lane, 4, ctypes.byref(v0), ctypes.byref(v1))
        raw = (ctypes.c_uint32 * 8)()
        L.oracle_pcg32_u32(v0.value, v1.value, 8, raw)
        got = (ctypes.c_float * 8)()
        L.oracle_sampler_1d(seed, lane, 8, got)
        expect = [np.float32(np.uint32((u >> 9) | 0x3F800000).view(np.float32) - np.float32(1.0)) for u in raw]
        assert [np.float32(x) for x in got] == expect


# ---------------------------------------------------------------- filter / ImageBlock

def test_gaussian_filter_spot_values(oracle):
    """src/rfilters/tests/test_rfilter.py:test02_gaussian (eval(0.2) ~ 0.9227, 0 beyond the radius)."""
    L = oracle.lib()
    assert abs(L.oracle_gaussian_eval(0.5, 0.2) - 0.9227) <= 8e-3
    assert L.oracle_gaussian_eval(0.5, 2.1) == 0.0
    assert L.oracle_gaussian_eval(0.5, -2.1) == 0.0


def test_imageblock_put_boundary(oracle):
    """src/render/tests/test_imageblock.py:test03_put_boundary: 3x3 block, put [1] at (1.5, 1.5)."""
    L = oracle.lib()
    a, b = L.oracle_gaussian_eval(0.5, 0.0), L.oracle_gaussian_eval(0.5, 1.0)
    c = b * b
    for coalesce in (False, True):
        f = np.zeros((3, 3, 1), np.float32)
        oracle.film_put(f, 1.5, 1.5, [1.0], coalesce=coalesce)
        assert np.allclose(f[..., 0].ravel(), [c, b, c, b, a, b, c, b, c], atol=1e-3)


@pytest.mark.parametrize("coalesce", [False, True])
def test_imageblock_put_brute_force(oracle, coalesce):
    """src/render/tests/test_imageblock.py:test02_put (gaussian, no border/offset/normalize):
    each cell gets eval(cell + .5 - pos.x) * eval(cell + .5 - pos.y); one point lies exactly on a boundary."""
    L = oracle.lib()
    ev = np.vectorize(lambda x: L.oracle_gaussian_eval(0.5, float(x)))
    for j in range(5):
        for i in range(5):
            px, py = np.float32(3.3 + 0.25 * i), np.float32(3 + 0.25 * j)
            f = np.zeros((6, 6, 1), np.float32)
            oracle.film_put(f, float(px), float(py), [1.0], coalesce=coalesce)
            cx = np.arange(6, dtype=np.float32) + np.float32(0.5) - px
            cy = np.arange(6, dtype=np.float32) + np.float32(0.5) - py
            ref = np.outer(ev(-cy), ev(-cx)).astype(np.float32)
            assert np.allclose(f[..., 0], ref, atol=1e-5), (i, j)


def test_box_filter_put(oracle):
    """Box reconstruction: the sample lands in exactly one pixel with unit weight."""
    f = np.zeros((4, 5, 4), np.float32)
    oracle.film_put(f, 2.7, 1.2, [1.0, 2.0, 3.0, 1.0], box=True)
    assert f.sum() == 7.0 and np.array_equal(f[1, 2], [1, 2, 3, 1])


# ---------------------------------------------------------------- warps

def test_warps(oracle):
    """src/core/tests/test_warp.py: square_to_cosine_hemisphere, square_to_uniform_disk_concentric."""
    L = oracle.lib()
    assert np.allclose(_vec(L, "oracle_square_to_cosine_hemisphere", 0.5, 0.5), [0, 0, 1])
    assert np.allclose(_vec(L, "oracle_square_to_cosine_hemisphere", 0.5, 0.0), [0, -1, 0], atol=1e-7)
    s = 1 / math.sqrt(2)
    assert np.allclose(_vec(L, "oracle_square_to_uniform_disk_concentric", 0.0, 0.0, n=2), [-s, -s])
    assert np.allclose(_vec(L, "oracle_square_to_uniform_disk_concentric", 0.5, 0.5, n=2), [0, 0])


def test_sincos_accuracy(oracle):
    """The oracle's shared sincos (Cephes polynomial, as Dr.Jit) is accurate to a few ulp."""
    L = oracle.lib()
    xs = np.linspace(-40, 40, 2001, dtype=np.float32)
    s, c = ctypes.c_float(), ctypes.c_float()
    err = 0.0
    for x in xs:
        L.oracle_sincos(float(x), ctypes.byref(s), ctypes.byref(c))
        err = max(err, abs(s.value - math.sin(float(x))), abs(c.value - math.cos(float(x))))
    assert err < 4e-7


# ---------------------------------------------------------------- BSDFs

def test_diffuse_eval_pdf(oracle):
    """src/bsdfs/tests/test_diffuse.py:test02_eval_pdf (reflectance 0.5)."""
    L = oracle.lib()
    refl = oracle.f32(0.5, 0.5, 0.5)
    wi = oracle.f32(0, 0, 1)
    for i in range(20):
        theta = i / 19.0 * (math.pi / 2)
        wo = oracle.f32(math.sin(theta), 0, math.cos(theta))
        val = oracle.f32(0, 0, 0)
        pdf = ctypes.c_float()
        L.oracle_diffuse_eval_pdf(refl.ctypes.data, wi.ctypes.data, wo.ctypes.data, val.ctypes.data,
                                  ctypes.byref(pdf))
        if wo[2] > 0:
            assert np.allclose(pdf.value, wo[2] / math.pi, rtol=1e-5, atol=1e-8)
            assert np.allclose(val, 0.5 * wo[2] / math.pi, rtol=1e-5, atol=1e-8)
        else:
            assert pdf.value == 0.0 and not val.any()


def _sweep_theta(lo, hi, steps, phi):
    th = np.linspace(lo, hi, steps, dtype=np.float32)
    return np.stack([np.cos(np.float32(phi)) * np.sin(th), np.sin(np.float32(phi)) * np.sin(th), np.cos(th)],
                    1).astype(np.float32)


def _sweep_phi(theta, steps):
    ph = np.linspace(0, 2 * np.pi, steps, dtype=np.float32)
    t = np.float32(theta)
    return np.stack([np.cos(ph) * np.sin(t), np.sin(ph) * np.sin(t), np.full_like(ph, np.cos(t))], 1).astype(
        np.float32)


BECKMANN, GGX = 0, 1


def test_beckmann_eval_pdf_tables(oracle, kats):
    """src/render/tests/test_microfacet.py:test02_eval_pdf_beckmann (Mitsuba 0.6 tables)."""
    L = oracle.lib()
    K = kats["beckmann_eval_pdf"]
    wi = oracle.f32(0, 0, 1)
    V = _sweep_theta(0, np.pi, 20, np.pi / 2)
    ev = lambda au, av: [L.oracle_microfacet_eval(BECKMANN, au, av, np.ascontiguousarray(v).ctypes.data) for v in V]
    pdf = lambda au, av: [L.oracle_microfacet_pdf(BECKMANN, au, av, 0, wi.ctypes.data,
                                                  np.ascontiguousarray(v).ctypes.data) for v in V]
    assert np.allclose(ev(0.1, 0.3), K["theta_eval_aniso"], rtol=1e-5, atol=1e-8)
    assert np.allclose(pdf(0.1, 0.3), K["theta_pdf_aniso"], rtol=1e-5, atol=1e-8)
    assert np.allclose(ev(0.1, 0.1), K["theta_eval_iso"], rtol=1e-5, atol=1e-8)
    assert np.allclose(pdf(0.1, 0.1), K["theta_pdf_iso"], rtol=1e-5, atol=1e-8)
    V = _sweep_phi(0.1, 20)
    assert np.allclose(ev(0.1, 0.3), K["phi_eval_aniso"], rtol=1e-5, atol=1e-8)
    assert np.allclose(pdf(0.1, 0.3), np.array(K["phi_pdf_aniso_over_cos0.1"]) * math.cos(0.1), rtol=1e-5, atol=1e-8)
    assert np.allclose(ev(0.1, 0.1), K["phi_eval_iso_const"], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("kind,name", [(BECKMANN, "beckmann_smith_g1"), (GGX, "ggx_smith_g1")])
def test_smith_g1_tables(oracle, kats, kind, name):
    """src/render/tests/test_microfacet.py:test03_smith_g1_{beckmann,ggx} (atol 1e-5 for the theta sweeps)."""
    L = oracle.lib()
    K = kats[name]
    wi = oracle.f32(0, 0, 1)
    g1 = lambda au, av, V: [L.oracle_microfacet_smith_g1(kind, au, av, np.ascontiguousarray(v).ctypes.data,
                                                         wi.ctypes.data) for v in V]
    V = _sweep_theta(np.pi / 3, np.pi / 2, 20, np.pi / 2)
    assert np.allclose(g1(0.1, 0.3, V), K["theta_aniso"], atol=1e-5)
    assert np.allclose(g1(0.1, 0.1, V), K["theta_iso"], atol=1e-5)
    V = _sweep_phi(np.pi / 2 * 0.98, 20)
    assert np.allclose(g1(0.1, 0.3, V), K["phi_aniso"], rtol=1e-5, atol=1e-8)
    assert np.allclose(g1(0.1, 0.1, V), K["phi_aniso"][0], rtol=1e-5, atol=1e-8)


def test_ggx_visible_sampling_pdf_consistency(oracle):
    """GGX visible-normal sampling: returned pdf == D(m) G1(wi, m) |wi.m| / wi.z (microfacet.h:362-365)."""
    L = oracle.lib()
    rng = np.random.default_rng(1)
    for _ in range(200):
        t = rng.uniform(0, 1.4)
        wi = oracle.f32(math.sin(t), 0.0, math.cos(t))
        m = oracle.f32(0, 0, 0)
        pdf = ctypes.c_float()
        L.oracle_microfacet_sample(GGX, 0.3, 0.3, 1, wi.ctypes.data, float(rng.uniform()), float(rng.uniform()),
                                   m.ctypes.data, ctypes.byref(pdf))
        assert abs(np.linalg.norm(m) - 1) < 1e-5 and m[2] > 0
        ref = L.oracle_microfacet_pdf(GGX, 0.3, 0.3, 1, wi.ctypes.data, m.ctypes.data)
        assert np.isclose(pdf.value, ref, rtol=1e-5)


def test_fresnel_conductor_limits(oracle):
    """Conductor Fresnel: normal incidence ((n-1)^2 + k^2) / ((n+1)^2 + k^2), 1 at grazing."""
    L = oracle.lib()
    n, k = 0.2, 3.0
    assert np.isclose(L.oracle_fresnel_conductor(1.0, n, k), ((n - 1) ** 2 + k * k) / ((n + 1) ** 2 + k * k),
                      rtol=1e-5)
    assert np.isclose(L.oracle_fresnel_conductor(0.0, n, k), 1.0, rtol=1e-5)


def test_beckmann_transcendentals_vs_libm(oracle):
    """exp / log / erf / erfinv / tan of the Beckmann path (oracle_math.h restatements; Dr.Jit's own are
    not vendored, so parity with the reference is unpinned at the last ulp): within a few ulp of libm /
    math.erf / scipy's erfinv over the ranges the sampling code reaches."""
    from scipy import special
    L = oracle.lib()

    def run(fn, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        y = np.zeros_like(x)
        L.oracle_math(fn, x.ctypes.data, y.ctypes.data, len(x))
        return y.astype(np.float64), x.astype(np.float64)

    y, x = run(0, np.linspace(-87, 88, 20001))
    assert np.max(np.abs(y / np.exp(x) - 1)) < 4e-7
    y, x = run(0, np.array([-100.0, 100.0, np.nan]))
    assert y[0] == 0 and np.isinf(y[1]) and np.isnan(y[2])
    y, x = run(1, np.concatenate([np.geomspace(1e-40, 1e30, 20001), np.linspace(0.5, 2, 2001)]))
    ref = np.log(x)
    assert np.max(np.abs(y - ref) / np.maximum(np.abs(ref), 1e-3)) < 4e-7
    y, x = run(1, np.array([0.0, -1.0, np.inf]))
    assert np.isneginf(y[0]) and np.isnan(y[1]) and np.isposinf(y[2])
    y, x = run(2, np.linspace(-5, 5, 40001))
    assert np.max(np.abs(y - special.erf(x))) < 3e-7
    y, x = run(3, np.linspace(-0.999999, 0.999999, 40001))
    ref = special.erfinv(x)
    assert np.max(np.abs(y - ref) / np.maximum(np.abs(ref), 1e-6)) < 2e-6
    y, x = run(4, np.linspace(-6.2, 6.2, 40001))
    ref = np.tan(x)
    ok = np.abs(np.cos(x)) > 1e-3
    assert np.max(np.abs(y - ref)[ok] / np.maximum(np.abs(ref[ok]), 1.0)) < 1e-5


@pytest.mark.parametrize("kind,au,av,visible,theta_i", [
    (BECKMANN, 0.3, 0.3, 1, 0.7), (BECKMANN, 0.2, 0.5, 1, 1.2), (BECKMANN, 0.3, 0.3, 0, 0.0),
    (BECKMANN, 0.15, 0.45, 0, 0.0), (GGX, 0.15, 0.45, 0, 0.0), (GGX, 0.2, 0.5, 1, 1.0)],
    ids=["beck_vis_iso", "beck_vis_aniso", "beck_iso", "beck_aniso", "ggx_aniso", "ggx_vis_aniso"])
def test_microfacet_sampling_matches_its_pdf(oracle, kind, au, av, visible, theta_i):
    """MicrofacetDistribution::sample (microfacet.h:244-360) draws normals distributed as its pdf(): the
    returned pdf equals pdf(wi, m), and sample moments of m match the pdf's moments by quadrature.  Covers
    the Beckmann elevation, the anisotropic azimuth inversion and the Beckmann visible-normal inversion."""
    L = oracle.lib()
    wi = oracle.f32(math.sin(theta_i), 0.0, math.cos(theta_i))
    rng = np.random.default_rng(7)
    n = 20000
    ms = np.zeros((n, 3))
    m = oracle.f32(0, 0, 0)
    pdf = ctypes.c_float()
    for i in range(n):
        L.oracle_microfacet_sample(kind, au, av, visible, wi.ctypes.data, float(rng.uniform()), float(rng.uniform()),
                                   m.ctypes.data, ctypes.byref(pdf))
        ms[i] = m
        if i < 300:
            ref = L.oracle_microfacet_pdf(kind, au, av, visible, wi.ctypes.data, m.ctypes.data)
            assert np.isclose(pdf.value, ref, rtol=2e-5, atol=1e-12)
    # quadrature of pdf(m) dω over the upper hemisphere
    th = (np.arange(600) + 0.5) * (np.pi / 2 / 600)
    ph = (np.arange(600) + 0.5) * (2 * np.pi / 600)
    T, Pp = np.meshgrid(th, ph, indexing="ij")
    M = np.stack([np.sin(T) * np.cos(Pp), np.sin(T) * np.sin(Pp), np.cos(T)], -1).astype(np.float32).reshape(-1, 3)
    w = np.array([L.oracle_microfacet_pdf(kind, au, av, visible, wi.ctypes.data, np.ascontiguousarray(v).ctypes.data)
                  for v in M]) * (np.sin(T).reshape(-1)) * (np.pi / 2 / 600) * (2 * np.pi / 600)
    assert abs(w.sum() - 1) < 0.01
    for f in (lambda v: v[:, 0], lambda v: v[:, 2], lambda v: v[:, 0] ** 2, lambda v: v[:, 1] ** 2):
        q, s = (f(M.astype(np.float64)) * w).sum() / w.sum(), f(ms).mean()
        assert abs(q - s) < 4 * f(ms).std() / math.sqrt(n) + 2e-3, (q, s)


def test_fixed_point_film_matches_float_film(oracle, amvpt_mod):
    """The oracle's fixed-point film (the device's AMVPT_OPT_DETERMINISTIC accumulation restated: each cell add
    rounded to 2^-32, summed as integers, converted once) equals the f32 ImageBlock film to summation order,
    does not depend on the thread split, and drops nothing at normal radiance."""
    from conftest import SCENES as _S
    s = amvpt_mod.load_file(os.path.join(_S, "cbox_grid.xml"), res=8, spp=16, gx=2, gy=2, reuse=4)
    sd, vd, p = s.describe(0, 0, 0)
    f, _, _ = oracle.render(sd, vd, p, threads=4)
    x1, _, st = oracle.render(sd, vd, p, threads=4, fixed_film=True)
    x2, _, _ = oracle.render(sd, vd, p, threads=3, fixed_film=True)
    assert np.array_equal(x1, x2) and st["range_drops"] == 0
    assert np.abs(x1 - f).max() <= 1e-5 * np.abs(f).max()
    g, _, _ = oracle.render(sd, vd, p, threads=4)   # the mode does not stick
    assert np.abs(g - f).max() <= 1e-5 * np.abs(f).max()


def test_oracle_bvh_mode_matches_brute_force(amvpt_mod, oracle):
    """The oracle's optional BVH (oracle_set_bvh: bench.py's CPU baseline on BVH scenes) gives the brute-force scan's
    records bit for bit on the 3.6 k-triangle mesh scene (path and G = 8)."""
    import os
    import numpy as np
    from conftest import SCENES
    for kw in (dict(res=8, spp=16), dict(res=8, spp=16, gx=4, gy=2, reuse=8)):
        s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_mesh.xml"), **kw)
        sd, vd, p = s.describe(0, 0, 0)
        f0, r0, _ = oracle.render(sd, vd, p, threads=8, record_pass=0)
        oracle.set_bvh(True)
        try:
            f1, r1, _ = oracle.render(sd, vd, p, threads=8, record_pass=0)
        finally:
            oracle.set_bvh(False)
        same = (r0 == r1) | (np.isnan(r0) & np.isnan(r1))
        assert same.all(), "%d record floats differ" % (~same).sum()
        assert np.array_equal(f0, f1)
