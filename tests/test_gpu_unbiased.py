"""Independent unbiasedness gate.

The bit-level parity tests pin the HIP pipeline to the CPU oracle; both are restatements of the
reference, so a misreading of mvpath_multi.h would agree with itself.  This gate checks the
statistics instead: every view of an AMVPT render (sa_reuse + sa_mis, G = 4 or 8: camera
selection, MIS weights and radiance reuse) against a high-spp render of the same views with
reuse off (G = 1: render_sample / sample_single, the stock path tracer of a14), both through the
drop-in host path (Integrator::render -> C-ABI -> HIP) on the GPU, K independent seeds per side.

1. Per-pixel Z-test, the method of the reference's render tests (src/render/tests/
   test_renders.py:159-230): Z statistic, two-sided p-value, Sidak-corrected level
   alpha = 1 - (1 - 0.01)^(1/N) over the N pixel channels, accepted when >= 99.75 % pass.  The
   reference compares against a stored image and its per-sample variance; here both sides are
   measured, z = |mean_A - mean_R| / sqrt(var_A / K + var_R / K).
   Scope: pixels whose 5 x 5 filter footprint is smooth in the reference image (relative range
   < 0.3) and >= 2 px inside their view tile.  The film is self-normalised (RGB / W, W = sum of
   MIS weight x filter weight), so a pixel's value is a weighted mean of the radiance over its
   footprint with weights proportional to the local density of (primary + reprojected) samples
   times their MIS weights.  That density varies between the two sides of a depth or normal
   discontinuity (different Jacobians per view), so at edges the AMVPT film is a differently
   weighted average than the path tracer's -- a property of the reference estimator, measured
   here as thin streaks along wall corners and box silhouettes (profiles/r02_unbiased_zmaps.txt),
   not a sampling bias; tile-edge pixels mix two views' content in the borderless quilt.
2. Per-view energy: the mean over each view's interior pixels, two-sample z over the K frames,
   |z| < 4.5 for every view -- a systematic bias (MIS weights that do not sum to one, a lost or
   doubled strategy) moves these means while edge effects of either sign average out.
3. Power: the same AMVPT frames scaled by 1.3 fail gate 1.
"""
import os

import numpy as np
import pytest
from scipy.ndimage import maximum_filter, minimum_filter
from scipy.special import erf

from conftest import SCENES

pytestmark = pytest.mark.gpu

CBOX = os.path.join(SCENES, "cbox_grid.xml")
VEACH = os.path.join(SCENES, "veach_grid.xml")
MESHLIGHT = os.path.join(SCENES, "cbox_meshlight.xml")
RECTLIGHTS = os.path.join(SCENES, "cbox_cubelight_rects.xml")
K = 24   # independent seeds per side


def _frames(amvpt_mod, path, seeds, **defines):
    scene = amvpt_mod.load_file(path, **defines)
    return np.stack([amvpt_mod.render(scene, seed=s)[..., :3].astype(np.float64) for s in seeds])


def _pair(amvpt_mod, path, defines, ref_spp=512):
    test = _frames(amvpt_mod, path, range(K), **defines)
    ref = _frames(amvpt_mod, path, range(1000, 1000 + K), **dict(defines, reuse=1, spp=ref_spp))
    assert np.isfinite(test).all() and np.isfinite(ref).all()
    return test, ref


def _interior(shape, res):
    H, W = shape
    y, x = np.mgrid[0:H, 0:W]
    return ((y % res) >= 2) & ((y % res) < res - 2) & ((x % res) >= 2) & ((x % res) < res - 2)


def _smooth(ref_mean, res, rel_range=0.3):
    """interior pixels whose 5 x 5 footprint has a relative range below rel_range in the reference"""
    lum = ref_mean.mean(-1)
    mx, mn = maximum_filter(lum, size=5), minimum_filter(lum, size=5)
    return _interior(lum.shape, res) & ((mx - mn) < rel_range * np.maximum(mx, 1e-6))


def _z_gate(test, ref, significance=0.01):
    """fraction of pixel channels whose p-value exceeds the Sidak-corrected level"""
    diff = np.abs(test.mean(0) - ref.mean(0))
    se = np.sqrt(test.var(0, ddof=1) / len(test) + ref.var(0, ddof=1) / len(ref))
    z = np.where(diff == 0.0, 0.0, diff / np.maximum(se, 1e-12))
    p = 2.0 * (1.0 - 0.5 * (1.0 + erf(z / np.sqrt(2.0))))
    alpha = 1.0 - (1.0 - significance) ** (1.0 / z.size)
    return float((p > alpha).mean()), float(p.min()), alpha


def _view_means(frames, res):
    """(K, n_views) mean over each view tile's interior"""
    Kf, H, W, _ = frames.shape
    inner = _interior((H, W), res)
    out = []
    for ty in range(H // res):
        for tx in range(W // res):
            m = np.zeros((H, W), bool)
            m[ty * res:(ty + 1) * res, tx * res:(tx + 1) * res] = True
            out.append(frames[:, m & inner].mean(axis=(1, 2)))
    return np.stack(out, 1)


CASES = [
    ("cbox_g4", CBOX, dict(res=48, spp=64, gx=2, gy=2, reuse=4)),
    ("cbox_g8", CBOX, dict(res=48, spp=64, gx=4, gy=2, reuse=8)),
    ("veach_g8", VEACH, dict(res=48, spp=64, gx=4, gy=2, reuse=8)),
]


@pytest.mark.parametrize("name,path,defines", CASES, ids=[c[0] for c in CASES])
def test_amvpt_views_unbiased_against_single_view(gpu_ready, amvpt_mod, name, path, defines):
    test, ref = _pair(amvpt_mod, path, defines)
    res = defines["res"]
    smooth = _smooth(ref.mean(0), res)
    frac, pmin, alpha = _z_gate(test[:, smooth], ref[:, smooth])
    full, _, _ = _z_gate(test[:, _interior(test.shape[1:3], res)], ref[:, _interior(ref.shape[1:3], res)])
    vt, vr = _view_means(test, res), _view_means(ref, res)
    zv = np.abs(vt.mean(0) - vr.mean(0)) / np.sqrt(vt.var(0, ddof=1) / K + vr.var(0, ddof=1) / K)
    print("%s: smooth-footprint gate %.4f of %d channels (p > %.3g, min p %.3g); all interior %.4f; "
          "per-view |z| max %.2f, mean ratio %s" % (
              name, frac, int(smooth.sum()) * 3, alpha, pmin, full, zv.max(),
              np.round(vt.mean(0) / vr.mean(0), 4).tolist()))
    assert frac >= 0.9975, "Z-test rejects: only %.4f of smooth-footprint pixel channels pass" % frac
    assert zv.max() < 4.5, "per-view mean differs: |z| = %s" % np.round(zv, 2).tolist()


def test_mesh_light_matches_rectangle_lights(gpu_ready, amvpt_mod):
    """Area emitter on a mesh (mesh.cpp:765-816: area-CDF face pick, barycentric point) against the
    same flat box emitting as six rectangles (rectangle.cpp sampling): two different unbiased
    estimators of one image, compared with the reference's Z-test (test_renders.py:159-230)."""
    defines = dict(res=48, spp=64, gx=2, gy=2, reuse=4)
    test = _frames(amvpt_mod, MESHLIGHT, range(K), **defines)
    ref = _frames(amvpt_mod, RECTLIGHTS, range(1000, 1000 + K), **dict(defines, spp=256))
    assert np.isfinite(test).all() and np.isfinite(ref).all()
    res = defines["res"]
    smooth = _smooth(ref.mean(0), res)
    frac, pmin, alpha = _z_gate(test[:, smooth], ref[:, smooth])
    vt, vr = _view_means(test, res), _view_means(ref, res)
    zv = np.abs(vt.mean(0) - vr.mean(0)) / np.sqrt(vt.var(0, ddof=1) / K + vr.var(0, ddof=1) / K)
    print("mesh light vs rectangles: gate %.4f (min p %.3g), per-view |z| max %.2f, mean ratio %s" % (
        frac, pmin, zv.max(), np.round(vt.mean(0) / vr.mean(0), 4).tolist()))
    assert frac >= 0.9975, "Z-test rejects: only %.4f of smooth-footprint pixel channels pass" % frac
    assert zv.max() < 4.5, "per-view mean differs: |z| = %s" % np.round(zv, 2).tolist()


def test_z_gate_detects_a_biased_estimator(gpu_ready, amvpt_mod):
    """The gate has power: the same AMVPT frames scaled by 1.3 (a 30 % bias) are rejected."""
    defines = dict(res=48, spp=64, gx=2, gy=2, reuse=4)
    test, ref = _pair(amvpt_mod, CBOX, defines)
    smooth = _smooth(ref.mean(0), 48)
    frac, _, _ = _z_gate(1.3 * test[:, smooth], ref[:, smooth])
    print("biased x1.3: %.4f pass" % frac)
    assert frac < 0.9975
