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
   Scope: every pixel >= 2 px inside its view tile except a GEOMETRIC edge mask computed from the
   scene, not from either image: pixels whose filter footprint (5 x 5 for the Gaussian, 3 x 3 for the
   box filter) contains a primary-hit discontinuity -- a change of shape or of geometric normal between
   neighbouring pixel centres (oracle.primary_hits) -- in the view itself or reprojected from any view
   of its group (the 3-D points of the group views' discontinuities projected into the view).  The film
   is self-normalised (RGB / W, W = sum of MIS weight x filter weight), so a pixel's value is a weighted
   mean of the radiance over its footprint with weights proportional to the local density of (primary +
   reprojected) samples times their MIS weights; that density differs on the two sides of a
   discontinuity (different Jacobians per view), so a footprint that straddles one is a differently
   weighted average than the path tracer's -- a property of the reference estimator.  The box-filter
   case tests that explanation: with a one-pixel footprint the rejections must shrink to the 3 x 3
   neighbourhood of the discontinuities themselves.  Tile-edge pixels mix two views' content in the
   borderless quilt.
2. Per-view energy: the mean over each view's interior pixels off the edge mask, two-sample z over the
   K frames, |z| < 4.5 for every view -- a systematic bias (MIS weights that do not sum to one, a lost or
   doubled strategy) moves these means.  (Round 5 took every interior pixel, assuming the edge effects of
   either sign average out; with a wide baseline -- the cone grid -- they do not, see the case list.)
3. Power: the same AMVPT frames scaled by 1.3 fail gate 1.
"""
import os

import numpy as np
import pytest
from scipy.ndimage import maximum_filter
from scipy.special import erf

from conftest import SCENES

pytestmark = pytest.mark.gpu

CBOX = os.path.join(SCENES, "cbox_grid.xml")
VEACH = os.path.join(SCENES, "veach_grid.xml")
MESHLIGHT = os.path.join(SCENES, "cbox_meshlight.xml")
RECTLIGHTS = os.path.join(SCENES, "cbox_cubelight_rects.xml")
MESH = os.path.join(SCENES, "cbox_mesh.xml")
CONE = os.path.join(SCENES, "cbox_cone.xml")
K = 24   # independent seeds per side


def _frames(amvpt_mod, path, seeds, **defines):
    scene = amvpt_mod.load_file(path, **defines)
    return np.stack([amvpt_mod.render(scene, seed=s)[..., :3].astype(np.float64) for s in seeds])


_PAIRS = {}


def _pair(amvpt_mod, path, defines, ref_spp=512):
    key = (path, tuple(sorted(defines.items())), ref_spp)
    if key not in _PAIRS:
        test = _frames(amvpt_mod, path, range(K), **defines)
        ref = _frames(amvpt_mod, path, range(1000, 1000 + K), **dict(defines, reuse=1, spp=ref_spp))
        assert np.isfinite(test).all() and np.isfinite(ref).all()
        _PAIRS.clear()   # one pair in memory at a time (the box-filter test reuses the last one)
        _PAIRS[key] = (test, ref)
    return _PAIRS[key]


def _interior(shape, res):
    H, W = shape
    y, x = np.mgrid[0:H, 0:W]
    return ((y % res) >= 2) & ((y % res) < res - 2) & ((x % res) >= 2) & ((x % res) < res - 2)


def _project(view, pts):
    """raster position (view-local pixel units) of world points in a perspective view: the raster part of
    PerspectiveCamera::sample_surface (perspective.cpp:327-385), in float64"""
    M = np.array(view.to_world_inv[:], dtype=np.float64).reshape(4, 4)
    S = np.array(view.camera_to_sample[:], dtype=np.float64).reshape(4, 4)
    h = np.concatenate([pts, np.ones((len(pts), 1))], 1)
    cam = h @ M.T
    scr = cam @ S.T
    scr = scr[:, :3] / scr[:, 3:4]
    ux = (scr[:, 0] - view.pp_offset[0]) * view.resolution[0]
    uy = (scr[:, 1] - view.pp_offset[1]) * view.resolution[1]
    return ux, uy, cam[:, 2] > 0


def _edge_mask(amvpt_mod, path, defines, G, radius):
    """Geometric edge mask (see the module docstring): primary-hit discontinuities of each view and of its
    group's views reprojected into it, dilated by the filter footprint (radius 2: Gaussian 5 x 5, 1: box)."""
    from oracle import oracle as O
    s = amvpt_mod.load_file(path, **defines)
    sd, vd, p = s.describe(0, 0, 0)
    hits = O.primary_hits(sd, vd, p)
    H, W = hits.shape[:2]
    gx, gy = p.grid_x, p.grid_y
    rx, ry = W // gx, H // gy
    ids, nrm, pts, view = hits[..., 0], hits[..., 1:4], hits[..., 4:7].astype(np.float64), hits[..., 7].astype(int)
    yy, xx = np.mgrid[0:H, 0:W]
    disc = np.zeros((H, W), bool)
    for dy, dx in ((0, 1), (1, 0)):
        a = (slice(0, H - dy), slice(0, W - dx))
        b = (slice(dy, H), slice(dx, W))
        same = (xx[a] // rx == xx[b] // rx) & (yy[a] // ry == yy[b] // ry)
        diff = (ids[a] != ids[b]) | ((nrm[a] * nrm[b]).sum(-1) < 0.99)
        disc[a] |= diff & same
        disc[b] |= diff & same
    marks = disc.copy()
    for j in range(p.n_views):
        sel = disc & (view == j) & (ids >= 0)
        if not sel.any():
            continue
        for k in range(G * (j // G), G * (j // G) + G):
            if k == j:
                continue
            ux, uy, front = _project(vd[k], pts[sel])
            ok = front & (ux >= 0) & (ux < rx) & (uy >= 0) & (uy < ry)
            ix, iy = k % gx, k // gx
            if p.reverse_x:
                ix = gx - 1 - ix
            if p.reverse_y:
                iy = gy - 1 - iy
            marks[(np.floor(uy[ok]).astype(int) + iy * ry), (np.floor(ux[ok]).astype(int) + ix * rx)] = True
    return maximum_filter(marks, size=2 * radius + 1)


def _z_gate(test, ref, significance=0.01):
    """fraction of pixel channels whose p-value exceeds the Sidak-corrected level"""
    diff = np.abs(test.mean(0) - ref.mean(0))
    se = np.sqrt(test.var(0, ddof=1) / len(test) + ref.var(0, ddof=1) / len(ref))
    z = np.where(diff == 0.0, 0.0, diff / np.maximum(se, 1e-12))
    p = 2.0 * (1.0 - 0.5 * (1.0 + erf(z / np.sqrt(2.0))))
    alpha = 1.0 - (1.0 - significance) ** (1.0 / z.size)
    return float((p > alpha).mean()), float(p.min()), alpha


def _view_means(frames, res, mask=None):
    """(K, n_views) mean over each view tile's interior (and `mask`)"""
    Kf, H, W, _ = frames.shape
    inner = _interior((H, W), res) if mask is None else mask
    out = []
    for ty in range(H // res):
        for tx in range(W // res):
            m = np.zeros((H, W), bool)
            m[ty * res:(ty + 1) * res, tx * res:(tx + 1) * res] = True
            out.append(frames[:, m & inner].mean(axis=(1, 2)))
    return np.stack(out, 1)


RES = 128   # per-view resolution: edges are 1-D, so the masked share of the interior falls with it (41 % here)
CASES = [
    ("cbox_g4", CBOX, dict(res=RES, spp=64, gx=2, gy=2, reuse=4), 4, 2),
    ("cbox_g8", CBOX, dict(res=RES, spp=64, gx=4, gy=2, reuse=8), 8, 2),
    ("veach_g8", VEACH, dict(res=RES, spp=64, gx=4, gy=2, reuse=8), 8, 2),
    ("cbox_g8_box", CBOX, dict(res=RES, spp=64, gx=4, gy=2, reuse=8, rfilter="box"), 8, 1),
    # the parts the restatement alone pins.  The adaptive fill (mvpath_multi.h:52-59,79-115) on the
    # C5 shape (8 x 4 grid, groups of 4, adaptive 3, one 16-spp pass) -- its reference side is the same views
    # with reuse off, where the fill does not apply; the 3.6 k-triangle OBJ/PLY box (per-lane BVH walks with ray
    # binning, a rough-conductor object); thin-lens views (thinlens.cpp:358-418), whose defocus spreads a
    # discontinuity over a circle of confusion of up to ~3 px here (aperture 0.05, focus 3.9, objects 3..4.9
    # away), so their mask is dilated by 5 px instead of the filter's 2
    ("c5_adaptive", CBOX, dict(res=64, spp=16, gx=8, gy=4, reuse=4, adaptive=3), 4, 2),
    ("mesh_g8", MESH, dict(res=RES, spp=64, gx=4, gy=2, reuse=8), 8, 2),
    ("cbox_g8_thinlens", CBOX, dict(res=RES, spp=64, gx=4, gy=2, reuse=8, cam="thinlens", aperture="0.05"), 8, 5),
    # the light-field cone layout (grid.cpp:182-205): every view off-axis through its own
    # lens_shift, so every Jacobian and film pdf of sample_surface sees a sheared projection
    ("cbox_g8_cone", CONE, dict(res=RES, spp=64, gx=4, gy=2, reuse=8, cone=12), 8, 2),
]


def _rejected(test, ref, mask, significance=0.01):
    """pixel-channel rejection map of the Z-test over `mask` (Sidak level over the mask's channels)"""
    diff = np.abs(test.mean(0) - ref.mean(0))
    se = np.sqrt(test.var(0, ddof=1) / len(test) + ref.var(0, ddof=1) / len(ref))
    z = np.where(diff == 0.0, 0.0, diff / np.maximum(se, 1e-12))
    p = 2.0 * (1.0 - 0.5 * (1.0 + erf(z / np.sqrt(2.0))))
    alpha = 1.0 - (1.0 - significance) ** (1.0 / (int(mask.sum()) * 3))
    return (p <= alpha) & mask[..., None]


@pytest.mark.parametrize("name,path,defines,G,radius", CASES, ids=[c[0] for c in CASES])
def test_amvpt_views_unbiased_against_single_view(gpu_ready, amvpt_mod, name, path, defines, G, radius):
    test, ref = _pair(amvpt_mod, path, defines)
    res = defines["res"]
    interior = _interior(test.shape[1:3], res)
    edges = _edge_mask(amvpt_mod, path, defines, G, radius)
    gate = interior & ~edges
    frac, pmin, alpha = _z_gate(test[:, gate], ref[:, gate])
    full, _, _ = _z_gate(test[:, interior], ref[:, interior])
    # per-view energy over the same off-mask pixels as the Z-test (round 6): the discontinuity pixels carry the
    # self-normalised film's footprint-straddle bias, which does not cancel within a view once the group's
    # baseline is wide -- tools/cone_control.py (profiles/r06d_cone_control.*): on the 12-degree cone grid and on a
    # plain cam_dir line through the same camera positions the central views' interior means read +0.14..0.19 %
    # (|z| up to 11 at 256 spp, growing with spp), all of it in the masked pixels; off the mask every view is
    # within 0.03 % (|z| < 2.1), with either filter
    vt, vr = _view_means(test, res, gate), _view_means(ref, res, gate)
    zv = np.abs(vt.mean(0) - vr.mean(0)) / np.sqrt(vt.var(0, ddof=1) / K + vr.var(0, ddof=1) / K)
    at, ar = _view_means(test, res), _view_means(ref, res)
    za = np.abs(at.mean(0) - ar.mean(0)) / np.sqrt(at.var(0, ddof=1) / K + ar.var(0, ddof=1) / K)
    print("%s: off-edge gate %.5f of %d channels (%.1f %% of the interior; p > %.3g, min p %.3g); all interior %.5f; "
          "per-view off-mask |z| max %.2f, mean ratio %s; all-interior |z| max %.2f, mean ratio %s" % (
              name, frac, int(gate.sum()) * 3, 100.0 * gate.sum() / interior.sum(), alpha, pmin, full, zv.max(),
              np.round(vt.mean(0) / vr.mean(0), 4).tolist(), za.max(), np.round(at.mean(0) / ar.mean(0), 4).tolist()))
    assert frac >= 0.9975, "Z-test rejects: only %.4f of off-edge pixel channels pass" % frac
    assert zv.max() < 4.5, "per-view mean differs: |z| = %s" % np.round(zv, 2).tolist()


def test_box_filter_confines_rejections_to_discontinuities(gpu_ready, amvpt_mod):
    """The stated cause of the edge rejections (a self-normalised film whose footprint straddles a
    discontinuity, see the module docstring), tested: the same config-M-shaped frames with the box filter
    (a one-pixel footprint) instead of the Gaussian (5 x 5) must lose most of their rejected interior
    channels, and those left must lie at the discontinuities themselves (3 x 3 mask)."""
    defines = dict(res=RES, spp=64, gx=4, gy=2, reuse=8)
    rej = {}
    for rf in ("gaussian", "box"):
        d = dict(defines, rfilter=rf)
        test, ref = _pair(amvpt_mod, CBOX, d)
        interior = _interior(test.shape[1:3], RES)
        rej[rf] = _rejected(test, ref, interior)
    near = _edge_mask(amvpt_mod, CBOX, dict(defines, rfilter="box"), 8, 1)
    n_g, n_b = int(rej["gaussian"].sum()), int(rej["box"].sum())
    n_b_off = int((rej["box"] & ~near[..., None]).sum())
    print("rejected interior channels: gaussian %d, box %d (%d off the 3 x 3 discontinuity mask)" % (n_g, n_b, n_b_off))
    assert n_b <= 0.25 * n_g + 10
    assert n_b_off <= 0.1 * max(n_b, 1) + 10


def test_mesh_light_matches_rectangle_lights(gpu_ready, amvpt_mod):
    """Area emitter on a mesh (mesh.cpp:765-816: area-CDF face pick, barycentric point) against the
    same flat box emitting as six rectangles (rectangle.cpp sampling): two different unbiased
    estimators of one image, compared with the reference's Z-test (test_renders.py:159-230)."""
    defines = dict(res=64, spp=64, gx=2, gy=2, reuse=4)
    test = _frames(amvpt_mod, MESHLIGHT, range(K), **defines)
    ref = _frames(amvpt_mod, RECTLIGHTS, range(1000, 1000 + K), **dict(defines, spp=256))
    assert np.isfinite(test).all() and np.isfinite(ref).all()
    res = defines["res"]
    gate = _interior(test.shape[1:3], res) & ~_edge_mask(amvpt_mod, MESHLIGHT, defines, 4, 2)
    frac, pmin, alpha = _z_gate(test[:, gate], ref[:, gate])
    vt, vr = _view_means(test, res), _view_means(ref, res)
    zv = np.abs(vt.mean(0) - vr.mean(0)) / np.sqrt(vt.var(0, ddof=1) / K + vr.var(0, ddof=1) / K)
    print("mesh light vs rectangles: gate %.4f (min p %.3g), per-view |z| max %.2f, mean ratio %s" % (
        frac, pmin, zv.max(), np.round(vt.mean(0) / vr.mean(0), 4).tolist()))
    assert frac >= 0.9975, "Z-test rejects: only %.4f of off-edge pixel channels pass" % frac
    assert zv.max() < 4.5, "per-view mean differs: |z| = %s" % np.round(zv, 2).tolist()


def test_z_gate_detects_a_biased_estimator(gpu_ready, amvpt_mod):
    """The gate has power: the same AMVPT frames scaled by 1.3 (a 30 % bias) are rejected."""
    defines = dict(res=RES, spp=64, gx=2, gy=2, reuse=4)
    test, ref = _pair(amvpt_mod, CBOX, defines)
    gate = _interior(test.shape[1:3], RES) & ~_edge_mask(amvpt_mod, CBOX, defines, 4, 2)
    frac, _, _ = _z_gate(1.3 * test[:, gate], ref[:, gate])
    print("biased x1.3: %.4f pass" % frac)
    assert frac < 0.9975


# ---------------------------------------------------------------------------------------------------------------
# Pooled energy of the C5 shape.  The per-view gate above read the adaptive C5 shape 0.12 %
# low on average (26 of 32 views).  The control (tools/adaptive_control.py, profiles/r06b_adaptive_control.*)
# found the shift with the fill off as well (adaptive 0: -0.10 % at 16 spp), shrinking with the samples per
# filter footprint (-0.039 % at 64 spp, -0.015 % at 256; -0.20 % with the 1-pixel box filter), and GONE from the
# ratio of means -- the K frames' RGB and W sums divided once -- which equals the reuse-off path tracer's to 1e-5
# at every spp, filter and resolution; the fill moves the pooled energy by 1e-5.  So it is the ratio bias of the
# reference's self-normalised film (hdrfilm develops RGB / W per frame, hdrfilm.cpp:400, and W sums per-sample
# MIS weights: E[sum wL / sum w] != E[sum wL] / E[sum w], an O(1/n) term), not a misread of the fill
# (mvpath_multi.h:52-59,79-112).  This gate pins all three facts on the C5 shape, with the frames as the
# independent units of every standard error.

C5 = dict(res=64, gx=8, gy=4, reuse=4)
KP = 64


def _raw(amvpt_mod, seeds, **defines):
    s = amvpt_mod.load_file(CBOX, **dict(C5, **defines))
    return np.stack([amvpt_mod.render(s, seed=k, raw=True).astype(np.float64) for k in seeds])


def _pooled(raw, res):
    """per frame: (mean of the developed interior pixels, interior RGB sum, interior W sum)"""
    inner = _interior(raw.shape[1:3], res)
    rgb, w = raw[:, inner, :3], raw[:, inner, 3:4]
    dev = rgb / np.where(w == 0.0, 1.0, w)
    return dev.mean(axis=(1, 2)), rgb.sum(axis=(1, 2)), w[..., 0].sum(axis=1)


def _rom(rgb, w):
    """pooled ratio of means (RGB and W summed over the frames, then divided) and its jackknife SE over frames"""
    n = len(rgb)
    full = rgb.sum() / w.sum() / 3.0
    loo = np.array([(rgb.sum() - rgb[i]) / (w.sum() - w[i]) / 3.0 for i in range(n)])
    return full, np.sqrt((n - 1) / n * ((loo - loo.mean()) ** 2).sum())


def test_pooled_energy_c5_shape(gpu_ready, amvpt_mod):
    res = C5["res"]
    a3 = _pooled(_raw(amvpt_mod, range(KP), spp=16, adaptive=3), res)
    a0 = _pooled(_raw(amvpt_mod, range(KP), spp=16, adaptive=0), res)          # same seeds: paired with a3
    g1 = _pooled(_raw(amvpt_mod, range(2000, 2000 + KP), spp=16, reuse=1), res)  # the reuse-off path tracer
    a3_64 = _pooled(_raw(amvpt_mod, range(KP), spp=64, adaptive=3), res)
    g1_64 = _pooled(_raw(amvpt_mod, range(2000, 2000 + KP), spp=64, reuse=1), res)
    # (1) the fill is energy-neutral: adaptive 3 against adaptive 0, paired by seed
    q = a3[0] / a0[0]
    fill, fill_se = q.mean(), q.std(ddof=1) / np.sqrt(KP)
    # (2) no bias in the ratio of means: AMVPT (fill on) against the reuse-off render, same spp
    r3, s3 = _rom(a3[1], a3[2])
    r1, s1 = _rom(g1[1], g1[2])
    rom, rom_se = r3 / r1, (r3 / r1) * np.hypot(s3 / r3, s1 / r1)
    r3b, s3b = _rom(a3_64[1], a3_64[2])
    r1b, s1b = _rom(g1_64[1], g1_64[2])
    rom64, rom64_se = r3b / r1b, (r3b / r1b) * np.hypot(s3b / r3b, s1b / r1b)
    # (3) the developed (per-frame) mean sits low by the ratio bias, which shrinks with spp
    shift16 = a3[0].mean() / g1[0].mean() - 1.0
    shift64 = a3_64[0].mean() / g1_64[0].mean() - 1.0
    se16 = np.hypot(a3[0].std(ddof=1) / a3[0].mean(), g1[0].std(ddof=1) / g1[0].mean()) / np.sqrt(KP)
    print("C5 shape pooled energy: fill effect %.6f +- %.6f; ratio of means AMVPT / reuse-off %.5f +- %.5f (16 spp), "
          "%.5f +- %.5f (64 spp); developed-mean shift %.5f +- %.5f (16 spp), %.5f (64 spp)" % (
              fill, fill_se, rom, rom_se, rom64, rom64_se, shift16, se16, shift64))
    assert abs(fill - 1.0) < 1e-4, "the adaptive fill moves the pooled energy by %.2e" % (fill - 1.0)
    assert abs(rom - 1.0) < 4.0 * rom_se + 2e-4, "ratio of means differs at 16 spp: %.5f +- %.5f" % (rom, rom_se)
    assert abs(rom64 - 1.0) < 4.0 * rom64_se + 2e-4, "ratio of means differs at 64 spp: %.5f +- %.5f" % (rom64, rom64_se)
    # the control measured -0.0010 +- 0.00015 (16 spp) and -0.00039 (64 spp); a misread MIS weight or a doubled
    # strategy would not leave the ratio of means alone, nor shrink with the sample count
    assert -0.0025 < shift16 < 0.0005, "developed-mean shift %.5f outside the ratio-bias budget" % shift16
    assert shift64 > shift16, "the shift does not shrink with spp: %.5f (16) vs %.5f (64)" % (shift16, shift64)


def test_pooled_energy_gate_has_power(gpu_ready, amvpt_mod):
    """The ratio-of-means gate rejects a 0.5 % energy error (RGB scaled by 1.005)."""
    res = C5["res"]
    a3 = _pooled(_raw(amvpt_mod, range(KP), spp=16, adaptive=3), res)
    g1 = _pooled(_raw(amvpt_mod, range(2000, 2000 + KP), spp=16, reuse=1), res)
    r3, s3 = _rom(1.005 * a3[1], a3[2])
    r1, s1 = _rom(g1[1], g1[2])
    rom, rom_se = r3 / r1, (r3 / r1) * np.hypot(s3 / r3, s1 / r1)
    print("x1.005: ratio of means %.5f +- %.5f" % (rom, rom_se))
    assert not abs(rom - 1.0) < 4.0 * rom_se + 2e-4
