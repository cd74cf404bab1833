"""The grid MultiSensor's camera layouts against an independent numpy restatement.

Oracle and device both consume the host's view table, so the bit-identity tests cannot see an error in it.
These CPU tests restate src/sensors/grid.cpp:84-226 (the cone / cam_dir / cam_end layouts, cam_off with its
negated y and z, the sub-sensor transform built by editing row 3 of `to_world.inverse_transpose`) and the lens
shift of perspective.cpp:173-198 / thinlens.cpp:189-196 (`camera_to_sample.entry(0, 2) += lens_shift`) in numpy,
with the reference's types for the layout scalars (float32 `dt`, `tan_off`, `offset`; float64 `shift` and
`fov_x`), and compare the host's view descriptors with it.  The matrix products and inverses are formed in
float64 here (the host forms them in float32 / a float64 cofactor inverse), so matrices compare to 2e-6.

Two properties pin the meaning as well as the arithmetic: in the cone layout the focus plane's centre projects
to every view's image centre (that is what the lens shift is for), and with reverse_x / reverse_y the quilt tile
(tx, ty) holds view (gx-1-tx) + gx (gy-1-ty) (grid.cpp:243-251, via the oracle's primary hits).
"""
import os

import numpy as np
import pytest

from conftest import SCENES

CONE = os.path.join(SCENES, "cbox_cone.xml")
F32 = np.float32


def _look_at(origin, target, up):
    """Transform4f::look_at (transform.h:273-301): matrix and inverse_transpose, float32"""
    o, t, u = (np.asarray(v, F32) for v in (origin, target, up))
    d = (t - o) / np.sqrt(F32(np.dot(t - o, t - o)))
    left = np.cross(u, d).astype(F32)
    left = left / np.sqrt(F32(np.dot(left, left)))
    nu = np.cross(d, left).astype(F32)
    M = np.eye(4, dtype=np.float64)
    M[:3, 0], M[:3, 1], M[:3, 2], M[:3, 3] = left, nu, d, o
    IT = np.eye(4, dtype=np.float64)   # inverse transpose: rows 0..2 = (left | up | dir) columns, row 3 = -R^T o
    IT[:3, 0], IT[:3, 1], IT[:3, 2] = left, nu, d
    IT[3, :3] = [-np.dot(left, o), -np.dot(nu, o), -np.dot(d, o)]
    IT[:3, 3] = 0.0
    return M, IT


def _layout(n, foc, fov_x, cone=None, cam_dir=None, cam_dist=None, cam_center=True, cam_end=None, cam_off=(0, 0, 0),
            look=((0, 0, 3.9), (0, 0, 0), (0, 1, 0))):
    """grid.cpp:84-226 -> per view (to_world, to_world_inv, lens_shift)"""
    M, IT = _look_at(*look)
    off = np.array(cam_off, F32)
    off[1], off[2] = -off[1], -off[2]
    if cam_end is not None:
        beg = M[:3, 3].astype(F32)
        d = np.linalg.inv(M)[:3, :3] @ (np.asarray(cam_end, F32) - beg)   # to_world.inverse() * (end - beg)
        cam_dist = F32(np.linalg.norm(d))
        cam_dir = (d / cam_dist).astype(F32)
        cam_center = False
    elif cam_dir is not None:
        cam_dir = np.asarray(cam_dir, F32)
        cam_dist = F32(np.linalg.norm(cam_dir)) if cam_dist is None else F32(cam_dist)
    out = []
    for i in range(n):
        dt = F32(i) / F32(n - 1)
        it = IT.copy()
        shift = 0.0
        if cone is not None:
            tan_off = F32(np.tan(np.float64(F32((dt - F32(0.5)) * F32(F32(cone) * F32(np.pi / 180.0))))))
            offset = F32(F32(foc) * tan_off)
            shift = 0.5 * float(tan_off) / np.tan(np.deg2rad(fov_x) * 0.5)
            it[3, 0] = F32(F32(it[3, 0]) + F32(offset + off[0]))
            it[3, 1] = F32(F32(it[3, 1]) + off[1])
            it[3, 2] = F32(F32(it[3, 2]) + off[2])
        else:
            f = F32(cam_dist * F32(dt - F32(0.5) * F32(cam_center)))
            o = (off + cam_dir * f).astype(F32)
            for k in range(3):
                it[3, k] = F32(F32(it[3, k]) + o[k])
        inv = it.T                     # the new to_world's inverse (world -> camera)
        out.append((np.linalg.inv(inv), inv, shift))
    return out


def _views(scene):
    sd, vd, p = scene.describe(0, 0, 0)
    V = []
    for i in range(p.n_views):
        v = vd[i]
        V.append(dict(tw=np.array(v.to_world[:], np.float64).reshape(4, 4),
                      twi=np.array(v.to_world_inv[:], np.float64).reshape(4, 4),
                      c2s=np.array(v.camera_to_sample[:], np.float64).reshape(4, 4), res=tuple(v.resolution)))
    return sd, vd, p, V


def _check_layout(amvpt_mod, scene, expect, fov_x):
    sd, vd, p, V = _views(scene)
    assert len(V) == len(expect)
    w, h = (int(x) for x in V[0]["res"])
    base = amvpt_mod.perspective_projection((w, h), (w, h), (0, 0), fov_x, 0.001, 100.0).astype(np.float64)
    for i, (v, (tw, twi, shift)) in enumerate(zip(V, expect)):
        assert np.allclose(v["twi"], twi, rtol=0, atol=2e-6), (i, v["twi"], twi)
        assert np.allclose(v["tw"], tw, rtol=0, atol=2e-6), (i, v["tw"], tw)
        c2s = base.copy()
        c2s[0, 2] = F32(F32(base[0, 2]) + F32(shift))
        assert np.allclose(v["c2s"], c2s, rtol=2e-7, atol=0), (i, v["c2s"], c2s)
        assert np.isclose(v["c2s"][0, 2] - base[0, 2], shift, rtol=1e-5, atol=1e-7), (i, shift)
    return p, V


@pytest.mark.parametrize("cam", ["perspective", "thinlens"])
@pytest.mark.parametrize("off", [(0, 0, 0), (0.05, 0.1, -0.2)], ids=["no_off", "cam_off"])
def test_cone_layout_matches_restatement(amvpt_mod, cam, off):
    """cone_deg (grid.cpp:108-112,182-205): camera-space x offset focus * tan_off, lens_shift tan_off / (2 tan(fov/2))"""
    s = amvpt_mod.load_file(CONE, res=32, spp=16, cam=cam, cone=12, offx=off[0], offy=off[1], offz=off[2])
    expect = _layout(8, 3.9, 39.3077, cone=12.0, cam_off=off)
    assert max(abs(e[2]) for e in expect) > 0.1   # the shift is large, not a rounding residue
    _check_layout(amvpt_mod, s, expect, 39.3077)


def test_cone_layout_converges_on_the_focus_plane(amvpt_mod):
    """The lens shift's purpose: every view of a cone grid images the focus plane's centre (here the world origin,
    3.9 in front of the grid's camera) at its own image centre."""
    s = amvpt_mod.load_file(CONE, res=32, spp=16, cone=20)
    _, _, p, V = _views(s)
    for i, v in enumerate(V):
        cam = v["twi"] @ np.array([0.0, 0.0, 0.0, 1.0])
        scr = v["c2s"] @ cam
        uv = scr[:2] / scr[3]
        assert np.allclose(uv, [0.5, 0.5], atol=2e-6), (i, uv)
    # without the shift (a plain cam_dir line of the same offsets) the origin would leave the centre
    xs = [(v["twi"] @ [0, 0, 0, 1.0])[0] for v in V]
    assert np.ptp(xs) > 1.0


def test_cam_end_and_cam_dir_layouts_match_restatement(amvpt_mod):
    """cam_end (grid.cpp:119-126: the camera-space direction to the end point, cam_center off) and cam_dir with
    cam_center false and cam_off (grid.cpp:113-118,131-133,207-217)."""
    xml = open(CONE).read()
    line = '<float name="cone_deg" value="$cone"/>'
    assert line in xml
    end = amvpt_mod.load_string(xml.replace(line, '<vector name="cam_end" value="0.6, 0.3, 3.5"/>'), res=32, spp=16,
                                offx=0.02, offy=-0.05, offz=0.1)
    _check_layout(amvpt_mod, end, _layout(8, 3.9, 39.3077, cam_end=(0.6, 0.3, 3.5), cam_off=(0.02, -0.05, 0.1)),
                  39.3077)
    d = amvpt_mod.load_string(xml.replace(line, '<vector name="cam_dir" value="0, 1, 0.5"/><float name="cam_dist" '
                                                'value="0.3"/><boolean name="cam_center" value="false"/>'),
                              res=32, spp=16, offx=0.1)
    _check_layout(amvpt_mod, d, _layout(8, 3.9, 39.3077, cam_dir=(0, 1, 0.5), cam_dist=0.3, cam_center=False,
                                        cam_off=(0.1, 0, 0)), 39.3077)


@pytest.mark.parametrize("revx,revy", [(False, True), (True, True), (True, False), (False, False)])
def test_reverse_axes_place_views_in_the_quilt(amvpt_mod, oracle, revx, revy):
    """sample_ray_idx (grid.cpp:269-297): quilt tile (tx, ty) is rendered by view (tx' + gx ty') with tx' = gx-1-tx
    under reverse_x and ty' = gy-1-ty under reverse_y (the oracle's primary hits carry the view index)."""
    s = amvpt_mod.load_file(CONE, res=8, spp=16, revx=str(revx).lower(), revy=str(revy).lower())
    sd, vd, p = s.describe(0, 0, 0)
    assert (p.reverse_x, p.reverse_y) == (int(revx), int(revy))
    hits = oracle.primary_hits(sd, vd, p)
    view = hits[..., 7].astype(int)
    for ty in range(p.grid_y):
        for tx in range(p.grid_x):
            vx = p.grid_x - 1 - tx if revx else tx
            vy = p.grid_y - 1 - ty if revy else ty
            tile = view[ty * 8:(ty + 1) * 8, tx * 8:(tx + 1) * 8]
            assert (tile == vx + p.grid_x * vy).all(), (tx, ty, np.unique(tile))
