"""GPU parity: the HIP pipeline (through the C-ABI) against the CPU oracle.

Bar (DESIGN.md "Parity"): every per-lane, per-view ImageBlock::put record
(position, RGB value, alpha, weight, validity) is bit-identical to the
oracle's on the same seeds; the accumulated film agrees to float-atomic
reordering (relative 1e-5 of the film's scale); sharded lane ranges sum to the
full frame.  Sizes are chosen so the oracle finishes in seconds.
"""
import os

import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu

CBOX = os.path.join(SCENES, "cbox_grid.xml")
CBOX_PATH = os.path.join(SCENES, "cbox_path.xml")


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def _gpu_render(amvpt_mod, sd, vd, p, plan, lane_begin=0, lane_end=None, records=True, flags=0, record_pass=0):
    """One frame through amvpt_render_ex (per-call options; records of pass 0 through the opts hook)."""
    torch = _torch()
    dev = amvpt_mod.DeviceScene(sd)
    C = 5 if p.film_alpha else 4
    lane_end = plan["lanes"] if lane_end is None else lane_end
    film = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda")
    rec = None
    if records:
        rec = torch.zeros((lane_end - lane_begin, plan["group"], 8), dtype=torch.float32, device="cuda")
    dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt_mod.LaneSet(lane_begin, lane_end, 0, 0, 0, 0), flags=flags,
                  records_ptr=rec.data_ptr() if rec is not None else None, record_pass=record_pass)
    torch.cuda.synchronize()
    return film.cpu().numpy(), (rec.cpu().numpy() if rec is not None else None)


def _bit_equal(a, b):
    return (a == b) | (np.isnan(a) & np.isnan(b))


def _check(amvpt_mod, oracle, scene, seed=0, spp=0, min_match=1.0, flags=0, record_pass=0, film_tol=1e-5):
    """film_tol=0: the deterministic film (AMVPT_OPT_DETERMINISTIC) against the oracle's fixed-point film,
    bit for bit (both sum the same 2^-32-rounded cell adds as integers, so the order of the sums is moot)."""
    sd, vd, p = scene.describe(0, seed, spp)
    plan = oracle.plan(p)
    if film_tol == 0:
        flags |= amvpt_mod.OPT_DETERMINISTIC
    gfilm, grec = _gpu_render(amvpt_mod, sd, vd, p, plan, flags=flags, record_pass=record_pass)
    ofilm, orec, _ = oracle.render(sd, vd, p, threads=16, record_pass=record_pass, fixed_film=film_tol == 0)
    eq = _bit_equal(grec, orec)
    match = eq.all(axis=(1, 2)).mean()
    if match < min_match:
        bad = np.argwhere(~eq.all(axis=(1, 2)))[:5, 0]
        for lane in bad:
            print("lane", lane, "\ngpu", grec[lane], "\noracle", orec[lane])
    assert match >= min_match, "lane records: %.6f bit-identical" % match
    if film_tol == 0:
        assert _bit_equal(gfilm, ofilm).all(), "deterministic film: %d floats differ" % (~_bit_equal(gfilm, ofilm)).sum()
        return gfilm, ofilm
    scale = np.abs(ofilm).max()
    err = np.abs(gfilm - ofilm).max() / scale
    assert err < film_tol, "film max relative difference %.3e" % err
    return gfilm, ofilm


def test_mvpath_single_view_reuse_off(gpu_ready, amvpt_mod, oracle):
    """G = 1 (render_sample / sample_single), 4-view grid, 16 spp."""
    s = amvpt_mod.load_file(CBOX, res=48, spp=16, reuse=1)
    _check(amvpt_mod, oracle, s)


def test_mvpath_amvpt_mis_g4(gpu_ready, amvpt_mod, oracle):
    """C2 shape at reduced size: 4 views, reuse 4, sa_mis (camera selection + MIS weights)."""
    s = amvpt_mod.load_file(CBOX, res=48, spp=16)
    _check(amvpt_mod, oracle, s)


def test_mvpath_amvpt_mis_g8_two_passes(gpu_ready, amvpt_mod, oracle):
    """M shape at reduced size: 8 views (4x2 grid), reuse 8, 32 spp in 2 passes of 16."""
    s = amvpt_mod.load_file(CBOX, res=24, spp=32, gx=4, gy=2, reuse=8)
    sd, vd, p = s.describe(0, 0, 0)
    assert oracle.plan(p)["passes"] == 2
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("res,spp,kw", [(48, 16, dict()), (24, 32, dict(gx=4, gy=2, reuse=8))])
def test_generic_kernels_on_diffuse_scene(gpu_ready, amvpt_mod, oracle, res, spp, kw):
    """The Cornell box is all-diffuse, so it normally runs the kDiff kernel instances;
    AMVPT_OPT_GENERIC_KERNELS (a per-call option) forces the generic ones, which must agree just as well."""
    s = amvpt_mod.load_file(CBOX, res=res, spp=spp, **kw)
    _check(amvpt_mod, oracle, s, flags=amvpt_mod.OPT_GENERIC_KERNELS)


@pytest.mark.parametrize("defines", [dict(rfilter="box"), dict(spp=24)], ids=["box_filter", "spp24"])
def test_block_window_splat(gpu_ready, amvpt_mod, oracle, defines):
    """The block-window splat (box filter, or spp per pass not a power of two): its put has block
    barriers, so the all-diffuse kernels skip a view only when no lane of the whole block splats it."""
    kw = dict(res=24, spp=32, gx=4, gy=2, reuse=8)
    kw.update(defines)
    _check(amvpt_mod, oracle, amvpt_mod.load_file(CBOX, **kw))


def test_mvpath_reuse_without_mis(gpu_ready, amvpt_mod, oracle):
    s = amvpt_mod.load_file(CBOX, res=48, spp=16, sa_mis="false")
    _check(amvpt_mod, oracle, s)


def test_mvpath_fast_mis(gpu_ready, amvpt_mod, oracle):
    s = amvpt_mod.load_file(CBOX, res=48, spp=16, fast_mis="true")
    _check(amvpt_mod, oracle, s)


def test_mvpath_seed_and_odd_spp(gpu_ready, amvpt_mod, oracle):
    """Non-power-of-two spp per pass (idx / spp division path) and a non-zero seed."""
    s = amvpt_mod.load_file(CBOX, res=32, spp=12, spp_pass_lim=6)
    _check(amvpt_mod, oracle, s, seed=7)


@pytest.mark.parametrize("res", [64, 256], ids=["res64", "c1_full_256"])
def test_path_integrator_c1(gpu_ready, amvpt_mod, oracle, res):
    """C1: stock `path` on a single perspective camera; 256^2 at 16 spp is BASELINE's config itself."""
    s = amvpt_mod.load_file(CBOX_PATH, res=res, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    assert (p.film_width, p.film_height, amvpt_mod.plan(p)[0]) == (res, res, 16)
    _check(amvpt_mod, oracle, s)


def _records(amvpt_mod, oracle, sd, vd, p, flags):
    torch = _torch()
    plan = oracle.plan(p)
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    rec = torch.zeros((plan["lanes"], plan["group"], 8), dtype=torch.float32, device="cuda")
    dev.render_ex(vd, p, film.data_ptr(), flags=flags, records_ptr=rec.data_ptr())
    torch.cuda.synchronize()
    return rec.cpu().numpy()


FAR_FLOOR = ('<rotate x="1" angle="-90"/>\n            <translate y="-1"/>',
             '<scale x="9" y="9"/><rotate x="1" angle="-90"/>\n            <translate y="-1"/>')


@pytest.mark.parametrize("case", ["grazing_top_face", "m_shape", "far_floor"])
def test_box_screen_keeps_records(gpu_ready, amvpt_mod, oracle, case):
    """The brute-force walks screen the Cornell cubes (box meshes) per lane and test only the faces a ray can
    reach (dgeom.h box_walk).  Its records must equal the full scan's (AMVPT_OPT_NO_BOX_SCREEN) bit for bit on
    large frames: a camera level with the small cube's top face (y = -0.4), whose camera rays graze that face
    and its edges, at 128^2 x 16 spp (the stock path tracer, max_depth 8: the bounces hit every face at every
    angle), and the config-M shape (8 views, G = 8) at 64^2 x 16 spp; plus the first against the oracle."""
    if case == "grazing_top_face":
        xml = open(CBOX_PATH).read().replace('origin="0, 0, 3.90" target="0, 0, 0"', 'origin="0, -0.4, 3.9" target="0, -0.4, 0"')
        assert 'origin="0, -0.4, 3.9"' in xml
        s = amvpt_mod.load_string(xml, res=128, spp=16)
    elif case == "far_floor":
        # a floor 18 units wide out of the room's open front, seen from a raised camera: suffix rays
        # start up to ~9 units from the cubes (box-space origins ~30), still under the scene-extent conditioning
        # bound (cond 3.3 x (1 + 9) < 100), so the cubes stay screened
        xml = open(CBOX_PATH).read().replace(*FAR_FLOOR).replace('origin="0, 0, 3.90"', 'origin="0, 2.5, 6.5"')
        assert 'scale x="9"' in xml and 'origin="0, 2.5, 6.5"' in xml
        s = amvpt_mod.load_string(xml, res=128, spp=16)
        assert amvpt_mod.scene_box_count(s) == 2
    else:
        s = amvpt_mod.load_file(CBOX, res=64, spp=16, gx=4, gy=2, reuse=8)
    sd, vd, p = s.describe(0, 0, 0)
    a = _records(amvpt_mod, oracle, sd, vd, p, 0)
    b = _records(amvpt_mod, oracle, sd, vd, p, amvpt_mod.OPT_NO_BOX_SCREEN)
    eq = _bit_equal(a, b).all(axis=(1, 2))
    assert eq.all(), "%d of %d lanes differ with the box screen" % ((~eq).sum(), eq.size)
    if case == "grazing_top_face":
        _check(amvpt_mod, oracle, amvpt_mod.load_string(xml, res=48, spp=16))


def _path_with_samples_per_pass(amvpt_mod, n, **defines):
    xml = open(CBOX_PATH).read().replace('<integrator type="path">',
                                         '<integrator type="path"><integer name="samples_per_pass" value="%d"/>' % n)
    return amvpt_mod.load_string(xml, **defines)


@pytest.mark.parametrize("spp,per_pass,record_pass", [(16, 4, 3), (12, 6, 1), (8, 1, 5)])
def test_path_passes_continue_the_sampler(gpu_ready, amvpt_mod, oracle, spp, per_pass, record_pass):
    """The stock path integrator split into passes (samples_per_pass, the same mechanism as its split of a
    frame above 2^32 - 1 samples, integrator.cpp:137-146,249-330): the sampler is seeded once and every pass
    continues each lane's PCG32 stream, so the records of a later pass are bit-identical to the oracle's
    only if the states are carried (rng_in / rng_out)."""
    s = _path_with_samples_per_pass(amvpt_mod, per_pass, res=32, spp=spp)
    sd, vd, p = s.describe(0, 0, 0)
    assert p.spp_pass_lim == per_pass and oracle.plan(p)["passes"] == spp // per_pass
    gfilm, ofilm = _check(amvpt_mod, oracle, s, record_pass=record_pass)
    # the whole frame: the same estimator as one pass of spp samples would be, different samples
    one = amvpt_mod.load_file(CBOX_PATH, res=32, spp=spp)
    sd1, vd1, p1 = one.describe(0, 0, 0)
    f1, _ = _gpu_render(amvpt_mod, sd1, vd1, p1, oracle.plan(p1), records=False)
    assert not np.array_equal(f1, gfilm)
    w, w1 = gfilm[..., -1].sum(), f1[..., -1].sum()
    assert abs(w / w1 - 1) < 2e-2   # splat weights: spp samples per pixel either way


def test_path_passes_on_two_chunk_streams(gpu_ready, amvpt_mod, oracle):
    """with the per-lane walk (no fused suffix) a multi-chunk pass alternates two chunk
    streams; an odd chunk count per pass (4096 lanes in chunks of 1400: 3) puts chunk c of pass p+1 on the
    other stream than chunk c of pass p, so the sampler-state planes are ordered only by the join at every pass
    boundary.  Records of the last pass and the film must still match the oracle."""
    s = _path_with_samples_per_pass(amvpt_mod, 4, res=32, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    plan = oracle.plan(p)
    assert plan["passes"] == 4 and plan["lanes"] == 4096
    torch = _torch()
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    rec = torch.zeros((plan["lanes"], plan["group"], 8), dtype=torch.float32, device="cuda")
    dev.render_ex(vd, p, film.data_ptr(), chunk_lanes=1400, traversal=2, records_ptr=rec.data_ptr(), record_pass=3)
    torch.cuda.synchronize()
    ofilm, orec, _ = oracle.render(sd, vd, p, threads=16, record_pass=3)
    assert _bit_equal(rec.cpu().numpy(), orec).all()
    gfilm = film.cpu().numpy()
    assert np.abs(gfilm - ofilm).max() / np.abs(ofilm).max() < 1e-5


@pytest.mark.parametrize("scene,defines", [
    ("cbox_path.xml", dict(res=64, spp=16, crop_w=40, crop_h=24, crop_x=10, crop_y=30)),
    ("cbox_batch.xml", dict(res=32, width=128, spp=16, crop_w=64, crop_h=16, crop_x=32, crop_y=8)),
], ids=["path_c1", "batch_mvpath"])
def test_crop_window(gpu_ready, amvpt_mod, oracle, scene, defines):
    """hdrfilm crop windows (hdrfilm.cpp:245-291; film.cpp:16-27,91-100): lanes span the crop, positions are
    film coordinates (+ crop_offset, mvpath.cpp:173-190), sample_ray_idx sees (pos - offset) / crop_size
    (mvpath_multi.h:12-16), ImageBlock::put subtracts the offset (imageblock.cpp:211,266,447) and a batch's
    reprojected views keep the full film's tile pitch; the single camera's projection includes the crop."""
    s = amvpt_mod.load_file(os.path.join(SCENES, scene), **defines)
    sd, vd, p = s.describe(0, 0, 0)
    assert (p.film_width, p.film_height, p.crop_offset_x, p.crop_offset_y) == (
        defines["crop_w"], defines["crop_h"], defines["crop_x"], defines["crop_y"])
    _check(amvpt_mod, oracle, s)


def test_sharded_lanes_sum_to_frame(gpu_ready, amvpt_mod, oracle):
    """Multi-GPU partitioning contract: lane ranges keep their global TEA seeds."""
    s = amvpt_mod.load_file(CBOX, res=32, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    plan = oracle.plan(p)
    L = plan["lanes"]
    full, _ = _gpu_render(amvpt_mod, sd, vd, p, plan, records=False)
    cuts = [0, L // 3, (2 * L) // 3 + 5, L]
    parts = sum(_gpu_render(amvpt_mod, sd, vd, p, plan, a, b, records=False)[0] for a, b in zip(cuts, cuts[1:]))
    err = np.abs(parts - full).max() / np.abs(full).max()
    assert err < 1e-5


def test_host_render_matches_oracle_develop(gpu_ready, amvpt_mod, oracle):
    """Integrator::render() through the host framework (develop=True) vs oracle develop()."""
    s = amvpt_mod.load_file(CBOX, res=32, spp=16)
    img = amvpt_mod.render(s)
    sd, vd, p = s.describe(0, 0, 0)
    ofilm, _, _ = oracle.render(sd, vd, p, threads=16)
    ref = oracle.develop(ofilm)
    rmse = float(np.sqrt(np.mean((img - ref) ** 2)))
    assert rmse < 1e-5, rmse


VEACH = os.path.join(SCENES, "veach_grid.xml")


def test_veach_mis_g8(gpu_ready, amvpt_mod, oracle):
    """C3 shape at reduced size: GGX rough conductors (tv_pdf MIS terms), twosided, sphere lights (f64 hit,
    cone sampling), 8 views, reuse 8, sa_mis."""
    s = amvpt_mod.load_file(VEACH, res=24, spp=16)
    _check(amvpt_mod, oracle, s)


def _cbox_spheres(amvpt_mod, **defines):
    """The Cornell box with its two cubes replaced by two large diffuse spheres and a small sphere light: the
    camera, visibility and suffix rays graze the silhouettes constantly, and the NEE rays toward the light
    end a ShadowEpsilon short of it -- the cases the f32 sphere screen and the deferred float64 tests decide."""
    import re
    xml = open(os.path.join(SCENES, "cbox_grid.xml")).read()
    xml = re.sub(r'<shape type="cube" id="small-box">.*?</shape>\s*<shape type="cube" id="large-box">.*?</shape>',
                 '<shape type="sphere"><point name="center" x="0.33" y="-0.6" z="0.3"/><float name="radius" value="0.4"/>'
                 '<ref id="white"/></shape>'
                 '<shape type="sphere"><point name="center" x="-0.35" y="-0.45" z="-0.3"/><float name="radius" value="0.55"/>'
                 '<ref id="white"/></shape>'
                 '<shape type="sphere"><point name="center" x="0.0" y="0.55" z="0.2"/><float name="radius" value="0.08"/>'
                 '<emitter type="area"><rgb name="radiance" value="20, 20, 20"/></emitter></shape>', xml, flags=re.S)
    assert xml.count('type="sphere"') == 3
    return amvpt_mod.load_string(xml, **defines)


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["auto_deferred", "wave_uniform_bvh", "per_lane_bvh"])
def test_sphere_grazing_rays(gpu_ready, amvpt_mod, oracle, mode):
    """Spheres under every walk: auto mode (brute-force suffix and wave-uniform coherent walks with the
    float64 tests deferred past the walk), the wave-uniform and the per-lane BVH walks (tested in place),
    all behind the f32 sphere screen (dgeom.h sphere_maybe) -- records bit-identical to the oracle."""
    amvpt_mod.set_traversal(mode)
    try:
        _check(amvpt_mod, oracle, _cbox_spheres(amvpt_mod, res=24, spp=16, gx=4, gy=2, reuse=8))
    finally:
        amvpt_mod.set_traversal(0)


@pytest.mark.parametrize("n_spheres", [64, 70], ids=["deferred_64", "in_place_70"])
def test_many_spheres(gpu_ready, amvpt_mod, oracle, n_spheres):
    """A field of small spheres in the Cornell box (with the two cubes): 64 spheres take the deferred float64
    tests of the wave-uniform walks (one 64-bit mask), 70 the in-place tests; the suffix walks the per-lane
    BVH with spheres -- records bit-identical to the oracle either way."""
    xml = open(os.path.join(SCENES, "cbox_grid.xml")).read()
    balls = []
    for i in range(n_spheres):
        x, y, z = -0.8 + 0.2 * (i % 9), -0.9 + 0.22 * ((i // 9) % 9), -0.6 + 0.45 * (i // 81)
        balls.append('<shape type="sphere"><point name="center" x="%.3f" y="%.3f" z="%.3f"/>'
                     '<float name="radius" value="0.07"/><ref id="white"/></shape>' % (x, y, z))
    xml = xml.replace("</scene>", "\n".join(balls) + "\n</scene>")
    s = amvpt_mod.load_string(xml, res=16, spp=16, gx=4, gy=2, reuse=8)
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("defines", [
    dict(distr="beckmann"),                                            # the reference's default model
    dict(distr="beckmann", vis="false"),
    dict(distr="beckmann", a3u=0.02, a3v=0.1, a4u=0.05, a4v=0.25),    # anisotropic, visible normals
    dict(distr="beckmann", vis="false", a3u=0.02, a3v=0.1, a4u=0.05, a4v=0.25),
    dict(distr="ggx", vis="false", a3u=0.02, a3v=0.1, a4u=0.05, a4v=0.25),
], ids=["beckmann_vis", "beckmann", "beckmann_vis_aniso", "beckmann_aniso", "ggx_aniso"])
def test_veach_microfacet_models(gpu_ready, amvpt_mod, oracle, defines):
    """roughconductor with Beckmann (exp eval, rational Smith G1, log elevation sampling, visible-normal
    sampling by erf / erfinv Newton inversion) and anisotropic non-visible sampling (tan azimuth
    inversion), microfacet.h:185-431: the device transcendentals are the oracle's operation for
    operation, so records stay bit-identical."""
    s = amvpt_mod.load_file(VEACH, res=24, spp=16, **defines)
    _check(amvpt_mod, oracle, s)


def test_veach_fast_mis_two_passes(gpu_ready, amvpt_mod, oracle):
    s = amvpt_mod.load_file(VEACH, res=16, spp=32, fast_mis="true")
    _check(amvpt_mod, oracle, s, seed=3)


def test_veach_single_view_g1(gpu_ready, amvpt_mod, oracle):
    s = amvpt_mod.load_file(VEACH, res=24, spp=16, reuse=1)
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("mode", [1, 2], ids=["wave_uniform_bvh", "per_lane_bvh"])
@pytest.mark.parametrize("scene", ["cbox", "veach"])
def test_bvh_walks_match(gpu_ready, amvpt_mod, oracle, scene, mode):
    """Auto mode brute-forces the suffix walks of these tiny scenes; the wave-uniform (mode 1) and
    per-lane (mode 2, large scenes) threaded-BVH walks must give the same records as the oracle."""
    amvpt_mod.set_traversal(mode)
    try:
        s = amvpt_mod.load_file(CBOX if scene == "cbox" else VEACH, res=24, spp=16, gx=4, gy=2, reuse=8)
        _check(amvpt_mod, oracle, s)
    finally:
        amvpt_mod.set_traversal(0)


@pytest.mark.parametrize("adaptive,extra", [(1, dict()), (3, dict(gx=4, gy=2, reuse=8, spp=32))])
def test_adaptive_fill(gpu_ready, amvpt_mod, oracle, adaptive, extra):
    """a13: adaptive fill (mvpath_multi.h:79-115) -- compaction in lane order, n_adapt re-traces per lane
    with the forked (wavefront, wavefront) sampler, non-coalesced splats of weight 1/(n_adapt+1)."""
    kw = dict(res=24, spp=16)
    kw.update(extra)
    s = amvpt_mod.load_file(CBOX, adaptive=adaptive, **kw)
    sd, vd, p = s.describe(0, 0, 0)
    assert p.adaptive == adaptive
    gf, of = _check(amvpt_mod, oracle, s)
    cnt = amvpt_mod.Counters()
    torch = _torch()
    film = torch.zeros_like(torch.from_numpy(gf)).cuda()
    amvpt_mod.DeviceScene(sd).render(vd, p, film.data_ptr(), counters=cnt)
    _, _, st = oracle.render(sd, vd, p, threads=16)
    assert cnt.adaptive_lanes == st["adaptive_lanes"] > 0


def test_adaptive_refuses_lane_shards_without_exchange(gpu_ready, amvpt_mod):
    s = amvpt_mod.load_file(CBOX, res=16, spp=16, adaptive=1)
    sd, vd, p = s.describe(0, 0, 0)
    torch = _torch()
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    amvpt_mod.set_adaptive_exchange(None)
    with pytest.raises(RuntimeError, match="amvpt_set_adaptive_exchange"):
        amvpt_mod.DeviceScene(sd).render(vd, p, film.data_ptr(), 0, 100)


def _counts_per_pass(render_range, shards, set_exchange):
    """Phase 1: each range's flagged-lane count per pass (the fill's output is discarded)."""
    counts = []
    for b, e in shards:
        got = []
        set_exchange(lambda local: (got.append(local), (0, local))[1])
        render_range(b, e)
        counts.append(got)
    set_exchange(None)
    return counts


def _exchange_from(counts, r):
    calls = iter(range(len(counts[0])))

    def fn(local):
        k = next(calls)
        assert local == counts[r][k]
        return sum(c[k] for c in counts[:r]), sum(c[k] for c in counts)
    return fn


def test_adaptive_lane_shards_with_exchange(gpu_ready, amvpt_mod, oracle):
    """C5's partition: adaptive > 0 over lane ranges, the fill's prefix/total supplied per pass by
    the host exchange (amvpt_set_adaptive_exchange); the ranges' films sum to the whole frame."""
    torch = _torch()
    s = amvpt_mod.load_file(CBOX, res=24, spp=32, gx=4, gy=2, reuse=4, adaptive=2)
    sd, vd, p = s.describe(0, 0, 0)
    plan = oracle.plan(p)
    assert plan["passes"] == 2
    n = plan["lanes"]
    shards = [(0, n // 3 + 5), (n // 3 + 5, 2 * n // 3 - 300), (2 * n // 3 - 300, n)]
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")

    def render_range(b, e):
        dev.render(vd, p, film.data_ptr(), b, e)
        torch.cuda.synchronize()
    counts = _counts_per_pass(render_range, shards, amvpt_mod.set_adaptive_exchange)
    assert all(len(c) == 2 for c in counts) and sum(counts[1]) > 0
    film.zero_()
    try:
        for r, (b, e) in enumerate(shards):
            amvpt_mod.set_adaptive_exchange(_exchange_from(counts, r))
            render_range(b, e)
    finally:
        amvpt_mod.set_adaptive_exchange(None)
    got = film.cpu().numpy()
    ref, _, st = oracle.render(sd, vd, p, threads=16)
    assert st["adaptive_lanes"] == 2 * sum(sum(c) for c in counts)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


BATCH = os.path.join(SCENES, "cbox_batch.xml")


@pytest.mark.parametrize("rev", ["false", "true"])
def test_batch_sensor(gpu_ready, amvpt_mod, oracle, rev):
    """`batch` MultiSensor (batch.cpp:163-181): strip layout, clamp-then-reverse view index."""
    s = amvpt_mod.load_file(BATCH, res=24, width=96, spp=16, rev=rev)
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("kw", [dict(res=32, spp=16), dict(res=32, spp=16, reuse=1), dict(res=24, spp=16, adaptive=1)],
                         ids=["g4_mis", "g1", "adaptive"])
def test_thinlens_views(gpu_ready, amvpt_mod, oracle, kw):
    """Thin-lens sub-sensors (thinlens.cpp:220-257,358-418): aperture sample drawn after the jitter
    and shared by every view's sample_surface; re-gathered by the adaptive fill."""
    s = amvpt_mod.load_file(CBOX, cam="thinlens", aperture="0.05", **kw)
    _check(amvpt_mod, oracle, s)


CONE = os.path.join(SCENES, "cbox_cone.xml")


@pytest.mark.parametrize("kw", [dict(), dict(cam="thinlens", aperture="0.05"),
                                dict(revx="true", offx=0.05, offy=0.1, offz=-0.2), dict(adaptive=3, revy="false")],
                         ids=["perspective", "thinlens", "revx_cam_off", "adaptive"])
def test_cone_layout_views(gpu_ready, amvpt_mod, oracle, kw):
    """The grid's light-field cone layout (grid.cpp:108-112,182-205): 8 views on a line, each with its own
    lens_shift in camera_to_sample (perspective.cpp:178-180, thinlens.cpp:195), so raygen, sensors_visible's
    reprojection and every Jacobian / film pdf of sample_surface see an off-axis projection; G = 8, sa_mis.
    The view table itself is pinned by tests/test_grid_layouts.py."""
    s = amvpt_mod.load_file(CONE, res=24, spp=16, **kw)
    sd, vd, p = s.describe(0, 0, 0)
    assert (p.n_views, p.reuse_count) == (8, 8)
    assert len({round(vd[i].camera_to_sample[2], 6) for i in range(8)}) == 8   # eight distinct lens shifts
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("film_tol", [1e-5, 0], ids=["float_film", "deterministic_film"])
def test_debug_mode_splats_the_adaptive_mask(gpu_ready, amvpt_mod, oracle, film_tol):
    """debug = true (mvpath_multi.h:54-56): each lane puts only its primary sample, with the adaptive mask as
    its value and weight 1, and the fill does not run; G = 8, adaptive 3.  Film against the oracle (the
    deterministic film bit for bit); the developed film is the local fraction of adaptive lanes."""
    line = '<integer name="adaptive" value="$adaptive"/>'
    xml = open(CBOX).read()
    assert line in xml
    s = amvpt_mod.load_string(xml.replace(line, line + '<boolean name="debug" value="true"/>'),
                              res=24, spp=32, gx=4, gy=2, reuse=8, adaptive=3)
    sd, vd, p = s.describe(0, 0, 0)
    assert p.debug == 1 and p.adaptive == 3
    gfilm, _ = _check(amvpt_mod, oracle, s, film_tol=film_tol)
    frac = gfilm[..., 0] / np.maximum(gfilm[..., -1], 1e-30)
    assert np.allclose(gfilm[..., 0], gfilm[..., 1]) and np.allclose(gfilm[..., 0], gfilm[..., 2])
    assert frac.min() >= 0.0 and frac.max() <= 1.0 + 1e-6
    assert 0.0 < frac.mean() < 1.0   # some lanes are adaptive, not all


MESH = os.path.join(SCENES, "cbox_mesh.xml")


def test_file_meshes_per_lane_bvh(gpu_ready, amvpt_mod, oracle):
    """OBJ (vertex normals + uv) and PLY (recomputed normals, rough conductor) meshes: 3.6k triangles, a
    BVH far above the wave-uniform limit, walked per lane from global memory."""
    s = amvpt_mod.load_file(MESH, res=16, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    n_nodes, n_prims = amvpt_mod.DeviceScene(sd).stats()
    assert n_nodes > 255 and n_prims == 6 + 1280 + 2304
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("kw", [dict(res=16, spp=16), dict(res=24, spp=16, gx=4, gy=2, reuse=8)], ids=["path_g1", "g8"])
def test_two_box_bvh_keeps_records(gpu_ready, amvpt_mod, oracle, kw):
    """The per-lane suffix walks of the 3.6 k-triangle mesh on the two-box BVH (dscene.h DNode2: both child boxes in
    a node, near-first by the ray's entry distances, a 16-entry LDS stack; dgeom.h trace_closest2 / trace_any2):
    records bit-identical to the oracle, binned and unbinned, and to the threaded walks (AMVPT_OPT_THREADED_BVH)."""
    s = amvpt_mod.load_file(MESH, **kw)
    sd, vd, p = s.describe(0, 0, 0)
    n2, depth = amvpt_mod.DeviceScene(sd).bvh2()
    print("two-box BVH: %d nodes, depth %d" % (n2, depth))
    assert n2 > 0 and 0 < depth <= 16
    _check(amvpt_mod, oracle, s)
    _check(amvpt_mod, oracle, s, flags=amvpt_mod.OPT_NO_BINNING)
    a = _records(amvpt_mod, oracle, sd, vd, p, 0)
    b = _records(amvpt_mod, oracle, sd, vd, p, amvpt_mod.OPT_THREADED_BVH)
    assert _bit_equal(a, b).all()


@pytest.mark.parametrize("kw", [dict(res=16, spp=16), dict(res=16, spp=16, gx=4, gy=2, reuse=8)], ids=["path_g1", "g8"])
def test_ray_binning_keeps_records(gpu_ready, amvpt_mod, oracle, kw):
    """Ray binning (k_bin_sort): the per-lane suffix walks of the 3.6 k-triangle mesh take each partition's
    extension and NEE rays in (direction octant, origin cell) order and write hits / verdicts back to the
    rays' entries.  Records are bit-identical to the oracle with binning (the default) and without it
    (AMVPT_OPT_NO_BINNING), and the binning kernel ran."""
    s = amvpt_mod.load_file(MESH, **kw)
    _check(amvpt_mod, oracle, s)
    _check(amvpt_mod, oracle, s, flags=amvpt_mod.OPT_NO_BINNING)
    torch = _torch()
    sd, vd, p = s.describe(0, 0, 0)
    dev = amvpt_mod.DeviceScene(sd)
    for flags, launched in [(0, True), (amvpt_mod.OPT_NO_BINNING, False)]:
        film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
        cnt = amvpt_mod.Counters()
        dev.render_ex(vd, p, film.data_ptr(), counters=cnt, flags=flags)
        torch.cuda.synchronize()
        assert (cnt.as_dict()["kernel_launches"]["k_bin"] > 0) == launched, flags


@pytest.mark.parametrize("chunk", [8192, 5000])
def test_many_chunks_per_pass(gpu_ready, amvpt_mod, oracle, chunk):
    """Many lane chunks per pass (the arena bound at full size): records stay bit-identical, the film
    equal up to atomic order.  5000 is not a multiple of the 1024-lane splat super-block (identity
    slot map at the seams)."""
    amvpt_mod.set_chunk_lanes(chunk)
    try:
        s = amvpt_mod.load_file(CBOX, res=24, spp=32, gx=4, gy=2, reuse=8)
        sd, vd, p = s.describe(0, 0, 0)
        assert oracle.plan(p)["lanes"] > 4 * chunk
        _check(amvpt_mod, oracle, s)
    finally:
        amvpt_mod.set_chunk_lanes(0)   # back to the automatic chunk


def test_two_chunk_streams(gpu_ready, amvpt_mod, oracle):
    """BVH scenes (per-depth wavefront suffix) take turns over up to four buffer sets on as many streams
    (16 chunks per pass here, so all four run): with many small chunks on every stream the records stay
    bit-identical to the oracle, as they are with every chunk on the render stream (AMVPT_OPT_ONE_STREAM)."""
    amvpt_mod.set_chunk_lanes(2048)
    try:
        s = amvpt_mod.load_file(MESH, res=16, spp=16, gx=4, gy=2, reuse=8)
        sd, vd, p = s.describe(0, 0, 0)
        assert oracle.plan(p)["lanes"] > 8 * 2048
        _check(amvpt_mod, oracle, s)
        _check(amvpt_mod, oracle, s, flags=amvpt_mod.OPT_ONE_STREAM)
    finally:
        amvpt_mod.set_chunk_lanes(0)


@pytest.mark.parametrize("scene", ["cbox", "mesh"])
def test_deterministic_film(gpu_ready, amvpt_mod, oracle, scene):
    """AMVPT_OPT_DETERMINISTIC: the splats are summed as 32.32 fixed point with integer atomics, so the
    film is bitwise identical across runs, chunk sizes and (mesh: two chunk streams) stream interleavings,
    and agrees with the float-atomic film and the oracle's film to float summation order."""
    torch = _torch()
    path = CBOX if scene == "cbox" else MESH
    s = amvpt_mod.load_file(path, res=16, spp=32, gx=4, gy=2, reuse=8)
    sd, vd, p = s.describe(0, 0, 0)
    plan = oracle.plan(p)
    dev = amvpt_mod.DeviceScene(sd)
    films = []
    for chunk, flags in [(0, amvpt_mod.OPT_DETERMINISTIC), (3000, amvpt_mod.OPT_DETERMINISTIC),
                         (0, amvpt_mod.OPT_DETERMINISTIC), (0, 0)]:
        film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
        cnt = amvpt_mod.Counters()
        dev.render_ex(vd, p, film.data_ptr(), chunk_lanes=chunk, flags=flags, counters=cnt)
        torch.cuda.synchronize()
        assert cnt.film_range_drops == 0
        films.append(film.cpu().numpy())
    assert _bit_equal(films[0], films[1]).all() and _bit_equal(films[0], films[2]).all()
    ofilm, _, _ = oracle.render(sd, vd, p, threads=16, record_pass=0)
    scale = np.abs(ofilm).max()
    assert np.abs(films[0] - films[3]).max() <= 1e-5 * scale
    assert np.abs(films[0] - ofilm).max() <= 1e-5 * scale
    # the oracle's fixed-point film (the same 2^-32-rounded cell adds, summed as integers): bit for bit
    xfilm, _, _ = oracle.render(sd, vd, p, threads=16, fixed_film=True)
    assert _bit_equal(films[0], xfilm).all()
    assert plan["lanes"] > 3000 * 4


def test_deterministic_film_counts_range_drops(gpu_ready, amvpt_mod, oracle):
    """a finite footprint-cell add of |v| >= 2^31 does not fit the 32.32 fixed-point film;
    it is dropped and counted (counters.film_range_drops), the count equal to the oracle's restatement of the
    same rule, and the rest of the film bit-identical to the oracle's fixed-point film.  A light of radiance
    1e12 seen directly makes such adds (1e12 x a filter weight); the float-atomic film keeps them."""
    torch = _torch()
    xml = open(CBOX_PATH).read().replace('value="18.387, 13.9873, 6.75357"', 'value="1e12, 1e12, 1e12"')
    s = amvpt_mod.load_string(xml, res=32, spp=4)
    sd, vd, p = s.describe(0, 0, 0)
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    cnt = amvpt_mod.Counters()
    dev.render_ex(vd, p, film.data_ptr(), flags=amvpt_mod.OPT_DETERMINISTIC, counters=cnt)
    torch.cuda.synchronize()
    xfilm, _, st = oracle.render(sd, vd, p, threads=16, fixed_film=True)
    assert st["range_drops"] > 0
    assert cnt.film_range_drops == st["range_drops"]
    assert _bit_equal(film.cpu().numpy(), xfilm).all()
    ffilm = torch.zeros_like(film)
    cnt2 = amvpt_mod.Counters()
    dev.render_ex(vd, p, ffilm.data_ptr(), counters=cnt2)
    torch.cuda.synchronize()
    assert cnt2.film_range_drops == 0 and ffilm.max().item() > 2.0 ** 31


def test_deterministic_film_needs_whole_window(gpu_ready, amvpt_mod):
    torch = _torch()
    s = amvpt_mod.load_file(CBOX, res=16, spp=16, gx=4, gy=2, reuse=8)
    sd, vd, p = s.describe(0, 0, 0)
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width // 2, 4), dtype=torch.float32, device="cuda")
    ov = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
    with pytest.raises(Exception, match="DETERMINISTIC"):
        dev.render_ex(vd, p, film.data_ptr(), window=(0, 0, p.film_width // 2, p.film_height),
                      overflow_ptr=ov.data_ptr(), overflow_capacity=1000, flags=amvpt_mod.OPT_DETERMINISTIC)


@pytest.mark.parametrize("gx,gy,reuse", [(4, 4, 16), (4, 3, 12)], ids=["g16", "g12"])
def test_large_view_groups(gpu_ready, amvpt_mod, oracle, gx, gy, reuse):
    """Group sizes above 8 (reuse_count = n_views = 12 or 16): camera selection over up to 15
    other views, G x (G-1) MIS pair terms, G splats per lane."""
    s = amvpt_mod.load_file(CBOX, res=16, spp=16, gx=gx, gy=gy, reuse=reuse)
    sd, vd, p = s.describe(0, 0, 0)
    assert oracle.plan(p)["group"] == reuse
    _check(amvpt_mod, oracle, s)


@pytest.mark.parametrize("scene,gx,gy,reuse,res", [
    ("cbox_grid.xml", 8, 4, 32, 12),    # the C5 light-field array as ONE group of 32 views
    ("cbox_grid.xml", 8, 8, 64, 8),     # 64 views: per-view state past 64 KB of LDS -> global plane
    ("veach_grid.xml", 5, 4, 20, 12),   # glossy: per-view BSDF sampling + G x (G-1) BSDF pdfs
    ("cbox_grid.xml", 16, 8, 128, 6),   # 128 views: masks beyond one 64-bit word
    ("cbox_grid.xml", 16, 16, 256, 4),  # 256 views: the largest group (four mask words)
    ("veach_grid.xml", 10, 8, 80, 6),   # glossy, 80 views, global per-view state
    ("cbox_grid.xml", 32, 16, 512, 2),  # 512 views: the 1024-bit instance (G = -1), a 32 x 16 light field
], ids=["cbox_g32", "cbox_g64", "veach_g20", "cbox_g128", "cbox_g256", "veach_g80", "cbox_g512"])
def test_groups_above_16_views(gpu_ready, amvpt_mod, oracle, scene, gx, gy, reuse, res):
    """Groups of 17..1024 views (the reference has no cap,
    mvpath.cpp:192-217): the runtime group-size instances with 256- / 1024-bit view masks (WMask<4>,
    WMask<16> in the vreq_w / lmask_w planes), 16-wave k_vis blocks walking several slots each, 64-thread
    k_mv_primary blocks whose per-view state leaves LDS for a global plane past 64 KB."""
    s = amvpt_mod.load_file(os.path.join(SCENES, scene), res=res, spp=16, gx=gx, gy=gy, reuse=reuse)
    sd, vd, p = s.describe(0, 0, 0)
    assert oracle.plan(p)["group"] == reuse
    # film: the records are bit-identical; the f32 film sums differ only in order.  At 512 views of 2 x 2 px
    # every film cell sums ~8192 splats (512 x 4 x 16 lanes into 4 cells per view), whose f32 summation order
    # alone moves a cell by up to 8192 x 2^-24 = 4.9e-4 relative (measured 2.3e-5, r04a), so a float-film
    # comparison could not stay at 1e-5.  Instead the G > 256 case compares the deterministic film with the
    # oracle's fixed-point film: both sum the same 2^-32-rounded cell adds as integers, so the order does not
    # matter and the films must be EQUAL (tolerance 0).  The smaller groups sum <= 4096 per cell and keep 1e-5.
    _check(amvpt_mod, oracle, s, film_tol=0 if reuse > 256 else 1e-5)


def test_group_above_1024_views_refused(gpu_ready, amvpt_mod):
    """Groups past 1024 views (sixteen mask words; over a million MIS pair terms per lane) fail loudly
    instead of rendering wrong."""
    torch = _torch()
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=1, spp=16, gx=33, gy=32, reuse=1056)
    sd, vd, p = s.describe(0, 0, 0)
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    with pytest.raises(Exception, match="1024"):
        dev.render(vd, p, film.data_ptr())


CBOX_ENV = os.path.join(SCENES, "cbox_env.xml")
VEACH_W = os.path.join(SCENES, "veach_grid.xml")


@pytest.mark.parametrize("defines", [
    dict(res=48, spp=16),                          # G = 4, area light + constant, uniform picking
    dict(res=48, spp=16, lw=3, ew=0.5),            # non-uniform emitter sampling (DiscreteDistribution)
    dict(res=32, spp=16, reuse=1),                 # G = 1 (render_sample / sample_single)
    dict(res=24, spp=32, gx=4, gy=2, reuse=8, ew=0.25, adaptive=3),
], ids=["g4_uniform", "g4_weighted", "g1", "g8_weighted_adaptive"])
def test_constant_environment_emitter(gpu_ready, amvpt_mod, oracle, defines):
    """`constant` environment emitter (constant.cpp): escaped rays see its radiance (valid alpha,
    mvpath_multi.h:140), emitter sampling picks it among the area light with the uniform-sphere
    direction and a shadow ray past the scene's bounding sphere, emitter-hit MIS uses 1/(4 pi)."""
    s = amvpt_mod.load_file(CBOX_ENV, **defines)
    _check(amvpt_mod, oracle, s)


def test_constant_environment_hidden(gpu_ready, amvpt_mod, oracle):
    """hide_emitters: escaped camera rays stay invalid (alpha 0) but still carry the emission."""
    s = amvpt_mod.load_file(CBOX_ENV, res=32, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    p.hide_emitters = 1
    plan = oracle.plan(p)
    gfilm, grec = _gpu_render(amvpt_mod, sd, vd, p, plan)
    ofilm, orec, _ = oracle.render(sd, vd, p, threads=16, record_pass=0)
    assert _bit_equal(grec, orec).all()
    assert np.abs(gfilm - ofilm).max() / np.abs(ofilm).max() < 1e-5


def test_veach_weighted_emitter_sampling(gpu_ready, amvpt_mod, oracle):
    """Non-uniform `sampling_weight`s on the four sphere lights (scene.cpp:100-119, 222-244;
    distr_1d.h:116-215): binary search over the float CDF, re-used sample, pmf = weight / sum."""
    s = amvpt_mod.load_file(VEACH_W, res=24, spp=16, w0=0.25, w1=1, w2=2.5, w3=4)
    _check(amvpt_mod, oracle, s)


SMALL_MESHLIGHT = dict(ball_file="meshes/quad_fan.obj", ring_type="obj", ring_file="meshes/quad_fan.obj")


@pytest.mark.parametrize("scene,adaptive", [("cbox", 0), ("cbox", 2), ("meshlight", 0)])
def test_fused_suffix_matches_wavefront_suffix(gpu_ready, amvpt_mod, oracle, scene, adaptive):
    """k_suffix_fused (paths in registers, brute-force scenes) vs the per-depth k_extend / k_bounce
    wavefronts (AMVPT_OPT_WAVEFRONT_SUFFIX) on the same lanes: records bit-identical, the same vertex and
    shadow-ray counts, and each launch path actually taken (kernel launch counters).  `meshlight`: the
    27-primitive mesh-light box (a 12-triangle cube light and a 5-triangle polygon mesh light), so the
    fused suffix samples and prices mesh emitters (Mesh::sample_position, mesh.cpp:765-816)."""
    torch = _torch()
    if scene == "meshlight":
        s = amvpt_mod.load_file(MESHLIGHT, res=32, spp=32, gx=4, gy=2, reuse=8, **SMALL_MESHLIGHT)
    else:
        s = amvpt_mod.load_file(CBOX, res=32, spp=32, gx=4, gy=2, reuse=8, adaptive=adaptive)
    sd, vd, p = s.describe(0, 0, 0)
    plan = oracle.plan(p)
    out = {}
    for fused in ("1", "0"):
        flags = 0 if fused == "1" else amvpt_mod.OPT_WAVEFRONT_SUFFIX
        dev = amvpt_mod.DeviceScene(sd)
        film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
        rec = torch.zeros((plan["lanes"], plan["group"], 8), dtype=torch.float32, device="cuda")
        dev.render_ex(vd, p, film.data_ptr(), flags=flags, records_ptr=rec.data_ptr())
        cnt = amvpt_mod.Counters()
        film2 = torch.zeros_like(film)
        dev.render_ex(vd, p, film2.data_ptr(), counters=cnt, flags=flags)
        torch.cuda.synchronize()
        out[fused] = (rec.cpu().numpy(), film2.cpu().numpy(), cnt.as_dict())
    (r1, f1, c1), (r0, f0, c0) = out["1"], out["0"]
    assert c1["kernel_launches"]["k_suffix"] > 0 and c1["kernel_launches"]["k_extend"] == 0
    assert c0["kernel_launches"]["k_suffix"] == 0 and c0["kernel_launches"]["k_extend"] > 0
    for k in ("vertices", "shadow_rays", "lanes", "adaptive_lanes", "view_splats"):
        assert c1[k] == c0[k], k
    assert _bit_equal(r1, r0).all()
    assert np.abs(f1 - f0).max() <= 1e-5 * np.abs(f0).max()


def test_mesh_scene_keeps_wavefront_suffix(gpu_ready, amvpt_mod):
    """Scenes above the brute-force size (the 3.6 k-triangle mesh box) run the per-depth suffix."""
    torch = _torch()
    s = amvpt_mod.load_file(MESH, res=16, spp=16, gx=4, gy=2, reuse=8)
    sd, vd, p = s.describe(0, 0, 0)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    cnt = amvpt_mod.Counters()
    amvpt_mod.DeviceScene(sd).render(vd, p, film.data_ptr(), counters=cnt)
    torch.cuda.synchronize()
    d = cnt.as_dict()
    assert d["kernel_launches"]["k_suffix"] == 0 and d["kernel_launches"]["k_extend"] > 0


MESHLIGHT = os.path.join(SCENES, "cbox_meshlight.xml")


@pytest.mark.parametrize("defines", [
    dict(res=32, spp=16),                               # G = 4, two mesh lights, uniform picking
    dict(res=24, spp=16, gx=4, gy=2, reuse=8),          # G = 8
    dict(res=24, spp=16, reuse=1),                      # G = 1 (render_sample)
], ids=["g4", "g8", "g1"])
def test_mesh_area_emitters(gpu_ready, amvpt_mod, oracle, defines):
    """Area emitters on meshes: Mesh::sample_position (mesh.cpp:765-816) picks a face from the
    float area CDF with DiscreteDistribution::sample_reuse and a uniform barycentric point
    (interpolated vertex normal on the icosphere, face normal on the flat cube);
    Shape::pdf_direction (shape.cpp:379-390) prices emitter hits by 1 / surface area."""
    s = amvpt_mod.load_file(MESHLIGHT, **defines)
    _check(amvpt_mod, oracle, s)


def test_small_mesh_light_scene_takes_fused_suffix(gpu_ready, amvpt_mod, oracle):
    """The 27-primitive mesh-light box runs the brute-force walks and k_suffix_fused (launch counters)
    and its lane records are bit-identical to the oracle's."""
    torch = _torch()
    s = amvpt_mod.load_file(MESHLIGHT, res=24, spp=16, gx=4, gy=2, reuse=8, **SMALL_MESHLIGHT)
    sd, vd, p = s.describe(0, 0, 0)
    dev = amvpt_mod.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    cnt = amvpt_mod.Counters()
    dev.render_ex(vd, p, film.data_ptr(), counters=cnt)
    torch.cuda.synchronize()
    c = cnt.as_dict()
    assert c["kernel_launches"]["k_suffix"] > 0 and c["kernel_launches"]["k_extend"] == 0
    _check(amvpt_mod, oracle, s)
