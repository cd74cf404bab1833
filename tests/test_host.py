"""Host framework (libamvpt_host.so, CPU side of the product): sensor math
goldens, XML loading into C-ABI descriptors, EXR I/O and error behaviour.
Nothing here touches a GPU."""
import json
import os

import numpy as np
import pytest

from conftest import SCENES

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_kats.json")


@pytest.fixture(scope="module")
def kats():
    with open(GOLDEN) as f:
        return json.load(f)


def test_parse_fov_golden(amvpt_mod, kats):
    """src/render/tests/test_sensor.py:test01_parse_fov."""
    for c in kats["parse_fov"]["cases"]:
        got = amvpt_mod.parse_fov(fov=c.get("fov", 0.0), fov_axis=c.get("fov_axis"),
                                  focal_length=c.get("focal_length"), aspect=c["aspect"])
        assert np.isclose(got, c["expected"], rtol=1e-5, atol=1e-8), c
    # fov_axis has no effect at aspect 1 (except diagonal)
    for axis in ("x", "y", "smaller", "larger"):
        assert np.isclose(amvpt_mod.parse_fov(fov=35.0, fov_axis=axis, aspect=1.0), 35.0)
    assert np.isclose(amvpt_mod.parse_fov(focal_length="25mm", fov_axis="y", aspect=1.0), 62.923526763916016)


def test_perspective_projection_golden(amvpt_mod, kats):
    """src/render/tests/test_sensor.py:test02_perspective_projection."""
    K = kats["perspective_projection"]
    m = amvpt_mod.perspective_projection(K["film_size"], K["crop_size"], K["crop_offset"], K["fov_x"], K["near"],
                                         K["far"])
    assert np.allclose(m, np.array(K["matrix"], dtype=np.float32), rtol=1e-5, atol=1e-8)


def test_parse_fov_errors(amvpt_mod):
    with pytest.raises(RuntimeError):
        amvpt_mod.parse_fov(fov=35.0, fov_axis="sideways", aspect=1.0)


def test_load_cbox_grid_descriptors(amvpt_mod):
    """scenes/cbox_grid.xml -> one grid sensor of gx*gy perspective views, mvpath params."""
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=32, spp=16, gx=4, gy=2, reuse=8)
    assert s.sensor_count() == 1
    w, h, c, spp = s.film_info(0)
    assert (w, h, spp) == (32 * 4, 32 * 2, 16) and c == 3
    sd, vd, p = s.describe(0, 0, 0)
    assert p.integrator == amvpt_mod.INTEGRATOR_MVPATH
    assert (p.n_views, p.grid_x, p.grid_y, p.multisensor) == (8, 4, 2, 1)
    assert (p.film_width, p.film_height) == (128, 64)
    assert p.max_depth == 8 and p.rr_depth == 5 and p.reuse_count == 8 and p.sa_reuse and p.sa_mis
    assert np.isclose(p.rfilter_stddev, 0.5)
    views = [vd[i] for i in range(p.n_views)]
    for v in views:
        tw = np.array(v.to_world[:], dtype=np.float64).reshape(4, 4)
        twi = np.array(v.to_world_inv[:], dtype=np.float64).reshape(4, 4)
        assert np.allclose(tw @ twi, np.eye(4), atol=1e-4)
        assert tuple(v.resolution) == (32, 32)
    # the grid spreads the camera origins: all distinct
    origins = {tuple(np.round(np.array(v.to_world[:]).reshape(4, 4)[:3, 3], 5)) for v in views}
    assert len(origins) == 8
    assert sd[0].shape_count == 8 and sd[0].emitter_count == 1


def test_xml_defaults_and_overrides(amvpt_mod):
    """<default name=...> values and $-substitution, overridden by load-time defines (mi.load_file(**kw))."""
    xml = """<scene version="3.0.0">
      <default name="spp" value="8"/>
      <default name="res" value="16"/>
      <integrator type="path"><integer name="max_depth" value="3"/></integrator>
      <sensor type="perspective">
        <float name="fov" value="45"/>
        <transform name="to_world"><lookat origin="0, 0, 4" target="0, 0, 0" up="0, 1, 0"/></transform>
        <sampler type="independent"><integer name="sample_count" value="$spp"/></sampler>
        <film type="hdrfilm"><integer name="width" value="$res"/><integer name="height" value="$res"/>
          <rfilter type="box"/></film>
      </sensor>
      <shape type="sphere"><float name="radius" value="1"/><bsdf type="diffuse"/></shape>
      <shape type="rectangle">
        <transform name="to_world"><translate value="0, 3, 0"/></transform>
        <emitter type="area"><rgb name="radiance" value="4, 4, 4"/></emitter>
      </shape>
    </scene>"""
    s = amvpt_mod.load_string(xml)
    assert s.film_info(0)[:2] == (16, 16) and s.film_info(0)[3] == 8
    s2 = amvpt_mod.load_string(xml, spp=32, res=24)
    assert s2.film_info(0)[:2] == (24, 24) and s2.film_info(0)[3] == 32
    sd, vd, p = s2.describe(0, 0, 0)
    assert p.integrator == amvpt_mod.INTEGRATOR_PATH and p.max_depth == 3 and p.rfilter == 0
    assert "path" in s2.integrator_string().lower()


def test_constant_emitter_loads(amvpt_mod):
    """`constant` (constant.cpp:52-65): radiance defaults to 1, one per scene; `envmap` stays refused."""
    s = amvpt_mod.load_string("<scene version='3.0.0'><emitter type='constant'>"
                              "<float name='sampling_weight' value='2'/></emitter>"
                              "<shape type='sphere'><float name='radius' value='2'/></shape>"
                              "<sensor type='perspective'><film type='hdrfilm'><integer name='width' value='8'/>"
                              "<integer name='height' value='8'/></film></sensor></scene>")
    sd, _, _ = s.describe(0, 0, 0)
    d = sd.contents
    assert d.emitter_count == 1 and d.has_environment == 1
    e = d.emitters[0]
    assert e.type == amvpt_mod.EMITTER_CONSTANT and e.shape == -1
    assert list(e.radiance) == [1.0, 1.0, 1.0] and e.sampling_weight == 2.0
    with pytest.raises(RuntimeError, match="one environment"):
        amvpt_mod.load_string("<scene version='3.0.0'><emitter type='constant'/><emitter type='constant'/></scene>")
    with pytest.raises(RuntimeError, match="envmap"):
        amvpt_mod.load_string("<scene version='3.0.0'><emitter type='envmap'/></scene>")


def test_xml_errors_are_loud(amvpt_mod):
    # plugins outside the implemented path (DESIGN.md "Scope") are refused, never ignored
    with pytest.raises(RuntimeError):
        amvpt_mod.load_string("<scene version='3.0.0'><emitter type='point'/></scene>")
    with pytest.raises(RuntimeError):
        amvpt_mod.load_string("<scene version='3.0.0'><shape type='nosuchshape'/></scene>")
    with pytest.raises(RuntimeError):
        amvpt_mod.load_string("<scene version='3.0.0'><integrator type='mvpath'>")  # truncated
    with pytest.raises(RuntimeError):
        amvpt_mod.load_file("/nonexistent/scene.xml")


def test_exr_round_trip(amvpt_mod, tmp_path):
    rng = np.random.default_rng(3)
    for c in (1, 3, 4):
        img = rng.standard_normal((7, 11, c)).astype(np.float32)
        img[0, 0, 0] = np.inf
        img[1, 1, 0] = np.nan
        path = str(tmp_path / ("t%d.exr" % c))
        amvpt_mod.write_exr(path, img)
        back = amvpt_mod.read_exr(path, 11, 7, c)
        assert np.array_equal(np.isnan(back), np.isnan(img))
        ok = ~np.isnan(img)
        assert np.array_equal(back[ok], img[ok])
        with open(path, "rb") as f:
            assert f.read(4) == b"\x76\x2f\x31\x01"  # OpenEXR magic


def test_plan_matches_oracle(amvpt_mod, oracle):
    """amvpt_plan (C-ABI, host-only) agrees with the oracle's pass plan for several configurations."""
    for kw in (dict(res=32, spp=16), dict(res=24, spp=64, gx=4, gy=2, reuse=8), dict(res=32, spp=12, spp_pass_lim=6),
               dict(res=16, spp=1), dict(res=1024, spp=64, gx=4, gy=2, reuse=8)):
        s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), **kw)
        _, _, p = s.describe(0, 0, 0)
        spp, spl, npass, lanes = amvpt_mod.plan(p)
        o = oracle.plan(p)
        assert (spp, spl, npass, lanes) == (o["spp"], o["spp_per_pass"], o["passes"], o["lanes"]), kw


def test_batch_sensor_loading(amvpt_mod):
    """batch.cpp:94-131: children side by side, horizontal resolution divisible by the child count."""
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_batch.xml"), res=32, width=128, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    assert (p.batch, p.multisensor, p.n_views, p.grid_x, p.grid_y) == (1, 1, 4, 4, 1)
    assert all(tuple(vd[i].resolution) == (32, 32) for i in range(4))
    with pytest.raises(RuntimeError, match="divisible"):
        amvpt_mod.load_file(os.path.join(SCENES, "cbox_batch.xml"), res=32, width=130, spp=16)


def _mesh_scene(shape_xml):
    return """<scene version="3.0.0">
      <integrator type="path"/>
      <sensor type="perspective"><float name="fov" value="45"/>
        <transform name="to_world"><lookat origin="0, 0, 4" target="0, 0, 0" up="0, 1, 0"/></transform>
        <film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>
      %s
      <shape type="rectangle"><transform name="to_world"><translate value="0, 3, 0"/></transform>
        <emitter type="area"><rgb name="radiance" value="1, 1, 1"/></emitter></shape>
    </scene>""" % shape_xml


def _mesh(amvpt_mod, xml):
    s = amvpt_mod.load_string(xml)
    sd, _, _ = s.describe(0, 0, 0)
    d = sd[0].shapes[0]
    nv, nf = d.vertex_count, d.face_count
    faces = np.ctypeslib.as_array(d.faces, shape=(nf * 3,)).reshape(nf, 3).copy()
    pos = np.ctypeslib.as_array(d.positions, shape=(nv * 3,)).reshape(nv, 3).copy()
    nrm = np.ctypeslib.as_array(d.normals, shape=(nv * 3,)).reshape(nv, 3).copy() if d.normals else None
    return s, d, faces, pos, nrm


def test_obj_fan_triangulation_and_dedup(amvpt_mod):
    """obj.cpp:270-330: polygons fan out as (v0, v[k-1], v[k]); vertices shared by (v, vt, vn) key."""
    path = os.path.join(SCENES, "meshes", "quad_fan.obj")
    s, d, faces, pos, nrm = _mesh(amvpt_mod, _mesh_scene('<shape type="obj"><string name="filename" value="%s"/></shape>' % path))
    assert d.vertex_count == 7 and d.face_count == 5
    assert faces.tolist() == [[0, 1, 2], [0, 2, 3], [0, 3, 4], [1, 5, 6], [1, 6, 2]]
    assert np.allclose(pos[5], [2, 0, 0])
    assert nrm is not None and np.allclose(nrm, [0, 0, 1], atol=1e-6)   # recomputed (planar mesh)


def test_obj_transform_and_normals(amvpt_mod):
    path = os.path.join(SCENES, "meshes", "icosphere.obj")
    xml = _mesh_scene('<shape type="obj"><string name="filename" value="%s"/><transform name="to_world">'
                      '<scale x="2" y="1" z="1"/><translate x="1"/></transform></shape>' % path)
    s, d, faces, pos, nrm = _mesh(amvpt_mod, xml)
    assert d.vertex_count == 642 and d.face_count == 1280
    assert np.allclose(pos[:, 0].min(), -1, atol=1e-5) and np.allclose(pos[:, 0].max(), 3, atol=1e-5)
    assert np.allclose(np.linalg.norm(nrm, axis=1), 1, atol=1e-5)
    # normals transform with the inverse transpose: on the unit sphere scaled by (2,1,1), n ~ (x/4, y, z)
    p0 = (pos - [1, 0, 0]) / [2, 1, 1]
    ref = p0 / [2, 1, 1]
    ref /= np.linalg.norm(ref, axis=1, keepdims=True)
    assert np.abs(nrm - ref).max() < 1e-4
    _, d2, _, _, nrm2 = _mesh(amvpt_mod, xml.replace('<string name="filename"', '<boolean name="face_normals" value="true"/><string name="filename"'))
    assert not d2.normals and nrm2 is None


def test_ply_binary_with_recomputed_normals(amvpt_mod):
    path = os.path.join(SCENES, "meshes", "torus.ply")
    s, d, faces, pos, nrm = _mesh(amvpt_mod, _mesh_scene('<shape type="ply"><string name="filename" value="%s"/></shape>' % path))
    assert d.vertex_count == 48 * 24 and d.face_count == 2304
    assert np.allclose(np.linalg.norm(nrm, axis=1), 1, atol=1e-5)
    # torus normal at a vertex points away from the tube centre ring
    ring = pos.copy()
    ring[:, 1] = 0
    ring = ring / np.linalg.norm(ring, axis=1, keepdims=True)
    radial = pos - ring
    radial /= np.linalg.norm(radial, axis=1, keepdims=True)
    assert (np.sum(radial * nrm, axis=1) > 0.99).all()


def test_mesh_errors(amvpt_mod):
    with pytest.raises(RuntimeError, match="not found"):
        amvpt_mod.load_string(_mesh_scene('<shape type="obj"><string name="filename" value="/nope.obj"/></shape>'))


def test_crop_window_descriptors_and_projection(amvpt_mod, oracle):
    """hdrfilm crop windows: the ImageBlock / lane space is the crop, the film keeps its full size, an invalid
    window is the reference's error (film.cpp:91-96), and crop pixel (x, y) sees what film pixel
    (x + crop_x, y + crop_y) of the uncropped camera sees (perspective_projection with the crop, sensor.h:319-356)."""
    import numpy as np
    path = os.path.join(SCENES, "cbox_path.xml")
    full = amvpt_mod.load_file(path, res=64)
    crop = amvpt_mod.load_file(path, res=64, crop_w=40, crop_h=24, crop_x=10, crop_y=30)
    assert crop.film_info()[:2] == (40, 24)
    sf, vf, pf = full.describe()
    sc, vc, pc = crop.describe()
    assert (pc.film_width, pc.film_height, pc.crop_offset_x, pc.crop_offset_y, pc.full_width, pc.full_height) == (
        40, 24, 10, 30, 64, 64)
    hf, hc = oracle.primary_hits(sf, vf, pf), oracle.primary_hits(sc, vc, pc)
    sub = hf[30:54, 10:50]
    assert (sub[..., 0] == hc[..., 0]).mean() > 0.99
    assert np.abs(sub[..., 4:7] - hc[..., 4:7])[sub[..., 0] == hc[..., 0]].max() < 1e-4
    with pytest.raises(RuntimeError, match="Invalid crop window specification"):
        amvpt_mod.load_file(path, res=64, crop_w=60, crop_x=10)
    # the grid sensor resizes its film, which resets any crop window (grid.cpp:230, film.cpp:102-106)
    g = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=16)
    gp = g.describe()[2]
    assert (gp.crop_offset_x, gp.full_width) == (0, gp.film_width)


_STRICT_BASE = """<scene version="3.0.0">
  <integrator type="{itype}">{iprops}</integrator>
  <sensor type="perspective">{sprops}
    <float name="fov" value="45"/>
    <transform name="to_world"><lookat origin="0, 0, 4" target="0, 0, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sample_count" value="16"/></sampler>
    <film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/>{fprops}</film>
  </sensor>
  <shape type="sphere"><float name="radius" value="1"/>{shprops}<bsdf type="diffuse">{bprops}</bsdf></shape>
  <shape type="rectangle">
    <transform name="to_world"><translate value="0, 3, 0"/></transform>
    <emitter type="area"><rgb name="radiance" value="4, 4, 4"/>{eprops}</emitter>
  </shape>{extra}
</scene>"""


def _strict(amvpt_mod, itype="path", iprops="", sprops="", fprops="", shprops="", bprops="", eprops="", extra=""):
    return amvpt_mod.load_string(_STRICT_BASE.format(itype=itype, iprops=iprops, sprops=sprops, fprops=fprops,
                                                     shprops=shprops, bprops=bprops, eprops=eprops, extra=extra))


def test_xml_unreferenced_properties_are_errors(amvpt_mod):
    """The XML loader refuses properties and child objects that no plugin read (xml.cpp:1089-1107), with the
    reference's message; a typo'd key no longer renders silently with defaults."""
    _strict(amvpt_mod)   # the base scene itself is clean
    cases = [
        (dict(iprops='<integer name="max_detph" value="3"/>'), r'unreferenced property "\["max_detph"\]" in '
                                                               r'integrator plugin of type "path"'),
        (dict(itype="mvpath", iprops='<boolean name="sa_resue" value="true"/>'), r'"\["sa_resue"\]" in integrator'),
        (dict(sprops='<float name="fov_x" value="3"/>'), r'"\["fov_x"\]" in sensor plugin of type "perspective"'),
        (dict(fprops='<integer name="widht" value="8"/>'), r'"\["widht"\]" in film plugin of type "hdrfilm"'),
        (dict(shprops='<float name="raduis" value="2"/>'), r'"\["raduis"\]" in shape plugin of type "sphere"'),
        (dict(bprops='<rgb name="reflectence" value="0.5"/>'), r'in bsdf plugin of type "diffuse"'),
        (dict(eprops='<float name="sampling_wieght" value="2"/>'), r'in emitter plugin of type "area"'),
        (dict(iprops='<integer name="a" value="1"/><integer name="b" value="1"/>'),
         r'unreferenced properties "\["a", "b"\]"'),
        (dict(extra='<integer name="stray" value="1"/>'), r'"\["stray"\]" in scene plugin'),
        (dict(fprops='<rfilter type="gaussian"><float name="stdev" value="1"/></rfilter>'),
         r'in reconstructionfilter plugin of type "gaussian"'),
        # a perspective camera has no aperture (thinlens.cpp reads it, perspective.cpp does not)
        (dict(sprops='<float name="aperture_radius" value="0.1"/>'), r'"\["aperture_radius"\]" in sensor'),
        (dict(bprops='<rfilter type="box"/>'), r'unreferenced object rfilter of type "box" \(within bsdf'),
    ]
    for kw, msg in cases:
        with pytest.raises(RuntimeError, match=msg):
            _strict(amvpt_mod, **kw)


def test_xml_unused_bsdf_and_wrapped_film_load(amvpt_mod):
    """the reference's loader instantiates every child of the scene, so a scene-level BSDF no shape
    uses reads its keys and loads (a typo in it still fails); a film given through <wrap> (wrap.cpp) is read by
    the perspective sensor like a plain <film> child."""
    unused = '<bsdf type="roughconductor" id="spare"><float name="alpha" value="0.2"/></bsdf>'
    s = _strict(amvpt_mod, extra=unused)
    assert s.describe(0, 0, 0)[0].contents.bsdf_count == _strict(amvpt_mod).describe(0, 0, 0)[0].contents.bsdf_count
    with pytest.raises(RuntimeError, match=r'"\["alhpa"\]" in bsdf plugin of type "roughconductor"'):
        _strict(amvpt_mod, extra=unused.replace("alpha", "alhpa"))
    # an unused BSDF of a plugin this port does not implement loads (the scene never renders it) --
    # also nested in a twosided; a USED one stays a loud error
    for extra in ('<bsdf type="dielectric" id="glass"><float name="int_ior" value="1.5"/></bsdf>',
                  '<bsdf type="twosided" id="ts"><bsdf type="plastic"><rgb name="diffuse_reflectance" value="0.5"/>'
                  '</bsdf></bsdf>'):
        assert _strict(amvpt_mod, extra=extra).describe(0, 0, 0)[0].contents.bsdf_count == \
            _strict(amvpt_mod).describe(0, 0, 0)[0].contents.bsdf_count
    with pytest.raises(RuntimeError, match="not implemented"):
        _strict(amvpt_mod, bprops="").__class__   # (the base scene's sphere BSDF is diffuse: fine)
        amvpt_mod.load_string(_STRICT_BASE.replace('<bsdf type="diffuse">{bprops}</bsdf>', '<bsdf type="dielectric"/>')
                              .format(itype="path", iprops="", sprops="", fprops="", shprops="", eprops="", extra=""))
    wrapped = _STRICT_BASE.replace(
        '<film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/>{fprops}</film>',
        '<wrap type="wrap"><string name="wrap_class" value="film"/><string name="wrap_type" value="hdrfilm"/>'
        '<integer name="width" value="12"/><integer name="height" value="8"/>{fprops}</wrap>')
    fill = dict(itype="path", iprops="", sprops="", fprops="", shprops="", bprops="", eprops="", extra="")
    w = amvpt_mod.load_string(wrapped.format(**fill))
    assert w.film_info()[:2] == (12, 8)
    # the wrapped film's own children are still checked
    with pytest.raises(RuntimeError, match=r"in reconstructionfilter plugin of type \"gaussian\""):
        amvpt_mod.load_string(wrapped.format(**dict(fill, fprops='<rfilter type="gaussian">'
                                                                    '<float name="stdev" value="1"/></rfilter>')))


def test_xml_accepts_every_key_the_reference_plugins_read(amvpt_mod):
    """Keys the reference's plugins query (so its loader accepts them) load here too, with the reference's
    meaning or its documented no-op on the JIT render path."""
    s = _strict(amvpt_mod,
                iprops='<float name="timeout" value="10"/><integer name="block_size" value="16"/>'
                       '<integer name="samples_per_pass" value="4"/><boolean name="hide_emitters" value="false"/>',
                sprops='<float name="near_clip" value="0.01"/><float name="far_clip" value="100"/>'
                       '<float name="focus_distance" value="4"/><float name="shutter_open" value="0"/>'
                       '<float name="shutter_close" value="0"/><float name="principal_point_offset_x" value="0"/>',
                fprops='<string name="component_format" value="float32"/><string name="file_format" value="openexr"/>'
                       '<boolean name="banner" value="false"/><string name="pixel_format" value="rgb"/>'
                       '<boolean name="sample_border" value="false"/>',
                shprops='<boolean name="flip_normals" value="false"/><point name="center" value="0, 0, 0"/>'
                        '<float name="silhouette_sampling_weight" value="1"/>',
                eprops='<float name="sampling_weight" value="1"/>')
    sd, vd, p = s.describe(0, 0, 0)
    assert p.spp_pass_lim == 4   # the path integrator's samples_per_pass (amvpt.h)
    for kw, msg in [
        (dict(sprops='<float name="shutter_open" value="1"/><float name="shutter_close" value="0.5"/>'),
         "Shutter opening time must be less than or equal to the shutter closing time"),
        (dict(sprops='<float name="shutter_close" value="0.5"/>'), "shutter interval"),
        (dict(fprops='<string name="file_format" value="pfm"/>'), "file_format"),
        (dict(eprops='<transform name="to_world"><translate value="0, 1, 0"/></transform>'),
         "Found a 'to_world' transformation -- this is not allowed"),
        (dict(iprops='<integer name="samples_per_pass" value="0"/>'), "samples_per_pass"),
    ]:
        with pytest.raises(RuntimeError, match=msg):
            _strict(amvpt_mod, **kw)


def test_path_samples_per_pass_must_divide_spp(amvpt_mod):
    """SamplingIntegrator::render: 'sample_count (%d) must be a multiple of spp_per_pass (%d).'"""
    s = _strict(amvpt_mod, iprops='<integer name="samples_per_pass" value="4"/>')
    assert s.describe(0, 0, 16)[2].spp_pass_lim == 4
    with pytest.raises(RuntimeError, match=r"sample_count \(10\) must be a multiple of spp_per_pass \(4\)\."):
        s.describe(0, 0, 10)
    s.describe(0, 0, 3)   # spp_per_pass = min(4, 3) = 3
