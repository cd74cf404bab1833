"""The drop-in boundary: both product libraries load, export every function the
public headers declare, and fail loudly (status + message) instead of falling
back when they cannot run.  No compute calls: these run on CPU."""
import ctypes
import os
import re

import pytest

from conftest import REPO, SCENES

HEADERS = [os.path.join(REPO, "include", h) for h in ("amvpt.h", "amvpt_host.h")]


def declared(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set(re.findall(r"\b(amvpt_[a-z0-9_]+)\s*\(", src))
    return sorted(n for n in names if not n.endswith("_t"))


def test_headers_declare_the_boundary():
    hip = declared(HEADERS[0])
    for fn in ("amvpt_scene_create", "amvpt_scene_destroy", "amvpt_render", "amvpt_render_records", "amvpt_plan",
               "amvpt_develop", "amvpt_last_error", "amvpt_abi_version"):
        assert fn in hip
    assert "amvpt_host_load_file" in declared(HEADERS[1])


def test_hip_library_exports_every_declared_symbol(amvpt_mod):
    L = amvpt_mod.hip_lib()
    missing = [n for n in declared(HEADERS[0]) if not hasattr(L, n)]
    assert not missing, missing


def test_host_library_exports_every_declared_symbol(amvpt_mod):
    L = amvpt_mod.host_lib()
    missing = [n for n in declared(HEADERS[1]) if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version_and_channels(amvpt_mod):
    L = amvpt_mod.hip_lib()
    assert L.amvpt_abi_version() >= 1
    p = amvpt_mod.Params()
    p.film_alpha = 0
    assert L.amvpt_film_channels(ctypes.byref(p)) == 4
    p.film_alpha = 1
    assert L.amvpt_film_channels(ctypes.byref(p)) == 5


def test_invalid_arguments_fail_loudly(amvpt_mod):
    L = amvpt_mod.hip_lib()
    h = ctypes.c_void_p()
    assert L.amvpt_scene_create(None, ctypes.byref(h)) != 0
    assert L.amvpt_last_error().decode()
    p = amvpt_mod.Params()
    rc = L.amvpt_render(None, None, ctypes.byref(p), 0, 1, None, None, None)
    assert rc != 0 and L.amvpt_last_error().decode()


def test_no_device_means_error_not_fallback(amvpt_mod):
    """Without a HIP device the product path refuses (no CPU fallback exists)."""
    if amvpt_mod.device_count() > 0:
        pytest.skip("a HIP device is visible")
    import amvpt
    from conftest import SCENES
    s = amvpt.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=8, spp=4)
    sd, vd, p = s.describe(0, 0, 0)
    with pytest.raises(RuntimeError):
        amvpt.DeviceScene(sd)
    with pytest.raises(RuntimeError):
        amvpt.render(s)


def test_product_modules_never_import_the_oracle():
    """Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use oracle/."""
    pkg = os.path.join(REPO, "mitsuba3-amvpt_amd")
    bad = re.compile(r"import\s+oracle|from\s+oracle|oracle_math\.h|amvpt_oracle|liboracle|oracle/")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", "Makefile")):
                txt = open(os.path.join(root, f), errors="ignore").read()
                assert not bad.search(txt), os.path.join(root, f)


def _cbox_desc(amvpt_mod, name="cbox_grid.xml"):
    from conftest import SCENES
    s = amvpt_mod.load_file(os.path.join(SCENES, name), res=8, spp=4)
    sd, vd, p = s.describe(0, 0, 0)
    return s, sd, vd, p


def _copy_scene(amvpt_mod, sd):
    """Deep-enough copy of a SceneDesc whose tables can be edited."""
    d = sd.contents
    shapes = (amvpt_mod.ShapeDesc * d.shape_count)(*[d.shapes[i] for i in range(d.shape_count)])
    bsdfs = (amvpt_mod.BsdfDesc * d.bsdf_count)(*[d.bsdfs[i] for i in range(d.bsdf_count)])
    ems = (amvpt_mod.EmitterDesc * d.emitter_count)(*[d.emitters[i] for i in range(d.emitter_count)])
    nd = amvpt_mod.SceneDesc(ctypes.cast(shapes, ctypes.POINTER(amvpt_mod.ShapeDesc)), d.shape_count,
                             ctypes.cast(bsdfs, ctypes.POINTER(amvpt_mod.BsdfDesc)), d.bsdf_count,
                             ctypes.cast(ems, ctypes.POINTER(amvpt_mod.EmitterDesc)), d.emitter_count, 0)
    return nd, shapes, bsdfs, ems


@pytest.mark.parametrize("breakage", ["emitter_range", "emitter_pair", "face_index", "bsdf_range",
                                      "env_count", "env_shape", "negative_weight", "zero_weights",
                                      "mesh_light_no_area"])
def test_scene_create_rejects_malformed_descriptors(amvpt_mod, breakage):
    """Malformed C-ABI input is refused with AMVPT_ERR_INVALID before any device work:
    shape.emitter outside [-1, emitter_count), emitter.shape / shape.emitter disagreeing, mesh face
    indices >= vertex_count, BSDF indices out of range."""
    L = amvpt_mod.hip_lib()
    s, sd, vd, p = _cbox_desc(amvpt_mod, "cbox_meshlight.xml" if breakage == "mesh_light_no_area" else "cbox_grid.xml")
    nd, shapes, bsdfs, ems = _copy_scene(amvpt_mod, sd)
    keep = []
    if breakage == "emitter_range":
        shapes[0].emitter = nd.emitter_count + 3
    elif breakage == "emitter_pair":
        light = ems[0].shape
        other = 1 if light != 1 else 2
        shapes[other].emitter = 0            # a second shape claims emitter 0
    elif breakage == "face_index":
        mesh = next(i for i in range(nd.shape_count) if shapes[i].type == 1)
        n = shapes[mesh].face_count * 3
        faces = (ctypes.c_uint32 * n)(*[shapes[mesh].faces[k] for k in range(n)])
        faces[n - 1] = shapes[mesh].vertex_count
        keep.append(faces)
        shapes[mesh].faces = ctypes.cast(faces, ctypes.POINTER(ctypes.c_uint32))
    elif breakage == "mesh_light_no_area":
        light = next(i for i in range(nd.shape_count) if shapes[i].type == 1 and shapes[i].emitter >= 0)
        flat = (ctypes.c_float * (3 * shapes[light].vertex_count))()   # every vertex at the origin
        keep.append(flat)
        shapes[light].positions = ctypes.cast(flat, ctypes.POINTER(ctypes.c_float))
    elif breakage == "env_count":
        nd.has_environment = 1               # claims a constant emitter the table does not hold
    elif breakage == "env_shape":
        env = (amvpt_mod.EmitterDesc * (nd.emitter_count + 1))(*[ems[i] for i in range(nd.emitter_count)])
        env[nd.emitter_count].type = amvpt_mod.EMITTER_CONSTANT
        env[nd.emitter_count].shape = 0      # a constant emitter attached to a shape
        env[nd.emitter_count].sampling_weight = 1.0
        keep.append(env)
        nd.emitters = ctypes.cast(env, ctypes.POINTER(amvpt_mod.EmitterDesc))
        nd.emitter_count += 1
        nd.has_environment = 1
    elif breakage == "negative_weight":
        ems[0].sampling_weight = -1.0        # DiscreteDistribution: entries must be non-negative
    elif breakage == "zero_weights":
        for i in range(nd.emitter_count):
            ems[i].sampling_weight = 0.0     # no probability mass
    else:
        shapes[0].bsdf = nd.bsdf_count
    h = ctypes.c_void_p()
    assert L.amvpt_scene_create(ctypes.byref(nd), ctypes.byref(h)) == 1   # AMVPT_ERR_INVALID
    assert L.amvpt_last_error().decode()


@pytest.mark.parametrize("name", ["cbox_grid.xml", "cbox_meshlight.xml"])
def test_scene_create_accepts_the_loaded_descriptor(amvpt_mod, name):
    """The unmodified loader output passes validation (then needs a device); area emitters on
    meshes are accepted (mesh.cpp:765-816)."""
    L = amvpt_mod.hip_lib()
    s, sd, vd, p = _cbox_desc(amvpt_mod, name)
    nd, shapes, bsdfs, ems = _copy_scene(amvpt_mod, sd)
    h = ctypes.c_void_p()
    rc = L.amvpt_scene_create(ctypes.byref(nd), ctypes.byref(h))
    if amvpt_mod.device_count() > 0:
        assert rc == 0
        L.amvpt_scene_destroy(h)
    else:
        assert rc == 5, L.amvpt_last_error()   # AMVPT_ERR_NO_DEVICE


def _box_count(amvpt_mod, nd):
    L = amvpt_mod.hip_lib()
    L.amvpt_scene_desc_boxes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    n = ctypes.c_uint32()
    assert L.amvpt_scene_desc_boxes(ctypes.byref(nd), ctypes.byref(n)) == 0, L.amvpt_last_error()
    return n.value


def test_box_meshes_are_recognised(amvpt_mod):
    """amvpt_scene_create's box-mesh detection (find_boxes, host side): the Cornell box's two `cube`s are
    boxes; its rectangles and the OBJ/PLY meshes are not; a cube with one vertex moved off its corner is not."""
    s, sd, vd, p = _cbox_desc(amvpt_mod, "cbox_grid.xml")
    nd, shapes, bsdfs, ems = _copy_scene(amvpt_mod, sd)
    assert _box_count(amvpt_mod, nd) == 2
    s2, sd2, _, _ = _cbox_desc(amvpt_mod, "cbox_mesh.xml")
    nd2, *_keep2 = _copy_scene(amvpt_mod, sd2)
    assert _box_count(amvpt_mod, nd2) == 0
    cube = next(i for i in range(nd.shape_count) if shapes[i].type == 1 and shapes[i].face_count == 12)
    n = 3 * shapes[cube].vertex_count
    pos = (ctypes.c_float * n)(*[shapes[cube].positions[k] for k in range(n)])
    pos[0] += 0.05   # vertex 0 leaves its corner
    shapes[cube].positions = ctypes.cast(pos, ctypes.POINTER(ctypes.c_float))
    assert _box_count(amvpt_mod, nd) == 1


def test_box_screen_conditioning_counts_the_whole_scene(amvpt_mod):
    """the screen maps suffix-ray ORIGINS into box space, and those lie anywhere on the scene, so a
    box is screened only while its conditioning x (1 + the scene's largest coordinate) < 100: the Cornell cubes
    (conditioning 3.3) stay boxes beside a floor 18 units wide, not beside one 200 units wide."""
    xml = open(os.path.join(SCENES, "cbox_path.xml")).read()
    rot = '<rotate x="1" angle="-90"/>\n            <translate y="-1"/>'
    assert rot in xml
    for scale, boxes in ((1, 2), (9, 2), (100, 0)):
        s = amvpt_mod.load_string(xml.replace(rot, '<scale x="%d" y="%d"/>' % (scale, scale) + rot), res=8, spp=4)
        assert amvpt_mod.scene_box_count(s) == boxes, scale
