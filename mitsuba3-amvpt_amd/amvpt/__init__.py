"""
amvpt -- Python front end of the MI355X-native AMVPT (`mvpath`) integrator.

A thin ctypes layer over the two in-tree native libraries:

* ``lib/libamvpt_hip.so``  -- the drop-in C-ABI of the hot path (include/amvpt.h),
  hand-written HIP kernels for gfx950;
* ``lib/libamvpt_host.so`` -- the Mitsuba-style host framework (XML scene subset,
  Properties, plugins, ``Integrator::render``) built on that C-ABI.

The surface mirrors the reference's Python API for the path
(``mi.load_file``, ``mi.load_string``, ``mi.render``, ``Bitmap.write``;
reference: src/python/python/__init__.py / src/render/python).  There is no
CPU fallback: rendering without a visible GPU raises ``RuntimeError``.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AMVPT_LIB_DIR selects a variant build (Makefile LIB=...) for A/B measurements.
LIB_DIR = os.environ.get("AMVPT_LIB_DIR") or os.path.join(os.path.dirname(_HERE), "lib")
HIP_LIB_PATH = os.path.join(LIB_DIR, "libamvpt_hip.so")
HOST_LIB_PATH = os.path.join(LIB_DIR, "libamvpt_host.so")

u32, i32, u64, f32, f64 = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_float, ctypes.c_double


class ShapeDesc(ctypes.Structure):
    _fields_ = [("type", u32), ("bsdf", i32), ("emitter", i32), ("flip_normals", u32),
                ("to_world", f32 * 16), ("to_object", f32 * 16),
                ("vertex_count", u32), ("face_count", u32),
                ("positions", ctypes.POINTER(f32)), ("normals", ctypes.POINTER(f32)),
                ("texcoords", ctypes.POINTER(f32)), ("faces", ctypes.POINTER(u32)),
                ("center", f32 * 3), ("radius", f32)]


class BsdfDesc(ctypes.Structure):
    _fields_ = [("type", u32), ("nested", i32 * 2), ("reflectance", f32 * 3), ("distribution", u32),
                ("sample_visible", u32), ("alpha_u", f32), ("alpha_v", f32), ("eta", f32 * 3),
                ("k", f32 * 3), ("has_specular_reflectance", u32), ("specular_reflectance", f32 * 3)]


class EmitterDesc(ctypes.Structure):
    _fields_ = [("type", u32), ("shape", i32), ("radiance", f32 * 3), ("sampling_weight", f32)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("shapes", ctypes.POINTER(ShapeDesc)), ("shape_count", u32),
                ("bsdfs", ctypes.POINTER(BsdfDesc)), ("bsdf_count", u32),
                ("emitters", ctypes.POINTER(EmitterDesc)), ("emitter_count", u32),
                ("has_environment", u32)]


class ViewDesc(ctypes.Structure):
    _fields_ = [("type", u32), ("to_world", f32 * 16), ("to_world_inv", f32 * 16),
                ("sample_to_camera", f32 * 16), ("camera_to_sample", f32 * 16),
                ("near_clip", f32), ("far_clip", f32), ("normalization", f32),
                ("resolution", f32 * 2), ("pp_offset", f32 * 2),
                ("aperture_radius", f32), ("focus_distance", f32)]


class Params(ctypes.Structure):
    _fields_ = [(n, u32) for n in (
        "integrator", "max_depth", "rr_depth", "hide_emitters", "sa_reuse", "sa_mis", "fast_mis",
        "debug", "adaptive", "spp_pass_lim", "reuse_count", "spp", "seed", "base_seed", "n_views",
        "multisensor", "grid_x", "grid_y", "reverse_x", "reverse_y", "film_width", "film_height",
        "film_alpha", "rfilter")] + [("rfilter_stddev", f32), ("batch", u32), ("crop_offset_x", u32),
                                      ("crop_offset_y", u32), ("full_width", u32), ("full_height", u32)]


class Counters(ctypes.Structure):
    _fields_ = [("lanes", u64), ("passes", u64), ("vertices", u64), ("reuse_lanes", u64),
                ("visibility_rays", u64), ("view_splats", u64), ("adaptive_lanes", u64),
                ("kernel_ms_primary", f64), ("kernel_ms_bounce", f64), ("kernel_ms_splat", f64),
                ("total_ms", f64), ("splat_fallback", u64),
                ("shadow_rays", u64), ("kernel_ms", f64 * 12), ("kernel_launches", u64 * 12),
                ("record_bytes", u64), ("nonfinite_samples", u64), ("negative_samples", u64),
                ("pushed_paths", u64), ("film_overflow", u64), ("film_range_drops", u64),
                ("chunk_lanes", u64), ("buffer_sets", u64), ("arena_bytes", u64),
                ("primary_record_bytes", u64), ("splat_record_bytes", u64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        for k in ("kernel_ms", "kernel_launches"):
            d[k] = {name: d[k][i] for i, name in enumerate(KERNELS)}
        return d


class LaneSet(ctypes.Structure):
    """amvpt_lane_set: contiguous lanes [lane_begin, lane_end), or (rect_width > 0) the lanes of a
    pixel rectangle of the quilt (one run of rect_width * spp_per_pass lanes per pixel row)."""
    _fields_ = [("lane_begin", u64), ("lane_end", u64), ("rect_x0", u32), ("rect_y0", u32),
                ("rect_width", u32), ("rect_height", u32)]


class FilmWindow(ctypes.Structure):
    """amvpt_film_window: device film holding quilt pixels [x0, x0+width) x [y0, y0+height), plus the
    overflow list (device; 16-B header with the u64 cell count, then 16-B entries) for cells outside."""
    _fields_ = [("film", ctypes.c_void_p), ("x0", u32), ("y0", u32), ("width", u32), ("height", u32),
                ("overflow", ctypes.c_void_p), ("overflow_capacity", u64)]


# amvpt_run_exchange_fn: (ctx, n_runs, *run_lane_begin, *run_count, *run_prefix, *total) -> 0 on success
RunExchangeFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, u32, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                 ctypes.POINTER(u64), ctypes.POINTER(u64))


class RenderOpts(ctypes.Structure):
    """amvpt_render_opts: per-call chunk size, traversal, path-selection flags, run exchange, records, and
    (ABI 10) the device-memory budget in MiB (0: automatic)."""
    _fields_ = [("chunk_lanes", u64), ("traversal", u32), ("flags", u32), ("exchange", RunExchangeFn),
                ("exchange_ctx", ctypes.c_void_p), ("records", ctypes.c_void_p), ("record_pass", u32),
                ("budget_mib", u32)]


# amvpt_render_opts.flags (results are identical; kernel-path selection for tests / A/B)
OPT_GENERIC_KERNELS, OPT_WAVEFRONT_SUFFIX, OPT_SPLIT_NEE, OPT_ONE_STREAM, OPT_DETERMINISTIC = 1, 2, 4, 8, 16
OPT_NO_BINNING = 32
OPT_NO_BOX_SCREEN = 64
OPT_THREADED_BVH = 128


def wrap_run_exchange(fn):
    """ctypes callback around `fn(run_lane_begin: list, run_count: list) -> (run_prefix: list, total)`
    (exceptions -> status 1)."""
    def cb(_ctx, n, begins, counts, prefix, total):
        try:
            pre, tot = fn([int(begins[i]) for i in range(n)], [int(counts[i]) for i in range(n)])
            for i in range(n):
                prefix[i] = int(pre[i])
            total[0] = int(tot)
            return 0
        except Exception:   # noqa: BLE001 -- reported to the C side as a failed exchange
            return 1
    return RunExchangeFn(cb)


# amvpt_kernel_id (include/amvpt.h): index -> name of Counters.kernel_ms / kernel_launches
KERNELS = ("k_prim_hit", "k_prim_req", "k_vis", "k_mv_primary", "k_raygen", "k_extend", "k_bounce", "k_shadow",
           "k_splat", "k_suffix", "k_select", "k_bin")


INTEGRATOR_MVPATH, INTEGRATOR_PATH = 0, 1
EMITTER_AREA, EMITTER_CONSTANT = 0, 1
_hip = None
_host = None


def hip_lib():
    """Load libamvpt_hip.so (the C-ABI of the hot path); raises if it was not built."""
    global _hip
    if _hip is None:
        if not os.path.exists(HIP_LIB_PATH):
            raise RuntimeError("libamvpt_hip.so missing: run `make -C mitsuba3-amvpt_amd` "
                               "(__graft_entry__.build()); the product path has no fallback")
        L = ctypes.CDLL(HIP_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        L.amvpt_last_error.restype = ctypes.c_char_p
        L.amvpt_abi_version.restype = u32
        L.amvpt_film_channels.restype = u32
        for fn in ("amvpt_device_count", "amvpt_set_device", "amvpt_scene_create", "amvpt_scene_destroy",
                   "amvpt_scene_stats", "amvpt_render", "amvpt_render_records", "amvpt_plan",
                   "amvpt_develop", "amvpt_set_chunk_lanes", "amvpt_set_traversal",
                   "amvpt_set_adaptive_exchange", "amvpt_set_bvh_build", "amvpt_render_ex", "amvpt_scene_desc_boxes",
                   "amvpt_release_device_memory"):
            if hasattr(L, fn):   # older variant builds (AMVPT_LIB_DIR A/B runs) may lack the newest knobs
                getattr(L, fn).restype = ctypes.c_int
        L.amvpt_render.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Params), u64, u64,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Counters)]
        if hasattr(L, "amvpt_render_ex"):
            L.amvpt_render_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Params),
                                          ctypes.POINTER(LaneSet), ctypes.POINTER(FilmWindow), ctypes.c_void_p,
                                          ctypes.POINTER(RenderOpts), ctypes.POINTER(Counters)]
        L.amvpt_render_records.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Params), u32, u64,
                                           u64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.amvpt_scene_create.argtypes = [ctypes.POINTER(SceneDesc), ctypes.POINTER(ctypes.c_void_p)]
        L.amvpt_scene_destroy.argtypes = [ctypes.c_void_p]
        L.amvpt_scene_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.amvpt_plan.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(u32), ctypes.POINTER(u32),
                                 ctypes.POINTER(u32), ctypes.POINTER(u64)]
        L.amvpt_develop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u32, u32, u32, ctypes.c_void_p]
        L.amvpt_set_chunk_lanes.argtypes = [u64]
        if hasattr(L, "amvpt_set_bvh_build"):
            L.amvpt_set_bvh_build.argtypes = [u32, ctypes.c_float]
        if hasattr(L, "amvpt_set_adaptive_exchange"):
            L.amvpt_set_adaptive_exchange.argtypes = [ExchangeFn, ctypes.c_void_p]
        L.amvpt_set_device.argtypes = [ctypes.c_int]
        if hasattr(L, "amvpt_release_device_memory"):
            L.amvpt_release_device_memory.argtypes = [ctypes.c_int]
        L.amvpt_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        _hip = L
    return _hip


def host_lib():
    global _host
    if _host is None:
        hip_lib()
        if not os.path.exists(HOST_LIB_PATH):
            raise RuntimeError("libamvpt_host.so missing: run `make -C mitsuba3-amvpt_amd`")
        L = ctypes.CDLL(HOST_LIB_PATH)
        L.amvpt_host_last_error.restype = ctypes.c_char_p
        L.amvpt_host_load_file.restype = ctypes.c_void_p
        L.amvpt_host_load_string.restype = ctypes.c_void_p
        L.amvpt_host_load_file.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.amvpt_host_load_string.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.amvpt_host_scene_free.argtypes = [ctypes.c_void_p]
        L.amvpt_host_sensor_count.argtypes = [ctypes.c_void_p]
        L.amvpt_host_sensor_count.restype = u32
        L.amvpt_host_film_info.argtypes = [ctypes.c_void_p, u32] + [ctypes.POINTER(u32)] * 4
        L.amvpt_host_render.argtypes = [ctypes.c_void_p, u32, u32, u32, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.POINTER(Counters)]
        L.amvpt_host_render_stream.argtypes = [ctypes.c_void_p, u32, u32, u32, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.POINTER(Counters)]
        L.amvpt_host_render_stats.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(u64)] * 3
        L.amvpt_host_render_multi.argtypes = [ctypes.c_void_p, u32, u32, u32, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_void_p,
                                              ctypes.POINTER(Counters)]
        L.amvpt_host_lane_shard.argtypes = [u64, u32, u32, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.amvpt_host_lane_shard.restype = None
        L.amvpt_host_view_group_partition.argtypes = [ctypes.POINTER(Params), u32, u32, ctypes.POINTER(u32),
                                                      ctypes.POINTER(u32)]
        L.amvpt_host_multi_stats.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(u64)] * 3
        L.amvpt_host_describe.argtypes = [ctypes.c_void_p, u32, u32, u32, ctypes.POINTER(ctypes.POINTER(SceneDesc)),
                                          ctypes.POINTER(ctypes.POINTER(ViewDesc)), ctypes.POINTER(Params)]
        L.amvpt_host_integrator_string.argtypes = [ctypes.c_void_p]
        L.amvpt_host_integrator_string.restype = ctypes.c_char_p
        L.amvpt_host_write_exr.argtypes = [ctypes.c_char_p, ctypes.c_void_p, u32, u32, u32]
        L.amvpt_host_read_exr.argtypes = [ctypes.c_char_p, ctypes.c_void_p, u32, u32, u32]
        L.amvpt_host_parse_fov.argtypes = [f64, ctypes.c_char_p, ctypes.c_char_p, f64]
        L.amvpt_host_parse_fov.restype = f64
        L.amvpt_host_perspective_projection.argtypes = [ctypes.POINTER(ctypes.c_int)] * 3 + [f32, f32, f32,
                                                                                              ctypes.POINTER(f32)]
        _host = L
    return _host


def _defines(kw):
    keys = [k.encode() for k in kw]
    vals = [str(v).encode() for v in kw.values()]
    K = (ctypes.c_char_p * max(1, len(keys)))(*keys)
    V = (ctypes.c_char_p * max(1, len(vals)))(*vals)
    return K, V, len(keys)


def _check(rc, lib):
    if rc != 0:
        raise RuntimeError((lib.amvpt_host_last_error() if lib is _host else lib.amvpt_last_error()).decode())


class Scene:
    """A loaded scene (Scene + its sensors/integrator), as `mi.load_file` returns."""

    def __init__(self, handle):
        self._h = handle
        self._lib = host_lib()

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.amvpt_host_scene_free(self._h)
            self._h = None

    def sensor_count(self):
        return self._lib.amvpt_host_sensor_count(self._h)

    def film_info(self, sensor=0):
        w, h, c, s = u32(), u32(), u32(), u32()
        _check(self._lib.amvpt_host_film_info(self._h, sensor, w, h, c, s), self._lib)
        return w.value, h.value, c.value, s.value

    def integrator_string(self):
        return self._lib.amvpt_host_integrator_string(self._h).decode()

    def describe(self, sensor=0, seed=0, spp=0):
        """(SceneDesc*, ViewDesc*, Params) exactly as render() passes them to the C-ABI."""
        sd = ctypes.POINTER(SceneDesc)()
        vd = ctypes.POINTER(ViewDesc)()
        p = Params()
        _check(self._lib.amvpt_host_describe(self._h, sensor, seed, spp, ctypes.byref(sd), ctypes.byref(vd),
                                             ctypes.byref(p)), self._lib)
        return sd, vd, p


def load_file(path, **defines):
    L = host_lib()
    K, V, n = _defines(defines)
    h = L.amvpt_host_load_file(path.encode(), K, V, n)
    if not h:
        raise RuntimeError(L.amvpt_host_last_error().decode())
    return Scene(h)


def load_string(xml, **defines):
    L = host_lib()
    K, V, n = _defines(defines)
    h = L.amvpt_host_load_string(xml.encode(), K, V, n)
    if not h:
        raise RuntimeError(L.amvpt_host_last_error().decode())
    return Scene(h)


def render(scene, sensor=0, seed=0, spp=0, raw=False, counters=None, stream=None):
    """Integrator::render(scene, sensor, seed, spp, develop=not raw) -> numpy (H, W, C), on the current
    device and `stream` (a hipStream_t handle; None: the default stream).  The device scene and the film
    are cached on the scene (render_stats)."""
    w, h, c, _ = scene.film_info(sensor)
    _, _, p = scene.describe(sensor, seed, spp)
    ch = (5 if p.film_alpha else 4) if raw else c
    out = np.zeros((h, w, ch), dtype=np.float32)
    cnt = counters if counters is not None else Counters()
    _check(scene._lib.amvpt_host_render_stream(scene._h, sensor, seed, spp, 1 if raw else 0,
                                               out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(stream or 0),
                                               ctypes.byref(cnt)), scene._lib)
    return out


def render_stats(scene):
    """render's cache counters on this scene: device-scene creations, film buffer allocations, renders."""
    a, b, c = u64(), u64(), u64()
    _check(scene._lib.amvpt_host_render_stats(scene._h, a, b, c), scene._lib)
    return {"scene_creates": a.value, "buffer_allocs": b.value, "renders": c.value}


def render_multi(scene, devices, sensor=0, seed=0, spp=0, raw=False, counters=None):
    """Integrator::render over several GPUs of this node (C++ threads, lane shards, one RCCL reduce of
    the RGBW ImageBlocks onto devices[0]; amvpt_host_render_multi) -> numpy (H, W, C)."""
    w, h, c, _ = scene.film_info(sensor)
    _, _, p = scene.describe(sensor, seed, spp)
    ch = (5 if p.film_alpha else 4) if raw else c
    out = np.zeros((h, w, ch), dtype=np.float32)
    cnt = counters if counters is not None else Counters()
    devs = (ctypes.c_int * len(devices))(*devices)
    _check(scene._lib.amvpt_host_render_multi(scene._h, sensor, seed, spp, 1 if raw else 0, devs, len(devices),
                                              out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cnt)), scene._lib)
    return out


def host_lane_shard(n_lanes, rank, world):
    """The C++ host's lane partition (amvpt_host_lane_shard), for checks against dist.lane_shard."""
    b, e = u64(), u64()
    host_lib().amvpt_host_lane_shard(n_lanes, rank, world, ctypes.byref(b), ctypes.byref(e))
    return b.value, e.value


def host_view_group_partition(params, rank, world):
    """The C++ host's view-group partition (amvpt_host_view_group_partition): (rect, window) or None."""
    r, w = (u32 * 4)(), (u32 * 4)()
    ok = host_lib().amvpt_host_view_group_partition(ctypes.byref(params), rank, world, r, w)
    return (tuple(r), tuple(w)) if ok else None


def multi_stats(scene):
    """render_multi's cache counters on this scene: scene creations, communicator inits, renders."""
    a, b, c = u64(), u64(), u64()
    _check(scene._lib.amvpt_host_multi_stats(scene._h, a, b, c), scene._lib)
    return {"scene_creates": a.value, "comm_inits": b.value, "renders": c.value}


def plan(params):
    L = hip_lib()
    spp, spl, npass, lanes = u32(), u32(), u32(), u64()
    _check(L.amvpt_plan(ctypes.byref(params), spp, spl, npass, lanes), L)
    return spp.value, spl.value, npass.value, lanes.value


# process-wide defaults of the legacy setters, also the defaults of render_ex's per-call options
_DEFAULTS = {"chunk_lanes": 0, "traversal": 0}


def set_traversal(mode):
    """BVH walk: 0 auto (brute force for tiny scenes), 1 wave-uniform, 2 per-lane (amvpt_set_traversal)."""
    L = hip_lib()
    _check(L.amvpt_set_traversal(u32(mode)), L)
    _DEFAULTS["traversal"] = int(mode)


def set_bvh_build(max_leaf_prims=4, traversal_cost=0.0):
    """SAH shape of later DeviceScene builds (amvpt_set_bvh_build)."""
    L = hip_lib()
    _check(L.amvpt_set_bvh_build(u32(max_leaf_prims), ctypes.c_float(traversal_cost)), L)


def set_chunk_lanes(n):
    L = hip_lib()
    _check(L.amvpt_set_chunk_lanes(u64(n)), L)
    _DEFAULTS["chunk_lanes"] = int(n)


# amvpt_exchange_fn: (ctx, local_count, *prefix, *total) -> 0 on success
ExchangeFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, u64, ctypes.POINTER(u64), ctypes.POINTER(u64))
_exchange_cb = None


def wrap_exchange(fn):
    """ctypes callback around `fn(local_count) -> (prefix, total)` (exceptions -> status 1)."""
    def cb(_ctx, local, prefix, total):
        try:
            pre, tot = fn(int(local))
            prefix[0], total[0] = int(pre), int(tot)
            return 0
        except Exception:   # noqa: BLE001 -- reported to the C side as a failed exchange
            return 1
    return ExchangeFn(cb)


def set_adaptive_exchange(fn):
    """Count exchange for adaptive renders over lane ranges (amvpt_set_adaptive_exchange).

    `fn(local_count) -> (prefix, total)`: flagged lanes in lower ranges and in the
    whole pass (see amvpt.dist.count_exchange); None clears it."""
    global _exchange_cb
    L = hip_lib()
    _exchange_cb = wrap_exchange(fn) if fn is not None else None
    _check(L.amvpt_set_adaptive_exchange(_exchange_cb if _exchange_cb else ExchangeFn(), None), L)


def scene_box_count(scene, sensor=0):
    """Box meshes amvpt_scene_create screens in the brute-force walks of `scene` (amvpt_scene_desc_boxes)."""
    L = hip_lib()
    sd, _, _ = scene.describe(sensor, 0, 0)
    L.amvpt_scene_desc_boxes.argtypes = [ctypes.c_void_p, ctypes.POINTER(u32)]
    n = u32()
    _check(L.amvpt_scene_desc_boxes(ctypes.cast(sd, ctypes.c_void_p), ctypes.byref(n)), L)
    return n.value


def release_device_memory(device=0):
    """Free the lane arena renders keep on `device` between frames (amvpt_release_device_memory, ABI 10)."""
    L = hip_lib()
    _check(L.amvpt_release_device_memory(int(device)), L)


def device_count():
    n = ctypes.c_int(0)
    hip_lib().amvpt_device_count(ctypes.byref(n))
    return n.value


def write_exr(path, img):
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w, c = img.shape
    L = host_lib()
    _check(L.amvpt_host_write_exr(path.encode(), img.ctypes.data_as(ctypes.c_void_p), w, h, c), L)


def read_exr(path, width, height, channels):
    out = np.zeros((height, width, channels), dtype=np.float32)
    L = host_lib()
    _check(L.amvpt_host_read_exr(path.encode(), out.ctypes.data_as(ctypes.c_void_p), width, height, channels), L)
    return out


def parse_fov(fov=0.0, fov_axis=None, focal_length=None, aspect=1.0):
    L = host_lib()
    r = L.amvpt_host_parse_fov(float(fov), fov_axis.encode() if fov_axis else None,
                               focal_length.encode() if focal_length else None, float(aspect))
    if r < 0:
        raise RuntimeError(L.amvpt_host_last_error().decode())
    return r


def perspective_projection(film_size, crop_size, crop_offset, fov_x, near_clip, far_clip):
    L = host_lib()
    I3 = ctypes.c_int * 2
    m = (f32 * 16)()
    L.amvpt_host_perspective_projection(I3(*film_size), I3(*crop_size), I3(*crop_offset), fov_x, near_clip,
                                        far_clip, m)
    return np.array(m[:], dtype=np.float32).reshape(4, 4)


class DeviceScene:
    """Direct handle on the C-ABI: amvpt_scene_create over host descriptors (bench / tests)."""

    def __init__(self, scene_desc_ptr):
        self._lib = hip_lib()
        h = ctypes.c_void_p()
        _check(self._lib.amvpt_scene_create(scene_desc_ptr, ctypes.byref(h)), self._lib)
        self.h = h

    def stats(self):
        n, p = u32(), u32()
        _check(self._lib.amvpt_scene_stats(self.h, n, p), self._lib)
        return n.value, p.value

    def bvh2(self):
        """(two-box BVH nodes, tree depth in inner nodes) -- amvpt_scene_bvh2 (0 nodes: threaded walks)"""
        n, d = u32(), u32()
        self._lib.amvpt_scene_bvh2.argtypes = [ctypes.c_void_p, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        _check(self._lib.amvpt_scene_bvh2(self.h, n, d), self._lib)
        return n.value, d.value

    def render(self, views_ptr, params, film_ptr, lane_begin=0, lane_end=2 ** 64 - 1, stream=None,
               counters=None):
        """amvpt_render over lanes [lane_begin, lane_end).  Without `counters` the render is not
        instrumented (no per-kernel event timing, no host synchronisation); with an amvpt.Counters
        it is filled (per-kernel HIP-event times, lane statistics) and returned."""
        _check(self._lib.amvpt_render(self.h, views_ptr, ctypes.byref(params), lane_begin, lane_end,
                                      ctypes.c_void_p(film_ptr), ctypes.c_void_p(stream),
                                      ctypes.byref(counters) if counters is not None else None),
               self._lib)
        return counters

    def render_ex(self, views_ptr, params, film_ptr, lanes=None, window=None, overflow_ptr=None,
                  overflow_capacity=0, stream=None, counters=None, chunk_lanes=None, traversal=None, flags=0,
                  exchange=None, records_ptr=None, record_pass=0, budget_mib=0):
        """amvpt_render_ex: `lanes` a LaneSet (None: the whole pass), `window` (x0, y0, width, height)
        of the quilt the film holds (None: the whole quilt), per-call options; `exchange` is
        `fn(run_lane_begin, run_count) -> (run_prefix, total)` (see amvpt.dist.run_exchange)."""
        if lanes is None:
            lanes = LaneSet(0, 2 ** 64 - 1, 0, 0, 0, 0)
        chunk_lanes = _DEFAULTS["chunk_lanes"] if chunk_lanes is None else chunk_lanes
        traversal = _DEFAULTS["traversal"] if traversal is None else traversal
        x0, y0, w, h = window if window is not None else (0, 0, params.film_width, params.film_height)
        fw = FilmWindow(ctypes.c_void_p(film_ptr), x0, y0, w, h, ctypes.c_void_p(overflow_ptr or 0),
                        overflow_capacity)
        cb = wrap_run_exchange(exchange) if exchange is not None else RunExchangeFn()
        o = RenderOpts(chunk_lanes, traversal, flags, cb, None, ctypes.c_void_p(records_ptr or 0), record_pass,
                       int(budget_mib))
        _check(self._lib.amvpt_render_ex(self.h, views_ptr, ctypes.byref(params), ctypes.byref(lanes),
                                         ctypes.byref(fw), ctypes.c_void_p(stream), ctypes.byref(o),
                                         ctypes.byref(counters) if counters is not None else None), self._lib)
        return counters

    def render_records(self, views_ptr, params, film_ptr, records_ptr, pass_index=0, lane_begin=0,
                       lane_end=2 ** 64 - 1, stream=None):
        _check(self._lib.amvpt_render_records(self.h, views_ptr, ctypes.byref(params), pass_index, lane_begin,
                                              lane_end, ctypes.c_void_p(film_ptr), ctypes.c_void_p(records_ptr),
                                              ctypes.c_void_p(stream)), self._lib)

    def __del__(self):
        if getattr(self, "h", None):
            self._lib.amvpt_scene_destroy(self.h)
            self.h = None
