"""
oracle.py -- TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU parity oracle
(oracle/build/liboracle.so, built from oracle/amvpt_oracle.cpp by oracle/Makefile).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product path never does.
"""
import ctypes
import os
import subprocess

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")
_lib = None


class OracleStats(ctypes.Structure):
    _fields_ = [("lanes", ctypes.c_uint64), ("vertices", ctypes.c_uint64), ("reuse_lanes", ctypes.c_uint64),
                ("visibility_rays", ctypes.c_uint64), ("adaptive_lanes", ctypes.c_uint64),
                ("seconds", ctypes.c_double), ("range_drops", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.POINTER(OracleStats)]
        L.oracle_plan.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 5
        L.oracle_set_exchange.argtypes = [ExchangeFn, ctypes.c_void_p]
        L.oracle_set_run_exchange.argtypes = [RunExchangeFn, ctypes.c_void_p]
        L.oracle_set_fixed_film.argtypes = [ctypes.c_int]
        L.oracle_set_bvh.argtypes = [ctypes.c_int]
        L.oracle_primary_hits.restype = ctypes.c_int
        L.oracle_primary_hits.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_render_rect.restype = ctypes.c_int
        L.oracle_render_rect.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint32] * 4 + [
            ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(OracleStats)]
        L.oracle_tea_float32.restype = ctypes.c_float
        L.oracle_tea_float64.restype = ctypes.c_double
        L.oracle_gaussian_eval.restype = ctypes.c_float
        L.oracle_gaussian_eval.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_microfacet_eval.restype = ctypes.c_float
        L.oracle_microfacet_eval.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        L.oracle_microfacet_smith_g1.restype = ctypes.c_float
        L.oracle_microfacet_smith_g1.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                                 ctypes.c_void_p]
        L.oracle_microfacet_pdf.restype = ctypes.c_float
        L.oracle_microfacet_pdf.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_float, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_microfacet_sample.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_float, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                               ctypes.c_void_p]
        L.oracle_fresnel_conductor.restype = ctypes.c_float
        L.oracle_fresnel_conductor.argtypes = [ctypes.c_float] * 3
        L.oracle_film_put.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_float, ctypes.c_void_p, ctypes.c_float,
                                                             ctypes.c_float, ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_square_to_cosine_hemisphere.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        L.oracle_square_to_uniform_disk_concentric.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        L.oracle_sincos.argtypes = [ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_math.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_diffuse_eval_pdf.argtypes = [ctypes.c_void_p] * 5
        L.oracle_tea.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_tea_float32.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.oracle_tea_float64.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.oracle_pcg32_u32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_sampler_1d.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        _lib = L
    return _lib


def plan(params):
    L = lib()
    a, b, c, g = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    lanes = ctypes.c_uint64()
    L.oracle_plan(ctypes.byref(params), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(lanes),
                  ctypes.byref(g))
    return dict(spp=a.value, spp_per_pass=b.value, passes=c.value, lanes=lanes.value, group=g.value)


ExchangeFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                              ctypes.POINTER(ctypes.c_uint64))
_exchange_cb = None


def set_exchange(fn):
    """Adaptive fill over a lane range: `fn(local_count) -> (prefix, total)` once per pass."""
    global _exchange_cb
    if fn is None:
        _exchange_cb = None
        lib().oracle_set_exchange(ExchangeFn(), None)
        return

    def cb(_ctx, local, prefix, total):
        try:
            pre, tot = fn(int(local))
            prefix[0], total[0] = int(pre), int(tot)
            return 0
        except Exception:   # noqa: BLE001
            return 1
    _exchange_cb = ExchangeFn(cb)
    lib().oracle_set_exchange(_exchange_cb, None)


RunExchangeFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64))
_run_exchange_cb = None


def set_run_exchange(fn):
    """Adaptive fill over a lane rectangle: `fn(run_lane_begin, run_count) -> (run_prefix, total)` once per
    pass (the amvpt_run_exchange_fn contract of include/amvpt.h)."""
    global _run_exchange_cb
    if fn is None:
        _run_exchange_cb = None
        lib().oracle_set_run_exchange(RunExchangeFn(), None)
        return

    def cb(_ctx, n, begins, counts, prefix, total):
        try:
            pre, tot = fn([int(begins[i]) for i in range(n)], [int(counts[i]) for i in range(n)])
            for i in range(n):
                prefix[i] = int(pre[i])
            total[0] = int(tot)
            return 0
        except Exception:   # noqa: BLE001
            return 1
    _run_exchange_cb = RunExchangeFn(cb)
    lib().oracle_set_run_exchange(_run_exchange_cb, None)


def render_rect(scene_desc_ptr, views_ptr, params, rect, threads=0, film=None):
    """Render the lanes of quilt pixels rect = (x0, y0, width, height) into a whole-quilt film."""
    L = lib()
    C = 5 if params.film_alpha else 4
    if film is None:
        film = np.zeros((params.film_height, params.film_width, C), dtype=np.float32)
    st = OracleStats()
    rc = L.oracle_render_rect(ctypes.cast(scene_desc_ptr, ctypes.c_void_p), ctypes.cast(views_ptr, ctypes.c_void_p),
                              ctypes.addressof(params), *[int(v) for v in rect], film.ctypes.data, threads,
                              ctypes.byref(st))
    if rc != 0:
        raise RuntimeError("oracle_render_rect failed (status %d)" % rc)
    return film, st.as_dict()


def set_bvh(on):
    """Closest-hit / any-hit queries through a BVH (scenes of > 64 primitives) instead of brute force: the same hits
    (the (t, index) rule); bench.py's CPU baseline uses it, the parity tests do not."""
    lib().oracle_set_bvh(1 if on else 0)


def render(scene_desc_ptr, views_ptr, params, lane_begin=0, lane_end=2 ** 64 - 1, threads=0,
           record_pass=None, film=None, fixed_film=False):
    """Render into a (H, W, C) float32 film; optionally return per-lane records of one pass.
    fixed_film: accumulate as the device's AMVPT_OPT_DETERMINISTIC film does (32.32 fixed-point integer
    sums, converted once), which makes the film independent of summation order: bit-comparable."""
    L = lib()
    L.oracle_set_fixed_film(1 if fixed_film else 0)
    try:
        return _render(L, scene_desc_ptr, views_ptr, params, lane_begin, lane_end, threads, record_pass, film)
    finally:
        L.oracle_set_fixed_film(0)


def _render(L, scene_desc_ptr, views_ptr, params, lane_begin, lane_end, threads, record_pass, film):
    C = 5 if params.film_alpha else 4
    if film is None:
        film = np.zeros((params.film_height, params.film_width, C), dtype=np.float32)
    rec = None
    if record_pass is not None:
        pl = plan(params)
        end = min(lane_end, pl["lanes"])
        rec = np.zeros((max(0, end - lane_begin), pl["group"], 8), dtype=np.float32)
    st = OracleStats()
    rc = L.oracle_render(ctypes.cast(scene_desc_ptr, ctypes.c_void_p), ctypes.cast(views_ptr, ctypes.c_void_p),
                         ctypes.addressof(params), lane_begin, lane_end, film.ctypes.data, threads,
                         rec.ctypes.data if rec is not None else None,
                         record_pass if record_pass is not None else 0, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError("oracle_render failed (status %d: unsupported configuration)" % rc)
    return film, rec, st.as_dict()


def f32(*vals):
    return np.ascontiguousarray(np.array(vals, dtype=np.float32))


def film_put(film, x, y, values, stddev=0.5, box=False, coalesce=True):
    """ImageBlock::put of one sample into `film` (H, W, C float32, modified in place)."""
    H, W, C = film.shape
    v = f32(*values)
    lib().oracle_film_put(W, H, C, 1 if box else 0, stddev, film.ctypes.data, x, y, v.ctypes.data,
                          1 if coalesce else 0)
    return film


def develop(film, alpha=False):
    """hdrfilm develop: RGB[A] / W (W == 0 -> 1), hdrfilm.cpp:400."""
    w = film[..., -1:]
    n = 4 if alpha else 3
    return film[..., :n] / np.where(w == 0, 1.0, w)


def primary_hits(scene_desc_ptr, views_ptr, params):
    """(H, W, 8) float32: primary hit through each quilt pixel centre -- shape index (-1: miss), geometric
    normal, hit point, view index (scene geometry only; the unbiasedness gate's edge mask)."""
    out = np.zeros((params.film_height, params.film_width, 8), dtype=np.float32)
    rc = lib().oracle_primary_hits(ctypes.cast(scene_desc_ptr, ctypes.c_void_p), ctypes.cast(views_ptr, ctypes.c_void_p),
                                   ctypes.addressof(params), out.ctypes.data)
    if rc != 0:
        raise RuntimeError("oracle_primary_hits failed (status %d)" % rc)
    return out
