"""Timed Msamples/s of config M (or $AB_CONFIG) for each variant: a library dir or an environment setting.

    python tools/ab_value.py <libdir> [<libdir> ...]    (dirs relative to mitsuba3-amvpt_amd/)
    python tools/ab_value.py --env AMVPT_BRUTE=0 --env AMVPT_BRUTE=1 ...   (current lib/)
Each variant runs in its own child process (one ctypes load per process).  With --kernels
the child also reports one instrumented frame's per-kernel HIP-event ms (ABI >= 4 only).
"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# bench.py's workloads (AB_CONFIG selects one; default M)
CONFIGS = {
    "M": dict(scene="cbox_grid.xml", res=1024, spp=64, gx=4, gy=2, reuse=8),
    "C3": dict(scene="veach_grid.xml", res=1024, spp=256, gx=4, gy=2, reuse=8),
    "mesh": dict(scene="cbox_mesh.xml", res=1024, spp=64, gx=4, gy=2, reuse=8),
    "C5": dict(scene="cbox_grid.xml", res=2048, spp=16, gx=8, gy=4, reuse=4, adaptive=3),
}


def child(steps=3, kernels=False):
    sys.path[:0] = [REPO, os.path.join(REPO, "mitsuba3-amvpt_amd")]
    import torch
    import amvpt
    if os.environ.get("AB_CHUNK"):
        amvpt.set_chunk_lanes(int(os.environ["AB_CHUNK"]))
    if os.environ.get("AB_TRAV"):
        amvpt.set_traversal(int(os.environ["AB_TRAV"]))
    if os.environ.get("AB_BVH"):   # "max_leaf_prims:traversal_cost" for the scene build (amvpt_set_bvh_build)
        leaf, cost = os.environ["AB_BVH"].split(":")
        amvpt.hip_lib().amvpt_set_bvh_build(int(leaf), float(cost))
    cfg = dict(CONFIGS[os.environ.get("AB_CONFIG", "M")])
    scene = cfg.pop("scene")
    s = amvpt.load_file(os.path.join(REPO, "scenes", scene), **cfg)
    sd, vd, p = s.describe(0, 0, 0)
    spp = cfg["spp"]
    dev = amvpt.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    lanes = p.film_width * p.film_height * spp
    flags = int(os.environ.get("AB_FLAGS", "0"), 0)   # amvpt_render_opts.flags (e.g. 32: OPT_NO_BINNING)

    def frame(**kw):
        if flags or kw:
            dev.render_ex(vd, p, film.data_ptr(), flags=flags | kw.pop("flags", 0), **kw)
        else:
            dev.render(vd, p, film.data_ptr())

    frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        frame()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"variant": os.environ.get("AB_VARIANT", "lib"), "msamples_s": round(lanes * steps / dt / 1e6, 2),
           "ms_per_frame": round(dt * 1e3 / steps, 2)}
    if hasattr(dev._lib, "amvpt_scene_bvh2"):
        out["bvh2"] = dev.bvh2()   # (two-box BVH nodes, depth): 0 nodes = the threaded walks
    if kernels:
        # one instrumented frame with every chunk on one stream (per-kernel event times do not overlap)
        c = amvpt.Counters()
        if hasattr(amvpt, "OPT_ONE_STREAM"):
            frame(counters=c, flags=amvpt.OPT_ONE_STREAM)
        else:
            dev.render(vd, p, film.data_ptr(), counters=c)
        torch.cuda.synchronize()
        d = c.as_dict()
        out["kernel_ms"] = {k: round(v, 2) for k, v in d["kernel_ms"].items() if v}
    print(json.dumps(out), flush=True)


def main():
    args = sys.argv[1:]
    kernels = "--kernels" in args
    args = [a for a in args if a != "--kernels"]
    if args[:1] == ["--child"]:
        child(kernels=kernels)
        return
    variants = []
    while args:
        a = args.pop(0)
        if a == "--env":
            kv = args.pop(0)
            env = dict(os.environ, AB_VARIANT=kv)
            for item in kv.split(","):
                k, v = item.split("=", 1)
                env[k] = v
            variants.append(env)
        else:
            variants.append(dict(os.environ, AB_VARIANT=a, AMVPT_LIB_DIR=os.path.join(REPO, "mitsuba3-amvpt_amd", a)))
    for env in variants:
        cmd = [sys.executable, os.path.abspath(__file__), "--child"] + (["--kernels"] if kernels else [])
        subprocess.run(cmd, env=env, check=True, timeout=300)


if __name__ == "__main__":
    main()
