"""bench.py -- Msamples/s of the AMVPT (`mvpath`) hot path on MI355X.

Workload (BASELINE.json metric): Cornell box seen by an
8-view grid sensor (4x2 quilt of 1024^2 views), 64 spp (4 passes of 16),
sa_reuse + sa_mis, reuse_count 8, max_depth 8, rr_depth 5, seed 0.
One step = one full frame of that workload on every rank (scene upload, film
allocation and plan are outside the timed region; inputs are resident in HBM).

Multi-GPU (one process per GPU, RCCL over xGMI): strong scaling by lane sharding
(SURVEY 8(e)).  Every rank renders the contiguous lane range lane_shard(L, r, N) of
every pass of the SAME 64-spp frame (a band of quilt rows; lanes keep their global
TEA seeds, so the image is the single-GPU one), and the RGBW ImageBlocks are summed
on rank 0 with one RCCL reduce inside the timed region.  `--weak` instead renders
passes [4r, 4r+4) of a (64*N)-spp frame (pass sharding; labelled "weak").

After the timed region rank 0 also reports `rmse_vs_oracle`: the per-pixel RMSE of
the developed film of a stated lane window of the same workload, HIP pipeline vs the
CPU oracle (oracle/, a restatement of mvpath; Dr.Jit llvm_rgb cannot be built here).

The JSON line carries the dominant kernel's roofline (HIP-event timing of the
kernel inside the timed region x its algorithmic bytes, DESIGN.md "Byte model")
and a CPU baseline: the oracle (CPU restatement, not Dr.Jit llvm_rgb) timed on
a bounded lane sample on this box's host cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "mitsuba3-amvpt_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "Msamples/sec (whole node), 8-view 1024² 64spp; per-pixel RMSE vs llvm_rgb"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


# SURVEY 8 config table.  M = the metric's workload (the default bench line); the others are
# reported on request (--config): C2 (4-view Cornell 512^2), C3 (Veach-MIS 8-view 1024^2 256 spp:
# glossy MIS, sphere lights; C4 = C3 lane-sharded over the node), C5 (the 32-view adaptive array:
# grid 8x4 of 2048^2 views, groups of 4, one 16-spp pass, adaptive 3) and `mesh` (config M's shape
# on the OBJ/PLY Cornell box: 3.6 k triangles, per-lane BVH walks).  All lane-sharded (strong).
CONFIGS = {
    "M": dict(scene="cbox_grid.xml", res=1024, spp=64, gx=4, gy=2, reuse=8, adaptive=0),
    "C2": dict(scene="cbox_grid.xml", res=512, spp=64, gx=2, gy=2, reuse=4, adaptive=0),
    "C3": dict(scene="veach_grid.xml", res=1024, spp=256, gx=4, gy=2, reuse=8, adaptive=0),
    "C5": dict(scene="cbox_grid.xml", res=2048, spp=16, gx=8, gy=4, reuse=4, adaptive=3),
    "mesh": dict(scene="cbox_mesh.xml", res=1024, spp=64, gx=4, gy=2, reuse=8, adaptive=0),
}


def group_size(p):
    """Views per group (mvpath.cpp:192-217)."""
    if not (p.sa_reuse and p.n_views > 1 and p.reuse_count != 1):
        return 1
    N = p.n_views
    G = min(p.reuse_count, N)
    if G == 0 or N % G:
        G = next((q for q in range(8, N) if N % q == 0), 0)
        if not G:
            G = next((q for q in range(8, 1, -1) if N % q == 0), 0) or N
    return G


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="M",
                    help="M: the metric's workload (default); C2, C3, C5, mesh: the other configs")
    ap.add_argument("--weak", action="store_true",
                    help="pass sharding: rank r renders its own passes of an (N x spp)-spp frame (weak scaling)")
    ap.add_argument("--rmse-lanes", type=int, default=1 << 20,
                    help="lanes of the RMSE window (0: skip); the window starts at quilt row H/4")
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--gx", type=int, default=None)
    ap.add_argument("--gy", type=int, default=None)
    ap.add_argument("--reuse", type=int, default=None)
    ap.add_argument("--adaptive", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    for k in ("res", "spp", "gx", "gy", "reuse", "adaptive"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)
    headline = cfg == CONFIGS["M"]   # PMC traffic in profiles/ was collected on exactly this workload
    scene_file = cfg.pop("scene")
    lane_sharded = not args.weak

    import torch
    import torch.distributed as dist

    import amvpt
    from amvpt import dist as adist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    hip = amvpt.hip_lib()
    hip.amvpt_set_device(local)

    scene = amvpt.load_file(os.path.join(REPO, "scenes", scene_file), **cfg)
    sd, vd, p = scene.describe(0, 0, 0)
    plan = amvpt.plan(p)
    spp, spp_pp, n_passes, lanes_per_pass = plan
    if lane_sharded:
        # strong scaling: this rank's lanes of every pass of ONE frame; the adaptive fill's
        # prefix/total come from one all-gather per pass (amvpt.dist.count_exchange)
        lane_begin, lane_end = adist.lane_shard(lanes_per_pass, rank, world)
        amvpt.set_adaptive_exchange(adist.count_exchange(device="cuda"))
    else:
        # pass sharding: this rank's passes are [rank*n_passes, (rank+1)*n_passes) of a world*spp frame
        lane_begin, lane_end = 0, 2 ** 64 - 1
        p = adist.pass_shard(p, rank, world, plan)
    dev = amvpt.DeviceScene(sd)
    C = 5 if p.film_alpha else 4
    film = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    samples_per_rank = (min(lane_end, lanes_per_pass) - lane_begin) * n_passes
    G = group_size(p)

    def step(counters=None):
        film.zero_()
        c = dev.render(vd, p, film.data_ptr(), lane_begin, lane_end, stream, counters)
        adist.reduce_film(film, dst=0)
        return c

    partition = "equal lane counts"
    if lane_sharded and world > 1 and args.warmup > 0:
        # load balance (outside the timed region): time this rank's range once, all-gather the
        # times and move the range boundaries to equal cost (amvpt.dist.balanced_shards)
        torch.cuda.synchronize()
        t_b = time.perf_counter()
        film.zero_()
        dev.render(vd, p, film.data_ptr(), lane_begin, lane_end, stream)
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t_b], dtype=torch.float64, device="cuda")
        ts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(ts, t)
        bounds = [adist.lane_shard(lanes_per_pass, r, world)[0] for r in range(world)] + [lanes_per_pass]
        bounds = adist.balanced_shards(bounds, [float(x.item()) for x in ts], align=max(64, 16 * spp_pp))
        lane_begin, lane_end = bounds[rank], bounds[rank + 1]
        samples_per_rank = (lane_end - lane_begin) * n_passes
        partition = "cost-balanced contiguous lane ranges (one timed warmup render per rank)"
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    total_samples = lanes_per_pass * n_passes * args.steps if lane_sharded else samples_per_rank * world * args.steps
    value = total_samples / elapsed / 1e6

    # ---- one instrumented frame (outside the timed region): per-kernel HIP-event times + lane counters
    cnt = amvpt.Counters()
    torch.cuda.synchronize()
    step(cnt)
    torch.cuda.synchronize()
    c = cnt.as_dict()
    lanes = c["lanes"]
    verts = c["vertices"]
    vbar = verts / max(1, lanes)
    hbar = c["reuse_lanes"] / max(1, lanes)
    stage_ms = {"primary": c["kernel_ms_primary"], "bounce": c["kernel_ms_bounce"], "splat": c["kernel_ms_splat"]}
    kms, kl = c["kernel_ms"], c["kernel_launches"]
    bytes_kernel = kernel_bytes(c, G, C)
    # the dominant single kernel (HIP events around each launch on the render stream)
    dom = max((k for k in kms if kl[k]), key=lambda k: kms[k])
    launches = kl[dom]
    per_launch_bytes = bytes_kernel[dom] / launches
    achieved = per_launch_bytes / (kms[dom] / launches * 1e-3) / 1e9
    kernel_name = {"k_splat": ("k_splat_multi<%d, %d>" % (G, C)) if G > 1 else "k_splat_single<%d>" % C,
                   "k_vis": "k_vis<%d," % G, "k_mv_primary": "k_mv_primary<%d," % G,
                   "k_prim_req": "k_prim_req<%d," % G, "k_suffix": "k_suffix_fused<",
                   "k_prim_hit": ("k_prim_hit_req<%d," % G) if kl.get("k_prim_req", 0) == 0 and G > 1
                   else "k_prim_hit<"}.get(dom, dom + "<")
    traffic, traffic_src = pmc_traffic(kernel_name, headline)
    valu = pmc_valu(kms, kl, G, headline)
    # SURVEY 8(d) whole-pipeline byte model
    P = p.film_width * p.film_height
    B_sample = 336.0 * vbar + 120.0 * (G - 1) * hbar + 32.0 * P / samples_per_rank
    pipeline_gbs = value / world * 1e6 * B_sample / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not p.adaptive:
        cpu = cpu_baseline(sd, vd, p, args.cpu_seconds)
    rmse = None
    if rank == 0 and args.rmse_lanes > 0 and not p.adaptive:
        rmse = rmse_window(dev, sd, vd, p, plan, args.rmse_lanes, stream)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if lane_sharded else "weak",
            "rmse_vs_oracle": rmse,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (%s on a %dx%d grid sensor; no external assets)" % (
                {"veach_grid.xml": "Veach-MIS-class scene: 4 GGX rough-conductor plates, 4 sphere lights",
                 "cbox_mesh.xml": "Cornell box of util.py:551-685 as OBJ/PLY meshes (3.6 k triangles)"}.get(
                    scene_file, "Cornell box of util.py:551-685"), p.grid_x, p.grid_y),
            "config": {
                "workload": "%s: %s, %d-view %dx%d per view (quilt %dx%d), %d spp%s (%d passes x %d), G=%d, sa_mis, "
                            "adaptive %d, max_depth 8, rr_depth 5, seed 0"
                            % (args.config, scene_file, p.n_views, cfg["res"], cfg["res"], p.film_width,
                               p.film_height, spp, "" if lane_sharded else "/GPU", n_passes, spp_pp, G,
                               p.adaptive),
                "samples_per_gpu_per_step": samples_per_rank,
                "partition": partition if lane_sharded else "pass-sharded",
                "adaptive_lanes_per_gpu_per_step": c["adaptive_lanes"],
                "parallelism": ("lane-sharded x%d (+ one count all-gather per pass) + RCCL reduce of the RGBW "
                                "ImageBlock" if lane_sharded else
                                "pass-sharded x%d + RCCL reduce of the RGBW ImageBlock") % world,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "kernel_symbol": kernel_name,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": int(per_launch_bytes),
                "avg_launch_ms": round(kms[dom] / launches, 4),
                "launches_per_step": launches,
                "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
                "kernel_ms": {k: round(v, 3) for k, v in kms.items() if kl[k]},
                "kernel_launches": {k: v for k, v in kl.items() if v},
                "kernel_bytes": {k: int(v) for k, v in bytes_kernel.items() if kl[k]},
                # VALU issue (the kernels are VALU/latency-bound, not HBM-bound): committed SQ PMC
                # wave-instruction counts per launch / this run's launch time, vs 1228.8 G/s
                "valu_issue": valu,
                "note": ("the dominant kernel keeps its paths in registers (k_suffix_fused): its algorithmic "
                         "HBM bytes are 96 B per path, so its HBM fraction is small by design; it is bound "
                         "by VALU issue (valu_issue) -- pipeline_model is the metric's roofline")
                        if dom == "k_suffix" else None,
                "pipeline_model": {"B_sample": round(B_sample, 1), "vbar": round(vbar, 4), "hbar": round(hbar, 4),
                                   "achieved_GBs": round(pipeline_gbs, 2),
                                   "frac": round(pipeline_gbs / HBM_PEAK_GBS, 5)},
            },
            "cpu_baseline": cpu,
            "counters": {k: c[k] for k in ("lanes", "vertices", "reuse_lanes", "visibility_rays", "view_splats",
                                             "nonfinite_samples", "negative_samples", "record_bytes",
                                             "splat_fallback")},
        }
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def rmse_window(dev, sd, vd, p, plan, n, stream):
    """Per-pixel RMSE (linear RGB, developed) of lanes [b, b + n) of every pass of the workload,
    HIP pipeline vs the CPU oracle.  The window starts at quilt row H/4 (through the cubes of the
    top row of views); every pixel that either film touched (W > 0) is compared -- the window's
    splats bleed into neighbouring rows and its reprojections into the other views."""
    import torch
    from amvpt import compare
    from oracle import oracle as O
    spp, spp_pp, n_passes, lanes_per_pass = plan
    W, H = p.film_width, p.film_height
    row = W * spp_pp                       # lanes per quilt row and pass
    b = min(lanes_per_pass, (H // 4) * row)
    e = min(lanes_per_pass, b + n)
    C = 5 if p.film_alpha else 4
    film = torch.zeros((H, W, C), dtype=torch.float32, device="cuda")
    dev.render(vd, p, film.data_ptr(), b, e, stream)
    torch.cuda.synchronize()
    g = film.cpu().numpy()
    del film
    threads = max(1, min(16, os.cpu_count() or 1))
    O.build()
    o, _, st = O.render(sd, vd, p, lane_begin=b, lane_end=e, threads=threads)
    touched = (g[..., -1] != 0) | (o[..., -1] != 0)
    m = compare.metrics(O.develop(g)[touched], O.develop(o)[touched])
    return {"rmse": m["rmse"], "max_abs": m["max_abs"], "pixels": int(touched.sum()),
            "window": "lanes [%d, %d) of each of the %d passes (quilt rows %d..%d)" % (
                b, e, n_passes, b // row, (e - 1) // row),
            "reference": "CPU oracle (restatement of mvpath, not Dr.Jit llvm_rgb)",
            "oracle_seconds": round(st["seconds"], 2)}


def kernel_bytes(c, G, C):
    """Algorithmic HBM bytes per frame of each kernel: every SoA
    stream element is written once by its producer and read once by its consumer."""
    lanes, verts, shadow = c["lanes"], c["vertices"], c["shadow_rays"]
    suffix = max(0, verts - lanes)        # suffix vertices (k_extend / k_bounce entries)
    pushed = min(lanes, suffix)           # paths that left the primary vertex (= paths that terminate)
    rec = c["record_bytes"] or 16         # lane records (4 x 16 B) + lane_out + view records (amvpt_counters)
    adapt = c["adaptive_lanes"]
    state = 80                            # path state: 5 float4 planes (store_state)
    nee = 52                              # NEE record: origin + destination, light point + thr, thr + contribution
    fused = c["kernel_launches"]["k_shadow"] == 0   # NEE traced inside k_bounce (brute-force scenes)
    return {
        # hit record out (+ the visibility requests when k_prim_req is fused into it)
        "k_prim_hit": (16 + (48 if c["kernel_launches"]["k_prim_req"] == 0 else 0)) * lanes,
        "k_prim_req": (16 + 48) * lanes,                            # hit in, visibility requests out
        "k_vis": (48 + G / 8.0) * lanes,                            # requests in (once), ballots out
        "k_mv_primary": (16 + G / 8.0 + rec) * lanes + state * pushed,  # hit + ballots in, records + paths out
        "k_raygen": state * (lanes if G == 1 else adapt),           # path state out
        "k_extend": 48 * suffix,                                    # ray in, hit out
        # state + hit in; survivors' state out; terminated paths' result out; NEE records out (split)
        "k_bounce": (state + 16) * suffix + state * (suffix - pushed) + 16 * pushed + (0 if fused else nee * shadow),
        "k_shadow": (nee + 32) * shadow,                            # NEE record in, result read-modify-write
        "k_splat": rec * lanes + 16 * adapt,                        # records in (film: PMC WRITE_SIZE)
        # fused suffix (brute-force scenes): each path's state in once, its result out once; the
        # vertices in between stay in registers
        "k_suffix": (state + 16) * pushed,
    }


def pmc_traffic(kernel_name, full_size):
    """HBM bytes per launch of `kernel_name` from the newest committed rocprofv3 PMC summary
    (profiles/r*_traffic.json, made by tools/pmc_traffic.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this bench at config M).  None when no summary matches."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_traffic.json")))
    if not files or not full_size:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    key = kernel_name.replace(" ", "")
    for k, v in d["kernels"].items():
        if key in k.replace(" ", ""):
            return int(v["hbm_bytes_per_launch"]), os.path.relpath(files[-1], REPO)
    return None, os.path.relpath(files[-1], REPO)


def pmc_valu(kms, kl, G, full_size):
    """Per kernel: VALU wave-instructions per launch (newest profiles/r*_valu.json, made by
    tools/pmc_valu.py from a SQ PMC pass of this bench at config M) over this run's mean launch
    time, as a fraction of the chip's VALU issue peak.  None off config M."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_valu.json")))
    if not files or not full_size:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    peak = d["peak_valu_ginst_s"]
    sym = {"k_splat": "k_splat_multi<%d," % G, "k_vis": "k_vis<%d," % G, "k_mv_primary": "k_mv_primary<%d," % G,
           "k_prim_req": "k_prim_req<%d," % G, "k_suffix": "k_suffix_fused<",
           "k_prim_hit": ("k_prim_hit_req<%d," % G) if kl.get("k_prim_req", 0) == 0 and G > 1 else "k_prim_hit<"}
    out = {"peak_Ginst_s": peak, "source": os.path.relpath(files[-1], REPO), "kernels": {}}
    for k in kms:
        if not kl[k]:
            continue
        key = sym.get(k, k + "<")
        hit = [v for n, v in d["kernels"].items() if key in n]
        if not hit:
            continue
        ginst = hit[0]["valu_insts_per_launch"] / (kms[k] / kl[k] * 1e-3) / 1e9
        out["kernels"][k] = {"valu_per_wave": round(hit[0]["valu_per_wave"], 1), "achieved_Ginst_s": round(ginst, 1),
                             "frac": round(ginst / peak, 4)}
    return out


def cpu_baseline(sd, vd, p, target_seconds):
    """Oracle (CPU restatement of mvpath, not Dr.Jit llvm_rgb) on a bounded lane sample of pass 0."""
    from oracle import oracle as O
    threads = max(1, min(16, os.cpu_count() or 1))
    try:
        O.build()
        n = 1 << 16
        while True:
            _, _, st = O.render(sd, vd, p, lane_begin=0, lane_end=n, threads=threads)
            if st["seconds"] >= 0.6 * target_seconds or n >= (1 << 27):
                break
            n = int(min(1 << 27, n * max(2.0, 1.2 * target_seconds / max(st["seconds"], 1e-3))))
            n = (n // 4096) * 4096
        return {"value": round(n / st["seconds"] / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
                "sample": "lanes [0, %d) of pass 0 of the same workload (%.1f s); CPU restatement of mvpath "
                          "(oracle/, brute-force intersection), not Dr.Jit llvm_rgb" % (n, st["seconds"])}
    except Exception as e:  # the baseline is reported, never the product path
        return {"value": None, "unit": "Msamples/s", "cores": threads, "kind": "port", "sample": "failed: %s" % e}


if __name__ == "__main__":
    main()
