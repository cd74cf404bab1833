"""bench.py -- Msamples/s of the AMVPT (`mvpath`) hot path on MI355X.

Workload (BASELINE.json metric): Cornell box seen by an
8-view grid sensor (4x2 quilt of 1024^2 views), 64 spp (4 passes of 16),
sa_reuse + sa_mis, reuse_count 8, max_depth 8, rr_depth 5, seed 0.
One step = one full frame of that workload on every rank (scene upload, film
allocation and plan are outside the timed region; inputs are resident in HBM).

Multi-GPU (one process per GPU, RCCL over xGMI): strong scaling; every rank
renders its share of the SAME frame (lanes keep their global TEA seeds, so the image is the
single-GPU one) inside the timed region, and rank 0 ends the step holding the whole ImageBlock:
  * view groups (C5, "4 views per GPU"; the default whenever the groups divide among the ranks):
    rank r renders the lanes of its groups' quilt tiles into a film window of those tiles + a
    4-px filter border (amvpt_render_ex), and the windows are gathered on rank 0 (borders and the
    few overflow cells summed) -- no full-quilt film per rank, no reduce;
  * lane bands (M / C3 / C4: one group of 8 views): rank r renders the contiguous lane range of
    a cost-balanced band of quilt rows of every pass, and the RGBW ImageBlocks are summed on
    rank 0 with one RCCL reduce.
`--weak` instead renders passes [4r, 4r+4) of a (64*N)-spp frame (pass sharding; labelled "weak").

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
    ap.add_argument("--partition", choices=("auto", "lanes", "view-groups"), default="auto",
                    help="multi-GPU partition of the frame (auto: view groups when they divide among the ranks)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--one-stream", action="store_true",
                    help="every chunk on the render stream in the timed frames too (kernel-trace profiles: "
                         "per-kernel durations that do not overlap; the default keeps the second chunk stream)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    for k in ("res", "spp", "gx", "gy", "reuse", "adaptive"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)
    prof_config = args.config if cfg == CONFIGS[args.config] else "custom"   # workload key of the PMC summaries
    scene_file = cfg.pop("scene")
    lane_sharded = not args.weak

    import torch
    import torch.distributed as dist

    import amvpt
    from amvpt import dist as adist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AMVPT_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks sharing the visible devices
    # (rank -> device local % count; collectives staged through the host, amvpt.dist.comm_device): a check
    # of the partitions and exchanges on real renders, not a measurement -- the metric runs over RCCL
    backend = os.environ.get("AMVPT_DIST_BACKEND", "nccl")
    if world > 1:
        dist.init_process_group(backend)
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    hip = amvpt.hip_lib()
    hip.amvpt_set_device(local)
    cdev = adist.comm_device("cuda")   # where this process group's collectives run

    scene = amvpt.load_file(os.path.join(REPO, "scenes", scene_file), **cfg)
    sd, vd, p = scene.describe(0, 0, 0)
    plan = amvpt.plan(p)
    spp, spp_pp, n_passes, lanes_per_pass = plan
    G = group_size(p)
    exchange = adist.run_exchange(device="cuda")   # per-call adaptive count exchange (amvpt_render_opts)
    groups = None
    if lane_sharded and world > 1 and args.partition != "lanes":
        groups = adist.view_group_partition(p, G, world)
        if groups is None and args.partition == "view-groups":
            raise SystemExit("view-group partition does not apply to this configuration / world size")
    if not lane_sharded:
        # pass sharding: this rank's passes are [rank*n_passes, (rank+1)*n_passes) of a world*spp frame
        p = adist.pass_shard(p, rank, world, plan)
    dev = amvpt.DeviceScene(sd)
    base_flags = amvpt.OPT_ONE_STREAM if args.one_stream else 0
    C = 5 if p.film_alpha else 4
    stream = torch.cuda.current_stream().cuda_stream
    quilt_bytes = p.film_width * p.film_height * C * 4
    if groups is not None:
        # view groups: this rank's tiles (lanes) and film window (tiles + filter border); rank 0 also
        # holds the whole quilt the windows are gathered into
        rect, win = groups[rank]
        wx0, wy0, ww, wh = win
        film = torch.zeros((wh, ww, C), dtype=torch.float32, device="cuda")
        ov_cap = 1 << 20
        overflow = torch.zeros(4 * (ov_cap + 1), dtype=torch.int32, device="cuda")
        quilt = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda") if rank == 0 else None
        lanes = amvpt.LaneSet(0, 0, *rect)
        samples_per_rank = rect[2] * rect[3] * spp_pp * n_passes
        partition = "view groups: %d groups of %d views per GPU, tiles %dx%d px + %d-px border window, gather to rank 0" % (
            p.n_views // G // world, G, rect[2], rect[3], adist.FILTER_BORDER)
        film_bytes = ww * wh * C * 4

        def step(counters=None, flags=0):
            film.zero_()
            overflow[:4].zero_()
            c = dev.render_ex(vd, p, film.data_ptr(), lanes=lanes, window=win, overflow_ptr=overflow.data_ptr(),
                              overflow_capacity=ov_cap, stream=stream, counters=counters, exchange=exchange,
                              flags=flags | base_flags)
            adist.gather_windows(film, win, overflow, quilt, [g[1] for g in groups], dst=0)
            return c
    else:
        if lane_sharded:
            # lane bands: this rank's lanes of every pass of ONE frame
            lane_begin, lane_end = adist.lane_shard(lanes_per_pass, rank, world)
        else:
            lane_begin, lane_end = 0, 2 ** 64 - 1
        film = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda")
        samples_per_rank = (min(lane_end, lanes_per_pass) - lane_begin) * n_passes
        partition = "equal lane counts" if lane_sharded else "pass-sharded"
        film_bytes = quilt_bytes
        band = [lane_begin, lane_end]

        def step(counters=None, flags=0):
            film.zero_()
            c = dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt.LaneSet(band[0], band[1], 0, 0, 0, 0),
                              stream=stream, counters=counters, exchange=exchange if world > 1 else None,
                              flags=flags | base_flags)
            adist.reduce_film(film, dst=0)
            return c

        if lane_sharded and world > 1 and args.warmup > 0:
            # load balance (outside the timed region): time this rank's range on a warm arena (one
            # untimed render first: the arena allocation and module load are one-time costs), from
            # the per-kernel HIP-event times (the adaptive exchange would synchronise the ranks'
            # wall clocks), all-gather the times and move the boundaries to equal cost
            dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt.LaneSet(band[0], band[1], 0, 0, 0, 0), stream=stream,
                          exchange=exchange)
            cb = amvpt.Counters()
            dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt.LaneSet(band[0], band[1], 0, 0, 0, 0), stream=stream,
                          counters=cb, exchange=exchange)
            own_ms = sum(cb.as_dict()["kernel_ms"].values())
            t = torch.tensor([own_ms], dtype=torch.float64, device=cdev)
            ts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(ts, t)
            shard_ms = [float(x.item()) for x in ts]
            bounds = [adist.lane_shard(lanes_per_pass, r, world)[0] for r in range(world)] + [lanes_per_pass]
            bounds = adist.balanced_shards(bounds, shard_ms, align=max(64, 16 * spp_pp))
            band[0], band[1] = bounds[rank], bounds[rank + 1]
            samples_per_rank = (band[1] - band[0]) * n_passes
            partition = ("cost-balanced bands of quilt rows (per-kernel time of a warm render per rank; measured "
                         "balance before %.3f)" % (sum(shard_ms) / world / max(shard_ms)))
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
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    total_samples = lanes_per_pass * n_passes * args.steps if lane_sharded else samples_per_rank * world * args.steps
    value = total_samples / elapsed / 1e6

    # ---- one instrumented frame (outside the timed region): per-kernel HIP-event times + lane counters.
    # Every chunk on the render stream (AMVPT_OPT_ONE_STREAM): with the second chunk stream the kernels of
    # two chunks overlap and their event intervals would double-count the frame (the same kernels and
    # results; the timed region above keeps the default two streams)
    cnt = amvpt.Counters()
    torch.cuda.synchronize()
    t_inst = time.perf_counter()
    step(cnt, flags=amvpt.OPT_ONE_STREAM)
    torch.cuda.synchronize()
    inst_frame_ms = (time.perf_counter() - t_inst) * 1e3
    c = cnt.as_dict()
    lanes = c["lanes"]
    verts = c["vertices"]
    vbar = verts / max(1, lanes)
    hbar = c["reuse_lanes"] / max(1, lanes)
    stage_ms = {"primary": c["kernel_ms_primary"], "bounce": c["kernel_ms_bounce"], "splat": c["kernel_ms_splat"]}
    kms, kl = c["kernel_ms"], c["kernel_launches"]
    bytes_kernel = kernel_bytes(c, G, C, min(p.adaptive, G - 1) if G > 1 else 0)
    # the dominant single kernel (HIP events around each launch on the render stream)
    dom = max((k for k in kms if kl[k]), key=lambda k: kms[k])
    launches = kl[dom]
    per_launch_bytes = bytes_kernel[dom] / launches
    achieved = per_launch_bytes / (kms[dom] / launches * 1e-3) / 1e9
    kernel_name = {"k_splat": ("k_splat_multi<%d, %d," % (G, C)) if G > 1 else "k_splat_single<%d>" % C,
                   "k_vis": "k_vis<%d," % G, "k_mv_primary": "k_mv_primary<%d," % G,
                   "k_prim_req": "k_prim_req<%d," % G, "k_suffix": "k_suffix_fused<",
                   "k_prim_hit": ("k_prim_hit_req<%d," % G) if kl.get("k_prim_req", 0) == 0 and G > 1
                   else "k_prim_hit<"}.get(dom, dom + "<")
    rev = source_revision()
    traffic, traffic_src = pmc_traffic(kernel_name, prof_config, rev)
    valu = pmc_valu(kms, kl, G, prof_config, rev)
    hbm_frac = achieved / HBM_PEAK_GBS
    frame = frame_pmc(prof_config, rev, ms_per_step)
    valu_dom = (valu or {}).get("kernels", {}).get(dom)
    # the measured limiter of the dominant kernel: VALU issue (committed SQ counts of this code revision
    # over this run's launch time) vs algorithmic HBM bytes over the same time
    bound = "valu" if valu_dom and valu_dom["frac"] > hbm_frac else "hbm"
    # SURVEY 8(d) whole-pipeline byte model
    P = p.film_width * p.film_height
    B_sample = 336.0 * vbar + 120.0 * (G - 1) * hbar + 32.0 * P / (lanes_per_pass * n_passes)
    pipeline_gbs = value / world * 1e6 * B_sample / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not p.adaptive:
        cpu = cpu_baseline(sd, vd, p, args.cpu_seconds)
    rmse = None
    if rank == 0 and args.rmse_lanes > 0 and not p.adaptive:
        print("[bench] RMSE window: %d lanes of every pass through the oracle" % args.rmse_lanes, file=sys.stderr,
              flush=True)
        rmse = rmse_window(dev, sd, vd, p, plan, args.rmse_lanes, stream)
    elif rank == 0 and args.rmse_lanes > 0:
        # the adaptive fill compacts and re-traces over the WHOLE pass, so no lane window of the full-size
        # frame can include it: the same workload at reduced view size, whole frame, fill included (and, on
        # one GPU, the oracle's time for it is the CPU baseline's sample)
        rmse, cpu_small = rmse_reduced_frame(scene_file, cfg, stream)
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_small

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world if backend != "gloo" else torch.cuda.device_count(),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if lane_sharded else "weak",
            "chunk_streams": 1 if args.one_stream else "auto (up to 4 for the per-depth wavefront suffix of BVH scenes)",
            "rmse_vs_oracle": rmse,
            "vs_baseline": None,
            **({"ranks": world, "dist_backend": backend,
                "note": "rehearsal: %d ranks share %d device(s) over gloo (host-staged collectives); a check of the "
                        "multi-rank path, not a measurement" % (world, torch.cuda.device_count())}
               if backend == "gloo" and world > 1 else {}),
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
                "film_bytes_per_gpu": film_bytes,
                "adaptive_lanes_per_gpu_per_step": c["adaptive_lanes"],
                "parallelism": (("view groups x%d (+ one per-row count all-gather per pass) + gather of the film "
                                 "windows to rank 0" if groups is not None else
                                 "lane bands x%d (+ one count all-gather per pass) + RCCL reduce of the RGBW "
                                 "ImageBlock") if lane_sharded else
                                "pass-sharded x%d + RCCL reduce of the RGBW ImageBlock") % world,
            },
            "roofline": {
                "bound": bound,
                "kernel": dom,
                "kernel_symbol": kernel_name,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(hbm_frac, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "source_revision": rev,
                "algorithmic_bytes_per_launch": int(per_launch_bytes),
                "avg_launch_ms": round(kms[dom] / launches, 4),
                "launches_per_step": launches,
                "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
                "kernel_ms": {k: round(v, 3) for k, v in kms.items() if kl[k]},
                # kernel_ms come from one instrumented frame with every chunk on one stream (no overlapped
                # intervals): they sum to at most this frame's wall time, which can exceed ms_per_step where
                # the timed frames run two chunk streams (the per-depth wavefront suffix of BVH scenes)
                "instrumented_frame_ms": round(inst_frame_ms, 3),
                "kernel_launches": {k: v for k, v in kl.items() if v},
                "kernel_bytes": {k: int(v) for k, v in bytes_kernel.items() if kl[k]},
                # VALU issue (the kernels are VALU/latency-bound, not HBM-bound): committed SQ PMC
                # wave-instruction counts per launch / this run's launch time, vs 1228.8 G/s
                "valu_issue": valu,
                "note": ("the dominant kernel keeps its paths in registers (k_suffix_fused): its algorithmic "
                         "HBM bytes are 96 B per pushed path, so its HBM fraction is small by design; bound = "
                         "the larger of its VALU-issue and HBM fractions -- pipeline_model is the metric's "
                         "roofline") if dom == "k_suffix" else None,
                # the whole frame by the counters: every kernel's PMC bytes (FETCH x2 + WRITE,
                # committed profiles of this source revision) x its launches per frame, over this run's ms_per_step;
                # and the frame's VALU issue (committed SQ_INSTS_VALU per frame over ms_per_step x 1228.8 G/s)
                "frame_traffic": frame["traffic"],
                "frame_hbm_frac": frame["hbm_frac"],
                "frame_valu_issue": frame["valu_issue"],
                "frame_source": frame["source"],
                "pipeline_model": {"B_sample": round(B_sample, 1), "vbar": round(vbar, 4), "hbar": round(hbar, 4),
                                   "achieved_GBs": round(pipeline_gbs, 2),
                                   "frac": round(pipeline_gbs / HBM_PEAK_GBS, 5)},
            },
            "cpu_baseline": cpu,
            "counters": {k: c[k] for k in ("lanes", "vertices", "reuse_lanes", "visibility_rays", "view_splats",
                                             "nonfinite_samples", "negative_samples", "record_bytes",
                                             "splat_fallback", "pushed_paths", "film_overflow", "film_range_drops",
                                             "primary_record_bytes", "splat_record_bytes", "chunk_lanes",
                                             "buffer_sets", "arena_bytes")},
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
    threads = host_cores()[0]
    O.build()
    o, _, st = O.render(sd, vd, p, lane_begin=b, lane_end=e, threads=threads)
    touched = (g[..., -1] != 0) | (o[..., -1] != 0)
    m = compare.metrics(O.develop(g)[touched], O.develop(o)[touched])
    return {"rmse": m["rmse"], "max_abs": m["max_abs"], "pixels": int(touched.sum()),
            "window": "lanes [%d, %d) of each of the %d passes (quilt rows %d..%d)" % (
                b, e, n_passes, b // row, (e - 1) // row),
            "reference": "CPU oracle (restatement of mvpath, not Dr.Jit llvm_rgb)",
            "oracle_seconds": round(st["seconds"], 2)}


def rmse_reduced_frame(scene_file, cfg, stream, res=64):
    """Adaptive configs: per-pixel RMSE (developed) of the whole frame of the same workload with `res`^2
    views (grid, spp, groups and adaptive kept), HIP pipeline vs the CPU oracle -- the adaptive fill
    (mvpath_multi.h:52-59,79-115) included; and the oracle's time for that frame as a CPU baseline."""
    import torch
    import amvpt
    from amvpt import compare
    from oracle import oracle as O
    small = dict(cfg, res=res)
    s = amvpt.load_file(os.path.join(REPO, "scenes", scene_file), **small)
    sd, vd, p = s.describe(0, 0, 0)
    spp, spp_pp, n_passes, lanes_per_pass = amvpt.plan(p)
    C = 5 if p.film_alpha else 4
    dev = amvpt.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda")
    cnt = amvpt.Counters()
    dev.render_ex(vd, p, film.data_ptr(), stream=stream, counters=cnt)
    torch.cuda.synchronize()
    g = film.cpu().numpy()
    del film
    threads, machine = host_cores()
    O.build()
    o, _, st = O.render(sd, vd, p, threads=threads)
    touched = (g[..., -1] != 0) | (o[..., -1] != 0)
    m = compare.metrics(O.develop(g)[touched], O.develop(o)[touched])
    lanes = lanes_per_pass * n_passes
    rmse = {"rmse": m["rmse"], "max_abs": m["max_abs"], "pixels": int(touched.sum()),
            "window": "the whole frame of the workload at %dx%d per view (quilt %dx%d, %d lanes + %d adaptive "
                      "re-traces on the GPU, %d in the oracle)" % (res, res, p.film_width, p.film_height, lanes,
                                                                   cnt.adaptive_lanes, st["adaptive_lanes"]),
            "reference": "CPU oracle (restatement of mvpath, not Dr.Jit llvm_rgb)",
            "oracle_seconds": round(st["seconds"], 2)}
    # the adaptive fill compacts and re-traces the whole pass, so no bounded lane window of the full-size frame
    # exists: this baseline is measured on the reduced frame and says so (`reduced_frame`); vs_baseline never uses it
    cpu = {"value": round(lanes / st["seconds"] / 1e6, 4), "unit": "Msamples/s", "cores": threads,
           "host_cpus": machine, "kind": "port", "reduced_frame": {"res": res, "lanes": lanes},
           "sample": "the whole %dx%d-per-view frame above, adaptive fill included (%.1f s); CPU restatement of "
                     "mvpath (oracle/, brute-force intersection), not Dr.Jit llvm_rgb" % (res, res, st["seconds"])}
    return rmse, cpu


def kernel_bytes(c, G, C, n_adapt=0):
    """Algorithmic HBM bytes per frame of each kernel: every SoA
    stream element is written once by its producer and read once by its consumer."""
    lanes, verts, shadow = c["lanes"], c["vertices"], c["shadow_rays"]
    suffix = max(0, verts - lanes)        # suffix vertices (k_extend / k_bounce entries)
    pushed = c["pushed_paths"]            # paths that entered the suffix (device counter; = paths that terminate)
    rec = c["record_bytes"] or 16         # lane records (4 x 16 B) + lane_out + view records (amvpt_counters)
    lane_rec = (80 if c["record_bytes"] else 16) * lanes   # the lane part: 4 lane-record planes + lane_out
    vrec_w, vrec_r = c.get("primary_record_bytes", 0), c.get("splat_record_bytes", 0)
    adapt = c["adaptive_lanes"]
    state = 80                            # path state: 5 float4 planes (store_state)
    nee = 40                              # NEE record: origin + destination, light point + the visible result
    fused = c["kernel_launches"]["k_shadow"] == 0   # NEE traced inside k_bounce (brute-force scenes)
    return {
        # hit record out (+ the visibility requests when k_prim_req is fused into it)
        "k_prim_hit": (16 + (48 if c["kernel_launches"]["k_prim_req"] == 0 else 0)) * lanes,
        "k_prim_req": (16 + 48) * lanes,                            # hit in, visibility requests out
        "k_vis": (48 + G / 8.0) * lanes,                            # requests in (once), ballots out
        # hit + ballots in, lane records + view records + paths out (view records: the device's count of the bytes
        # written, 4 per view in all-diffuse waves, 32 otherwise; ABI 10)
        "k_mv_primary": (16 + G / 8.0) * lanes + lane_rec + (vrec_w if vrec_w else (rec - lane_rec / max(1, lanes)) * lanes)
                        + state * pushed,
        "k_raygen": state * (lanes if G == 1 else adapt),           # path state out
        "k_extend": 48 * suffix,                                    # ray in, hit out
        # state + hit in; survivors' state out; terminated paths' result out; NEE records out (split)
        "k_bounce": (state + 16) * suffix + state * (suffix - pushed) + 16 * pushed + (0 if fused else nee * shadow),
        "k_shadow": (nee + 12) * shadow,                            # NEE record in, the visible result written
        # lane records in + the view records it reads (device count: only visited / splatting / indirect views,
        # ABI 10); film: PMC WRITE_SIZE
        "k_splat": lane_rec + (vrec_r if vrec_r else (rec - lane_rec / max(1, lanes)) * lanes) + 16 * adapt,
        # fused suffix (brute-force scenes): each path's state in once, its result out once; the
        # vertices in between stay in registers
        "k_suffix": (state + 16) * pushed,
        # the adaptive fill's compaction: 1 B of mask per lane in, 4 B per selected lane out
        "k_select": lanes + 4 * adapt / max(1, n_adapt),
        # ray binning: each binned ray read twice (histogram, scatter) and written once in bin order
        "k_bin": 96 * (suffix + (shadow if not fused else 0)),
    }


def source_revision():
    """Revision stamp of the kernel sources (sha256 over csrc/, first 16 hex digits): committed PMC
    summaries carry the stamp of the code they were measured on, and the bench uses only matching ones."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(PKG, "csrc")
    for n in sorted(os.listdir(d)):
        if n.endswith((".hip", ".h", ".cpp")):
            h.update(n.encode())
            h.update(open(os.path.join(d, n), "rb").read())
    return h.hexdigest()[:16]


def _profile(pattern, config, rev):
    """Newest committed profile summary (profiles/<pattern>) measured on this config and source revision;
    (data, path) or (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", pattern)), key=os.path.getmtime)
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        if d.get("config", "M") == config and d.get("source_revision") == rev:
            return d, os.path.relpath(f, REPO)
    return None, "no profiles/%s for config %s at source revision %s (stale profiles refused)" % (pattern, config, rev)


def pmc_traffic(kernel_name, config, rev):
    """HBM bytes per launch of `kernel_name` from a committed rocprofv3 PMC summary (profiles/r*_traffic.json,
    tools/pmc_traffic.py: separate FETCH_SIZE and WRITE_SIZE passes of this bench) of this config and
    source revision; (None, reason) otherwise."""
    d, src = _profile("r*_traffic*.json", config, rev)
    if d is None:
        return None, src
    key = kernel_name.replace(" ", "")
    for k, v in d["kernels"].items():
        if key in k.replace(" ", ""):
            return int(v["hbm_bytes_per_launch"]), src
    return None, src


def frame_pmc(config, rev, ms_per_step):
    """Whole-frame counters from the committed profiles of this config and source revision: HBM bytes per frame
    (each kernel's FETCH x2 + WRITE per launch x its launches, over the frames the profiled run rendered), their
    fraction of the HBM peak over ms_per_step, and the frame's VALU wave-instructions over ms_per_step x the issue
    peak (a time-weighted VALU-issue fraction of the whole frame)."""
    out = {"traffic": None, "hbm_frac": None, "valu_issue": None, "source": []}
    t, src = _profile("r*_traffic*.json", config, rev)
    out["source"].append(src)
    if t is not None:
        frames = t.get("frames_profiled", 2)
        out["traffic"] = int(sum(v["hbm_bytes_per_launch"] * v["launches"] for v in t["kernels"].values()) / frames)
        out["hbm_frac"] = round(out["traffic"] / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9), 5)
    v, src = _profile("r*_valu*.json", config, rev)
    out["source"].append(src)
    if v is not None:
        frames = v.get("frames_profiled", 2)
        insts = sum(k["valu_insts_per_launch"] * k["launches"] for k in v["kernels"].values()) / frames
        out["valu_issue"] = round(insts / (ms_per_step * 1e-3) / (v["peak_valu_ginst_s"] * 1e9), 5)
    return out


def pmc_valu(kms, kl, G, config, rev):
    """Per kernel: VALU wave-instructions per launch (committed profiles/r*_valu.json of this config and source
    revision, tools/pmc_valu.py) over this run's mean launch time, as a fraction of the chip's VALU issue peak."""
    d, src = _profile("r*_valu*.json", config, rev)
    if d is None:
        return {"source": src, "kernels": {}}
    peak = d["peak_valu_ginst_s"]
    sym = {"k_splat": ("k_splat_multi<%d," % G) if G > 1 else "k_splat_single<", "k_vis": "k_vis<%d," % G, "k_mv_primary": "k_mv_primary<%d," % G,
           "k_prim_req": "k_prim_req<%d," % G, "k_suffix": "k_suffix_fused<",
           "k_prim_hit": ("k_prim_hit_req<%d," % G) if kl.get("k_prim_req", 0) == 0 and G > 1 else "k_prim_hit<"}
    out = {"peak_Ginst_s": peak, "source": src, "kernels": {}}
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


def host_cores():
    """(usable, machine): the host CPUs this process may run on -- its affinity set, bounded by the cgroup
    CPU quota when one is set (a GPU box's share of a larger machine) -- and os.cpu_count()."""
    machine = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else machine
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and txt and txt[0] != "max":
            usable = min(usable, max(1, int(int(txt[0]) / int(txt[1]))))
        elif path.endswith("quota_us") and txt and int(txt[0]) > 0:
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            usable = min(usable, max(1, int(txt[0]) // period))
        break
    return usable, machine


def cpu_baseline(sd, vd, p, target_seconds):
    """Oracle (CPU restatement of mvpath, not Dr.Jit llvm_rgb) on a bounded lane sample of pass 0, one
    thread per usable host core."""
    from oracle import oracle as O
    threads, machine = host_cores()
    n_prims = sum(sd[0].shapes[i].face_count if sd[0].shapes[i].type == 1 else 1 for i in range(sd[0].shape_count))
    bvh = n_prims > 64   # BVH scenes: the oracle's own BVH (oracle_set_bvh; same hits), not a brute-force scan
    try:
        O.build()
        O.set_bvh(bvh)
        n = 1 << 16
        while True:
            _, _, st = O.render(sd, vd, p, lane_begin=0, lane_end=n, threads=threads)
            print("[bench] cpu baseline: %d lanes in %.1f s" % (n, st["seconds"]), file=sys.stderr, flush=True)
            if st["seconds"] >= 0.6 * target_seconds or n >= (1 << 27):
                break
            n = int(min(1 << 27, n * max(2.0, 1.2 * target_seconds / max(st["seconds"], 1e-3))))
            n = (n // 4096) * 4096
        return {"value": round(n / st["seconds"] / 1e6, 4), "unit": "Msamples/s", "cores": threads,
                "host_cpus": machine, "cores_note": "threads = the CPUs this process may use (affinity set, "
                "cgroup CPU quota); host_cpus = os.cpu_count() of the machine", "kind": "port",
                "sample": "lanes [0, %d) of pass 0 of the same workload (%.1f s); CPU restatement of mvpath "
                          "(oracle/, %s), not Dr.Jit llvm_rgb" % (
                              n, st["seconds"], "its median-split BVH over %d primitives (oracle_set_bvh)" % n_prims
                              if bvh else "brute-force intersection over %d primitives" % n_prims)}
    except Exception as e:  # the baseline is reported, never the product path
        return {"value": None, "unit": "Msamples/s", "cores": threads, "kind": "port", "sample": "failed: %s" % e}
    finally:
        O.set_bvh(False)


if __name__ == "__main__":
    main()
