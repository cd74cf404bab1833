"""Multi-GPU partitioning of the mvpath hot path (one process per GPU).

The path has no exchange step inside a frame: every lane (pixel sample) is
independent and seeds its own sampler from its global lane index
(TEA(seed_value, lane), mvpath.cpp:227-235), so a frame shards without any
data-path collective.  The only collective is the final sum of the RGBW
ImageBlocks (an RCCL reduce of the film, ImageBlock::put is additive).

Three partitions are provided:
  * view_groups -- C5's "4 views per GPU" (SURVEY 8(e)): rank r owns whole view groups
    (mvpath_multi.h:31-38: a lane's reprojections stay inside its primary view's group), i.e. a
    rectangle of quilt tiles; it renders the lanes of those pixels (amvpt_lane_set rect form) into a
    film window of its tiles plus a 4-pixel filter border, and the frame is assembled on rank 0 by a
    gather of the windows (borders summed) plus the few cells that fall outside (the overflow list).
    The adaptive fill exchanges one count per pixel row of the rectangle (run_exchange).
  * pass_shard  -- weak scaling (bench.py): rank r renders the passes
    [r * P, (r + 1) * P) of a (world * spp)-spp frame by offsetting the seed by
    spp_per_pass * P * r -- exactly the seeds those passes get in a single
    (world * spp)-spp render (seed_value = spp_per_pass * pass + seed).
  * lane_shard  -- strong scaling: rank r renders lanes [begin, end) of every
    pass of the same frame (amvpt_render's lane_begin/lane_end).  With
    adaptive > 0 the fill needs one tiny exchange per pass (count_exchange).
    balanced_shards moves the boundaries to equal measured cost (bands of quilt
    rows differ in path length: 0.92 -> ~0.99 balance at 8 ranks on config M).
"""


def comm_device(device=None):
    """The device collectives run on: `device` under RCCL ("nccl"), the CPU under gloo.  gloo moves host
    buffers only, so a gloo process group over GPU renders (several ranks rehearsing the multi-GPU path on
    one device: bench.py's AMVPT_DIST_BACKEND=gloo) stages every collective's tensors through the host."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
        return "cpu"
    return device


def pass_shard(params, rank, world, plan):
    """Params for `rank`'s share of a world * spp frame. `plan` = amvpt.plan(params)."""
    spp, spp_pp, n_passes, _ = plan
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    p = type(params).from_buffer_copy(params)
    p.seed = params.seed + spp_pp * n_passes * rank
    return p


def lane_shard(n_lanes, rank, world):
    """[begin, end) lanes of `rank` (contiguous, sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    q, r = divmod(n_lanes, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def balanced_shards(bounds, shard_ms, align=4096):
    """Contiguous lane ranges of (about) equal cost, from one measurement of the current ones.

    `bounds` are the world + 1 boundaries of the ranges the ranks rendered (lane_shard's, at
    first) and `shard_ms` their measured times.  The cost density is taken as uniform inside each
    measured range (piecewise-linear cumulative cost) and the new boundaries cut it into equal
    parts, aligned to `align` lanes (whole pixels, whole 16-lane splat rows).  Ranges stay
    ordered by rank, so the adaptive fill's count exchange keeps its prefix order.  Returns the
    new world + 1 boundaries."""
    world = len(shard_ms)
    if len(bounds) != world + 1 or world < 1:
        raise ValueError("need world + 1 bounds for world shard times")
    cum = [0.0]
    for t in shard_ms:
        cum.append(cum[-1] + max(float(t), 1e-9))
    total = cum[-1]
    out = [bounds[0]]
    j = 0
    for r in range(1, world):
        target = total * r / world
        while cum[j + 1] < target:
            j += 1
        frac = (target - cum[j]) / (cum[j + 1] - cum[j])
        x = bounds[j] + frac * (bounds[j + 1] - bounds[j])
        x = int(round(x / align)) * align
        out.append(min(max(x, out[-1]), bounds[-1]))
    out.append(bounds[-1])
    return out


def count_exchange(device=None):
    """`fn(local) -> (prefix, total)` over torch.distributed (one all-gather of one
    integer per rank and pass): the adaptive fill's index space is the whole pass's
    compressed lane array (mvpath_multi.h:81-90), so a lane-sharded rank needs the
    number of flagged lanes in the ranges of lower ranks (lane_shard orders ranges
    by rank) and in the whole pass.  Install it with amvpt.set_adaptive_exchange."""
    import torch
    import torch.distributed as dist

    def fn(local):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return 0, local
        t = torch.tensor([local], dtype=torch.int64, device=comm_device(device))
        out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        counts = [int(o.item()) for o in out]
        return sum(counts[:dist.get_rank()]), sum(counts)
    return fn


def reduce_film(film, dst=0):
    """Sum the ranks' RGBW ImageBlocks on `dst` (RCCL over xGMI on GPUs, gloo on CPU; a GPU film under
    gloo goes through the host, comm_device)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if film.is_cuda and comm_device(film.device) == "cpu":
            t = film.cpu()
            dist.reduce(t, dst=dst)
            if dist.get_rank() == dst:
                film.copy_(t)
        else:
            dist.reduce(film, dst=dst)
    return film


# ---------------------------------------------------------------------------------------------------
# View-group partition (C5)
# ---------------------------------------------------------------------------------------------------

FILTER_BORDER = 4   # the smallest border: the default Gaussian (radius 2) with a cell to spare


def filter_border(params):
    """Pixels around a rank's tiles its splats can reach (host/multi.cpp filter_border): ImageBlock::put's
    footprint reaches ceil(radius - 1/2) cells coalesced, ceil(radius + 1/2) not coalesced, radius = 4
    stddev (gaussian.cpp:48-60); the box filter stays in its pixel.  At least FILTER_BORDER."""
    import math
    import numpy as np
    if params.rfilter == 0:   # AMVPT_RFILTER_BOX
        return FILTER_BORDER
    stddev = params.rfilter_stddev if params.rfilter_stddev > 0 else 0.5
    radius = float(np.float32(4.0) * np.float32(stddev))
    return max(FILTER_BORDER, int(math.ceil(np.float32(radius) + np.float32(0.5))))


def view_tile(params, v):
    """Quilt tile (tx, ty) of view v: the inverse of GridSensor::sample_ray_idx's index
    (grid.cpp:269-297; batch.cpp:163-181 is the grid_y = 1 case) -- the splat's tile offset."""
    gx = max(1, params.grid_x)
    gy = max(1, params.grid_y)
    ix, iy = v % gx, v // gx
    if params.reverse_x:
        ix = gx - 1 - ix
    if params.reverse_y:
        iy = gy - 1 - iy
    return ix, iy


def tiles_rect(params, views):
    """Pixel rectangle (x0, y0, w, h) of the quilt tiles of `views`, or None when they do not form one."""
    gx, gy = max(1, params.grid_x), max(1, params.grid_y)
    sx, sy = params.film_width // gx, params.film_height // gy
    tiles = {view_tile(params, v) for v in views}
    xs = sorted({t[0] for t in tiles})
    ys = sorted({t[1] for t in tiles})
    if len(tiles) != len(xs) * len(ys) or xs != list(range(xs[0], xs[-1] + 1)) or ys != list(range(ys[0], ys[-1] + 1)):
        return None
    return xs[0] * sx, ys[0] * sy, len(xs) * sx, len(ys) * sy


def view_group_partition(params, group, world):
    """Per rank: (lane rectangle, film window) of the view-group partition, or None when it does not
    apply (fewer groups than ranks, groups not divisible among ranks, a grid without separate tiles,
    or tiles that do not form rectangles).  Rank r owns groups [r * n / world, (r + 1) * n / world)."""
    if not params.multisensor or group < 1 or params.n_views % group:
        return None
    n_groups = params.n_views // group
    if world < 1 or n_groups < world or n_groups % world:
        return None
    per = n_groups // world
    out = []
    for r in range(world):
        rect = tiles_rect(params, range(r * per * group, (r + 1) * per * group))
        if rect is None:
            return None
        x0, y0, w, h = rect
        b = filter_border(params)
        wx0, wy0 = max(0, x0 - b), max(0, y0 - b)
        wx1 = min(params.film_width, x0 + w + b)
        wy1 = min(params.film_height, y0 + h + b)
        out.append((rect, (wx0, wy0, wx1 - wx0, wy1 - wy0)))
    return out


def exclusive_prefix(all_begins, all_counts, begins):
    """Flagged lanes below each run in `begins`, given every rank's runs (all_begins, all_counts)."""
    import numpy as np
    b = np.asarray(all_begins, dtype=np.int64)
    c = np.asarray(all_counts, dtype=np.int64)
    order = np.argsort(b, kind="stable")
    b, c = b[order], c[order]
    csum = np.concatenate([[0], np.cumsum(c)])
    idx = np.searchsorted(b, np.asarray(begins, dtype=np.int64), side="left")
    return [int(csum[i]) for i in idx], int(csum[-1])


def run_exchange(device=None):
    """`fn(run_lane_begin, run_count) -> (run_prefix, total)` over torch.distributed: the adaptive fill's
    count exchange for any lane set (amvpt_run_exchange_fn, include/amvpt.h).  One all-gather of the
    run counts and one of the padded (lane begin, count) pairs per pass; runs of different ranks are
    disjoint, so each run's prefix is the count of every run (any rank) that starts below it."""
    import torch
    import torch.distributed as dist

    def fn(begins, counts):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return exclusive_prefix(begins, counts, begins)
        world = dist.get_world_size()
        dev = comm_device(device)
        n = torch.tensor([len(begins)], dtype=torch.int64, device=dev)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n)
        m = max(1, max(int(x.item()) for x in ns))
        buf = torch.zeros((m, 2), dtype=torch.int64)
        buf[:, 0] = 2 ** 62
        if begins:
            buf[:len(begins), 0] = torch.tensor(begins, dtype=torch.int64)
            buf[:len(begins), 1] = torch.tensor(counts, dtype=torch.int64)
        buf = buf.to(dev) if dev else buf
        outs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf)
        allr = torch.cat(outs).cpu().numpy()
        return exclusive_prefix(allr[:, 0], allr[:, 1], begins)
    return fn


def overflow_entries(overflow):
    """(quilt float indices int64, values float32) of an overflow list (int32 tensor: 4 header words,
    then 4 words per entry), as torch tensors on the list's device."""
    import torch
    cnt = int(overflow[:2].view(torch.int64)[0].item())
    cap = overflow.numel() // 4 - 1
    if cnt > cap:
        raise RuntimeError("film overflow list full: %d > %d" % (cnt, cap))
    e = overflow[4:4 + 4 * cnt].view(cnt, 4)
    idx = (e[:, 0].to(torch.int64) & 0xffffffff) | (e[:, 1].to(torch.int64) << 32)
    return idx, e[:, 2].contiguous().view(torch.float32)


def gather_windows(window_film, window, overflow, quilt, windows, dst=0):
    """Assemble the whole-quilt ImageBlock on `dst` from every rank's film window (their borders
    overlap: summed) and overflow list (summed into their floats).  `windows` lists every rank's
    (x0, y0, w, h); `quilt` (H, W, C) is written on dst only (zeroed first).  Point-to-point
    sends to dst (RCCL over xGMI on GPUs, gloo on CPU); a single process just adds its own."""
    import torch
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    rank = dist.get_rank() if multi else 0
    world = dist.get_world_size() if multi else 1
    idx, val = overflow_entries(overflow)
    dev = comm_device(window_film.device) if multi else window_film.device   # gloo: through the host
    if multi:
        n = torch.tensor([idx.numel()], dtype=torch.int64, device=dev)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n)
        counts = [int(x.item()) for x in ns]
    else:
        counts = [idx.numel()]
    if rank != dst:
        ops = [dist.P2POp(dist.isend, window_film.contiguous().to(dev), dst)]
        if counts[rank]:
            ops.append(dist.P2POp(dist.isend, idx.contiguous().to(dev), dst))
            ops.append(dist.P2POp(dist.isend, val.contiguous().to(dev), dst))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return None
    C = quilt.shape[2]
    quilt.zero_()
    recv = {}
    ops = []
    for r in range(world):
        if r == rank:
            continue
        x0, y0, w, h = windows[r]
        t = torch.empty((h, w, C), dtype=quilt.dtype, device=dev)
        recv[r] = [t]
        ops.append(dist.P2POp(dist.irecv, t, r))
        if counts[r]:
            ti = torch.empty(counts[r], dtype=torch.int64, device=dev)
            tv = torch.empty(counts[r], dtype=torch.float32, device=dev)
            recv[r] += [ti, tv]
            ops += [dist.P2POp(dist.irecv, ti, r), dist.P2POp(dist.irecv, tv, r)]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    flat = quilt.view(-1)
    for r in range(world):
        x0, y0, w, h = windows[r]
        if r == rank:
            quilt[y0:y0 + h, x0:x0 + w] += window_film
            if idx.numel():
                flat.index_add_(0, idx.to(quilt.device), val.to(quilt.device))
        else:
            quilt[y0:y0 + h, x0:x0 + w] += recv[r][0].to(quilt.device)
            if counts[r]:
                flat.index_add_(0, recv[r][1].to(quilt.device), recv[r][2].to(quilt.device))
    return quilt
