"""Multi-GPU partitioning of the mvpath hot path (one process per GPU).

The path has no exchange step inside a frame: every lane (pixel sample) is
independent and seeds its own sampler from its global lane index
(TEA(seed_value, lane), mvpath.cpp:227-235), so a frame shards without any
data-path collective.  The only collective is the final sum of the RGBW
ImageBlocks (an RCCL reduce of the film, ImageBlock::put is additive).

Two partitions are provided:
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
        t = torch.tensor([local], dtype=torch.int64, device=device)
        out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        counts = [int(o.item()) for o in out]
        return sum(counts[:dist.get_rank()]), sum(counts)
    return fn


def reduce_film(film, dst=0):
    """Sum the ranks' RGBW ImageBlocks on `dst` (RCCL over xGMI on GPUs, gloo on CPU)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(film, dst=dst)
    return film
