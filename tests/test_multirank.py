"""Multi-rank partitioning on CPU (gloo, world_size 2): the shards of
amvpt.dist rendered by the CPU oracle and summed with a collective equal the
single-process frame.  This is the same code path bench.py runs over RCCL
(pass_shard + reduce_film); only the renderer (oracle on CPU instead of the
HIP pipeline) differs."""
import os
import socket
import tempfile

import numpy as np
import pytest

from conftest import PKG, REPO, SCENES

CBOX = os.path.join(SCENES, "cbox_grid.xml")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, mode, out_dir, kw=None):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import amvpt
    from amvpt import dist as adist
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = amvpt.load_file(CBOX, **(kw or dict(res=16, spp=16, gx=2, gy=2, reuse=4)))
        sd, vd, p = s.describe(0, 0, 0)
        plan = amvpt.plan(p)
        if mode == "pass":
            pr = adist.pass_shard(p, rank, world, plan)
            film, _, _ = O.render(sd, vd, pr, threads=2)
        else:
            b, e = adist.lane_shard(plan[3], rank, world)
            O.set_exchange(adist.count_exchange())
            film, _, _ = O.render(sd, vd, p, lane_begin=b, lane_end=e, threads=2)
            O.set_exchange(None)
        t = torch.from_numpy(film)
        adist.reduce_film(t, dst=0)
        if rank == 0:
            np.save(os.path.join(out_dir, "film.npy"), t.numpy())
    finally:
        dist.destroy_process_group()


def _group_worker(rank, world, port, out_dir, kw):
    """One rank of the view-group partition (C5's "4 views per GPU") on the CPU oracle: render the
    lanes of this rank's tile rectangle with the per-run count exchange, cut the film into the rank's
    window + overflow list exactly as amvpt_render_ex hands them over, and gather on rank 0."""
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import amvpt
    from amvpt import dist as adist
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kw = dict(kw)
        xml = kw.pop("xml", None)
        s = amvpt.load_string(xml, **kw) if xml else amvpt.load_file(CBOX, **kw)
        sd, vd, p = s.describe(0, 0, 0)
        G = O.plan(p)["group"]
        part = adist.view_group_partition(p, G, world)
        assert part is not None
        rect, win = part[rank]
        O.set_run_exchange(adist.run_exchange())
        full, st = O.render_rect(sd, vd, p, rect, threads=2)
        O.set_run_exchange(None)
        x0, y0, w, h = win
        window = torch.from_numpy(np.ascontiguousarray(full[y0:y0 + h, x0:x0 + w]))
        outside = full.copy()
        outside[y0:y0 + h, x0:x0 + w] = 0
        flat = outside.reshape(-1)
        nz = np.flatnonzero(flat)
        ov = np.zeros(4 * (len(nz) + 1), dtype=np.int32)
        ov[0:2] = np.array([len(nz)], dtype=np.int64).view(np.int32)
        e = ov[4:].reshape(-1, 4)
        e[:, 0] = (nz & 0xffffffff).astype(np.uint32).view(np.int32)
        e[:, 1] = (nz >> 32).astype(np.int32)
        e[:, 2] = flat[nz].view(np.int32)
        quilt = torch.zeros(full.shape, dtype=torch.float32)
        out = adist.gather_windows(window, win, torch.from_numpy(ov), quilt, [q[1] for q in part], dst=0)
        if rank == 0:
            np.save(os.path.join(out_dir, "film.npy"), out.numpy())
            np.save(os.path.join(out_dir, "lanes.npy"), np.array([st["lanes"], st["adaptive_lanes"]]))
    finally:
        dist.destroy_process_group()


def _run_groups(world, kw):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_group_worker, args=(world, _free_port(), d, kw), nprocs=world, join=True)
        return np.load(os.path.join(d, "film.npy"))


C5_SMALL = dict(res=16, spp=16, gx=8, gy=4, reuse=4, adaptive=3)


@pytest.mark.parametrize("world", [2, 4])
def test_view_group_partition_equals_single_process(oracle, amvpt_mod, world):
    """C5's view-group partition: each rank renders the lanes of its groups' tiles (an
    8 x 4 grid of 16^2 views, groups of 4, adaptive 3, per-row count exchange); the gathered windows +
    overflow cells equal the single-process frame."""
    got = _run_groups(world, C5_SMALL)
    s = amvpt_mod.load_file(CBOX, **C5_SMALL)
    sd, vd, p = s.describe(0, 0, 0)
    ref, _, st = oracle.render(sd, vd, p, threads=4)
    assert st["adaptive_lanes"] > 0
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def _wide_filter_xml(stddev):
    return open(CBOX).read().replace('<rfilter type="$rfilter"/>',
                                     '<rfilter type="gaussian"><float name="stddev" value="%g"/></rfilter>' % stddev)


def test_view_group_partition_with_a_wide_filter(oracle, amvpt_mod):
    """A Gaussian of stddev 1.5 (radius 6) splats up to 7 cells past a rank's tiles: the window border
    follows the filter (a fixed 4-px border sent those cells to the overflow list, past its cap
    at C5 sizes), and the gathered frame still equals the single-process one."""
    from amvpt import dist as adist
    kw = dict(C5_SMALL, adaptive=0, xml=_wide_filter_xml(1.5))
    s = amvpt_mod.load_string(kw["xml"], **{k: v for k, v in kw.items() if k != "xml"})
    sd, vd, p = s.describe(0, 0, 0)
    assert abs(p.rfilter_stddev - 1.5) < 1e-7 and adist.filter_border(p) == 7
    (x0, y0, w, h), (wx, wy, ww, wh) = adist.view_group_partition(p, 4, 2)[1]
    assert x0 - wx in (0, 7) and wy == max(0, y0 - 7)
    got = _run_groups(2, kw)
    ref, _, _ = oracle.render(sd, vd, p, threads=4)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_view_group_partition_geometry(amvpt_mod):
    """Tiles of each rank's groups form rectangles that tile the quilt; M (one group of 8) has none."""
    from amvpt import dist as adist
    s = amvpt_mod.load_file(CBOX, **C5_SMALL)
    _, _, p = s.describe(0, 0, 0)
    for world in (1, 2, 4, 8):
        part = adist.view_group_partition(p, 4, world)
        assert part is not None and len(part) == world
        cover = np.zeros((p.film_height, p.film_width), dtype=np.int32)
        for (x0, y0, w, h), (wx, wy, ww, wh) in part:
            cover[y0:y0 + h, x0:x0 + w] += 1
            assert wx <= x0 and wy <= y0 and wx + ww >= x0 + w and wy + wh >= y0 + h
        assert (cover == 1).all()
    assert adist.view_group_partition(p, 4, 3) is None           # 8 groups over 3 ranks
    m = amvpt_mod.load_file(CBOX, res=16, spp=16, gx=4, gy=2, reuse=8)
    assert adist.view_group_partition(m.describe(0, 0, 0)[2], 8, 2) is None


def test_run_exchange_prefixes():
    """The per-run prefix of the adaptive count exchange: flagged lanes of every run below it."""
    from amvpt import dist as adist
    begins = [0, 100, 200, 300]
    counts = [3, 5, 7, 11]
    pre, tot = adist.exclusive_prefix([300, 0, 200, 100], [11, 3, 7, 5], [100, 300])
    assert pre == [3, 15] and tot == 26
    fn = adist.run_exchange()
    assert fn(begins, counts) == ([0, 3, 8, 15], 26)


def _run(mode, world=2, kw=None):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), mode, d, kw), nprocs=world, join=True)
        return np.load(os.path.join(d, "film.npy"))


def test_lane_sharded_frame_equals_single_process(oracle, amvpt_mod):
    got = _run("lane")
    s = amvpt_mod.load_file(CBOX, res=16, spp=16, gx=2, gy=2, reuse=4)
    sd, vd, p = s.describe(0, 0, 0)
    ref, _, _ = oracle.render(sd, vd, p, threads=4)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_pass_sharded_frame_equals_double_spp_frame(oracle, amvpt_mod):
    """bench.py's weak scaling: 2 ranks x 16 spp == one 32-spp frame (2 passes of 16)."""
    got = _run("pass")
    s = amvpt_mod.load_file(CBOX, res=16, spp=32, gx=2, gy=2, reuse=4)
    sd, vd, p = s.describe(0, 0, 0)
    assert amvpt_mod.plan(p)[2] == 2
    ref, _, _ = oracle.render(sd, vd, p, threads=4)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_adaptive_lane_shards_exchange_counts(oracle, amvpt_mod):
    """C5's partition: adaptive > 0 over lane ranges; the fill learns its prefix and the pass's
    total from one all-gather per pass (amvpt.dist.count_exchange) and the sum is the frame."""
    kw = dict(res=16, spp=32, gx=2, gy=2, reuse=4, adaptive=2)
    got = _run("lane", world=3, kw=kw)
    s = amvpt_mod.load_file(CBOX, **kw)
    sd, vd, p = s.describe(0, 0, 0)
    ref, _, st = oracle.render(sd, vd, p, threads=4)
    assert st["adaptive_lanes"] > 0
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_adaptive_pass_shards(oracle, amvpt_mod):
    """Pass sharding keeps the adaptive fill local: each pass compacts only its own lanes."""
    kw = dict(res=16, spp=16, gx=2, gy=2, reuse=4, adaptive=1)
    got = _run("pass", kw=kw)
    s = amvpt_mod.load_file(CBOX, **dict(kw, spp=32))
    sd, vd, p = s.describe(0, 0, 0)
    ref, _, _ = oracle.render(sd, vd, p, threads=4)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_shard_arithmetic(amvpt_mod):
    from amvpt import dist as adist
    for n in (0, 1, 7, 1000, 2 ** 33 + 3):
        for w in (1, 2, 3, 8):
            spans = [adist.lane_shard(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1
    with pytest.raises(ValueError):
        adist.lane_shard(10, 2, 2)


def test_host_lane_shard_matches_dist(amvpt_mod):
    """The C++ host's multi-GPU partition (amvpt_host_lane_shard, used by amvpt_host_render_multi)
    is the same contiguous lane_shard as the torch.distributed path's (amvpt.dist)."""
    from amvpt import dist
    for lanes in (0, 1, 7, 100, 4096 * 2048 * 16, 2 ** 27 + 13):
        for world in (1, 2, 3, 8):
            shards = [amvpt_mod.host_lane_shard(lanes, r, world) for r in range(world)]
            assert shards == [dist.lane_shard(lanes, r, world) for r in range(world)]
            assert shards[0][0] == 0 and shards[-1][1] == lanes
            assert all(shards[r][1] == shards[r + 1][0] for r in range(world - 1))


def test_balanced_shards_equalise_measured_cost():
    """amvpt.dist.balanced_shards: contiguous, ordered, aligned ranges that split a piecewise-uniform cost
    into equal parts (the bench's one-measurement rebalance of the strong-scaling partition)."""
    from amvpt import dist as adist
    n, world = 1 << 20, 4
    bounds = [adist.lane_shard(n, r, world)[0] for r in range(world)] + [n]
    # shard 3 is twice as expensive per lane as the others
    new = adist.balanced_shards(bounds, [1.0, 1.0, 1.0, 2.0], align=256)
    assert new[0] == 0 and new[-1] == n and all(a <= b for a, b in zip(new, new[1:]))
    assert all(x % 256 == 0 for x in new[1:-1])
    dens = lambda x: 2.0 if x >= bounds[3] else 1.0
    cost = [sum(dens(x) for x in range(a, b, 256)) for a, b in zip(new, new[1:])]
    assert max(cost) / min(cost) < 1.01
    # equal costs keep (aligned) equal ranges; one rank may own an empty range
    assert adist.balanced_shards(bounds, [1.0] * 4, align=256) == bounds
    with pytest.raises(ValueError):
        adist.balanced_shards(bounds, [1.0] * 3)


def test_host_view_group_partition_matches_dist(amvpt_mod):
    """The C++ host's view-group partition (amvpt_host_view_group_partition, used by render_multi) equals
    amvpt.dist.view_group_partition (the bench's), including the configurations where neither applies."""
    from amvpt import dist as adist
    cases = [dict(C5_SMALL), dict(res=16, spp=16, gx=4, gy=2, reuse=4), dict(res=16, spp=16, gx=4, gy=2, reuse=2),
             dict(res=16, spp=16, gx=4, gy=2, reuse=8), dict(res=16, spp=16, gx=3, gy=2, reuse=2),
             dict(C5_SMALL, xml=_wide_filter_xml(1.5)), dict(C5_SMALL, xml=_wide_filter_xml(2.2)),
             dict(C5_SMALL, rfilter="box")]
    for kw in cases:
        xml = kw.pop("xml", None)
        _, _, p = (amvpt_mod.load_string(xml, **kw) if xml else amvpt_mod.load_file(CBOX, **kw)).describe(0, 0, 0)
        from oracle import oracle as O
        G = O.plan(p)["group"]
        for world in (1, 2, 3, 4, 8):
            py = adist.view_group_partition(p, G, world)
            cc = [amvpt_mod.host_view_group_partition(p, r, world) for r in range(world)]
            if py is None:
                assert any(c is None for c in cc), (kw, world)   # render_multi then takes lane bands
            else:
                assert [(tuple(a), tuple(b)) for a, b in py] == cc, (kw, world)


def test_render_multi_fails_fast_on_a_bad_device(amvpt_mod):
    """a device list with an invalid id is an error before any device work starts (no thread
    waits in a collective or an exchange)."""
    s = amvpt_mod.load_file(CBOX, res=16, spp=16)
    with pytest.raises(RuntimeError, match="not visible"):
        amvpt_mod.render_multi(s, [0, 99])


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_render_multi_rank_failures_never_block(amvpt_mod, n):
    """Failure injection into amvpt_host_render_multi's rank coordination (host/ranks.h, on the CPU): one
    rank failing in setup, before / between / after its count exchanges, before the gather or at the end
    makes the call return that rank's own error -- not a peer's "a peer failed" echo -- and no thread stays
    blocked in a barrier or in the exchange (each case runs under a watchdog)."""
    import ctypes
    import threading
    L = amvpt_mod.host_lib()
    L.amvpt_host_test_ranks.argtypes = [ctypes.c_int] * 4
    L.amvpt_host_test_ranks.restype = ctypes.c_int
    msgs = {0: "injected setup failure", 1: "before the exchanges", 2: "between exchanges",
            3: "after the exchanges", 4: "before the gather", 5: "injected finish failure"}

    def run(*args):
        out = {}
        t = threading.Thread(target=lambda: out.update(rc=L.amvpt_host_test_ranks(*args),
                                                       err=L.amvpt_host_last_error().decode()))
        t.start()
        t.join(timeout=30)
        assert not t.is_alive(), "rank coordination blocked: %r" % (args,)
        return out["rc"], out["err"]

    assert run(n, 4, -1, -1)[0] == 0                       # healthy: every exchange prefix checked
    for phase, msg in msgs.items():
        for rank in sorted({0, n // 2, n - 1}):
            rc, err = run(n, 4, rank, phase)
            assert rc == 1 and err.startswith("rank %d: " % rank) and msg in err, (phase, rank, rc, err)
