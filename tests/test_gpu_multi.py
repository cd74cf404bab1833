"""The C++ host's multi-GPU entry (amvpt_host_render_multi: one thread per device, lane shards,
ncclReduce of the RGBW ImageBlocks, develop on devices[0]) on the GPUs this box has.  With one
device the reduce is RCCL's single-rank path and the result must equal amvpt_host_render up to the
film's float-atomic summation order (relative 1e-5 of the film scale);
the partition itself is checked against amvpt.dist on CPU (test_multirank.py)."""
import os

import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene,defines", [
    ("cbox_grid.xml", dict(res=32, spp=32, gx=4, gy=2, reuse=8)),
    ("cbox_grid.xml", dict(res=32, spp=16, reuse=4, adaptive=3)),
    ("cbox_env.xml", dict(res=32, spp=16, reuse=4, lw=3)),
], ids=["g8", "g4_adaptive", "env_weighted"])
def test_render_multi_single_device_equals_render(gpu_ready, amvpt_mod, scene, defines):
    s = amvpt_mod.load_file(os.path.join(SCENES, scene), **defines)
    c1, c2 = amvpt_mod.Counters(), amvpt_mod.Counters()
    ref = amvpt_mod.render(s, raw=True, counters=c1)
    out = amvpt_mod.render_multi(s, [0], raw=True, counters=c2)
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()
    assert c1.lanes == c2.lanes and c1.vertices == c2.vertices and c1.view_splats == c2.view_splats
    dev, img = amvpt_mod.render_multi(s, [0]), amvpt_mod.render(s)
    assert np.abs(dev - img).max() <= 1e-4 * max(1.0, np.abs(img).max())


def test_render_multi_caches_scene_and_communicators(gpu_ready, amvpt_mod):
    """the second frame through render_multi reuses the cached per-device scene copy,
    stream, films and communicators (no scene upload / BVH build, no communicator init)."""
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=32, spp=16, reuse=4, adaptive=2)
    a = amvpt_mod.render_multi(s, [0], raw=True)
    st1 = amvpt_mod.multi_stats(s)
    b = amvpt_mod.render_multi(s, [0], raw=True)
    st2 = amvpt_mod.multi_stats(s)
    assert st1["scene_creates"] == 1 and st1["renders"] == 1
    assert st2["scene_creates"] == st1["scene_creates"] and st2["comm_inits"] == st1["comm_inits"]
    assert st2["renders"] == 2
    assert np.abs(a - b).max() <= 1e-5 * np.abs(a).max()
    if amvpt_mod.device_count() >= 2:
        # two devices: lane bands (one group of 4 views) through the ncclReduce, cached likewise
        c = amvpt_mod.render_multi(s, [0, 1], raw=True)
        d = amvpt_mod.render_multi(s, [0, 1], raw=True)
        st3 = amvpt_mod.multi_stats(s)
        assert st3["comm_inits"] == 1 and st3["scene_creates"] == 2
        assert np.abs(c - a).max() <= 1e-5 * np.abs(a).max() and np.abs(d - a).max() <= 1e-5 * np.abs(a).max()


def test_render_multi_view_groups_on_two_devices(gpu_ready, amvpt_mod):
    """the multi-device path itself (view-group windows sent to devices[0] and accumulated, the
    in-process per-run count exchange) against render(); needs two visible GPUs."""
    if amvpt_mod.device_count() < 2:
        pytest.skip("one GPU visible: the two-device exchange and gather need two")
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=32, spp=16, gx=8, gy=4, reuse=4, adaptive=3)
    ref = amvpt_mod.render(s, raw=True)
    out = amvpt_mod.render_multi(s, [0, 1], raw=True)
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()


def test_concurrent_renders_with_different_exchanges(gpu_ready, amvpt_mod):
    """two host threads render different lane sets on one device at once, each with its
    own adaptive count exchange (per-call amvpt_render_opts, no process-global callback); each film equals
    the same render done alone."""
    import threading
    import torch
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=32, spp=32, reuse=4, adaptive=2)
    sd, vd, p = s.describe(0, 0, 0)
    lanes = amvpt_mod.plan(p)[3]
    halves = [(0, lanes // 2), (lanes // 2, lanes)]
    dev = amvpt_mod.DeviceScene(sd)
    # each half's flagged-lane counts per pass, learned from a render that reports them
    counts = []
    for b, e in halves:
        got = []
        film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
        dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt_mod.LaneSet(b, e, 0, 0, 0, 0),
                      exchange=lambda bb, cc, got=got: (got.append(cc[0] if cc else 0), ([0] * len(cc), sum(cc)))[1])
        torch.cuda.synchronize()
        counts.append(got)

    def exchange_for(r):
        it = iter(range(len(counts[0])))

        def fn(bb, cc):
            k = next(it)
            return [sum(c[k] for c in counts[:r])] * len(cc), sum(c[k] for c in counts)
        return fn

    def render(r, out):
        film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt_mod.LaneSet(*halves[r], 0, 0, 0, 0),
                          stream=st.cuda_stream, exchange=exchange_for(r))
        st.synchronize()
        out[r] = film.cpu().numpy()

    alone = {}
    for r in (0, 1):
        render(r, alone)
    together = {}
    th = [threading.Thread(target=render, args=(r, together)) for r in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ref = amvpt_mod.render(s, raw=True)
    for r in (0, 1):
        assert np.abs(together[r] - alone[r]).max() <= 1e-5 * np.abs(ref).max()
    assert np.abs(together[0] + together[1] - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.parametrize("defines", [
    dict(res=32, spp=32, gx=4, gy=2, reuse=8),     # one group of 8 views: lane bands
    dict(res=32, spp=16, gx=8, gy=4, reuse=4),     # eight groups of 4: view groups, windows + overflow cells
], ids=["lane_bands", "view_groups"])
def test_render_multi_shared_device_rehearsal(gpu_ready, amvpt_mod, defines):
    """VERDICT r05 "multi-device execution has never happened": a device list naming the box's one GPU several times
    runs amvpt_host_render_multi's partitions for real -- a thread, scene copy, stream and film per rank, lane bands or
    view-group windows with their overflow cells, the sum onto devices[0] (amvpt_film_accumulate standing in for RCCL)
    -- and must equal render() up to the film's float-atomic summation order, with the same lane counts."""
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), **defines)
    c1 = amvpt_mod.Counters()
    ref = amvpt_mod.render(s, raw=True, counters=c1)
    for devs in ([0, 0], [0, 0, 0, 0]):
        c2 = amvpt_mod.Counters()
        out = amvpt_mod.render_multi(s, devs, raw=True, counters=c2)
        assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max(), devs
        assert c1.lanes == c2.lanes and c1.view_splats == c2.view_splats and c1.vertices == c2.vertices, devs
    img, dev = amvpt_mod.render(s), amvpt_mod.render_multi(s, [0, 0])
    assert np.abs(dev - img).max() <= 1e-4 * max(1.0, np.abs(img).max())


def test_render_multi_shared_device_refuses_the_adaptive_exchange(gpu_ready, amvpt_mod):
    """The adaptive fill's count exchange needs every rank's render in flight at once, which one device's lane arena
    does not allow: the rehearsal refuses it with a message instead of blocking."""
    s = amvpt_mod.load_file(os.path.join(SCENES, "cbox_grid.xml"), res=32, spp=16, reuse=4, adaptive=2)
    with pytest.raises(Exception, match="shared-device rehearsal"):
        amvpt_mod.render_multi(s, [0, 0], raw=True)
