"""One rank of the multi-rank rehearsal on one device (tests/test_gpu_dist.py): launched by
torch.distributed.run with AMVPT_DIST_BACKEND semantics = gloo, every rank on the same visible device.
It runs bench.py's two partitions of a frame on the HIP path -- lane bands with the adaptive count
exchange + reduce of the ImageBlocks, and view groups with film windows + overflow lists + the gather on
rank 0 -- through amvpt.dist exactly as bench.py calls it, and rank 0 compares each assembled frame with
the single-process render of the same frame (written as JSON to argv[1])."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "mitsuba3-amvpt_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import amvpt
    from amvpt import dist as adist

    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    amvpt.hip_lib().amvpt_set_device(torch.cuda.current_device())
    stream = torch.cuda.current_stream().cuda_stream
    exchange = adist.run_exchange(device="cuda")
    res = {}
    cases = {
        # lane bands (config M's shape, one group of 8 views), with the adaptive fill's count exchange
        "lanes_adaptive": dict(file="cbox_grid.xml", kw=dict(res=64, spp=32, gx=4, gy=2, reuse=8, adaptive=2),
                               part="lanes"),
        # view groups (C5's shape: 8 x 4 grid, groups of 4), windows + overflow, gathered on rank 0
        "groups_adaptive": dict(file="cbox_grid.xml", kw=dict(res=32, spp=16, gx=8, gy=4, reuse=4, adaptive=3),
                                part="groups"),
        # lane bands over the BVH mesh scene (per-lane walks, binning, chunk streams)
        "lanes_mesh": dict(file="cbox_mesh.xml", kw=dict(res=32, spp=16, gx=4, gy=2, reuse=8), part="lanes"),
    }
    for name, c in cases.items():
        s = amvpt.load_file(os.path.join(REPO, "scenes", c["file"]), **c["kw"])
        sd, vd, p = s.describe(0, 0, 0)
        spp, spp_pp, n_passes, lanes_per_pass = amvpt.plan(p)
        G = {1: 1}.get(p.n_views, min(p.reuse_count, p.n_views))
        dev = amvpt.DeviceScene(sd)
        C = 5 if p.film_alpha else 4
        cnt = amvpt.Counters()
        if c["part"] == "groups":
            groups = adist.view_group_partition(p, G, world)
            assert groups is not None, name
            rect, win = groups[rank]
            wx0, wy0, ww, wh = win
            film = torch.zeros((wh, ww, C), dtype=torch.float32, device="cuda")
            ov_cap = 1 << 16
            overflow = torch.zeros(4 * (ov_cap + 1), dtype=torch.int32, device="cuda")
            quilt = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda") if rank == 0 else None
            dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt.LaneSet(0, 0, *rect), window=win,
                          overflow_ptr=overflow.data_ptr(), overflow_capacity=ov_cap, stream=stream, counters=cnt,
                          exchange=exchange)
            torch.cuda.synchronize()
            frame = adist.gather_windows(film, win, overflow, quilt, [g[1] for g in groups], dst=0)
        else:
            b, e = adist.lane_shard(lanes_per_pass, rank, world)
            film = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda")
            dev.render_ex(vd, p, film.data_ptr(), lanes=amvpt.LaneSet(b, e, 0, 0, 0, 0), stream=stream,
                          counters=cnt, exchange=exchange)
            torch.cuda.synchronize()
            frame = adist.reduce_film(film, dst=0)
        lanes = torch.tensor([cnt.lanes, cnt.adaptive_lanes], dtype=torch.int64)
        dist.all_reduce(lanes)
        if rank == 0:
            one = torch.zeros((p.film_height, p.film_width, C), dtype=torch.float32, device="cuda")
            c1 = amvpt.Counters()
            dev.render_ex(vd, p, one.data_ptr(), stream=stream, counters=c1)
            torch.cuda.synchronize()
            g, o = frame.cpu().numpy(), one.cpu().numpy()
            res[name] = {"max_rel": float(np.abs(g - o).max() / max(1e-30, np.abs(o).max())),
                         "lanes": [int(lanes[0]), int(lanes[1])], "lanes_single": [int(c1.lanes), int(c1.adaptive_lanes)],
                         "film_sum": float(o[..., -1].sum()), "world": world}
        del dev
        dist.barrier()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
