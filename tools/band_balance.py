"""Load balance of config M's strong-scaling partition, measured on one GPU.

Renders each of the N lane shards (amvpt.dist.lane_shard, the bands of quilt rows the N
ranks of `bench.py --gpus N` take) on its own and times it; the slowest shard bounds the
N-GPU frame.  Prints one JSON line: per-shard ms, and the strong-scaling efficiency the
partition allows (sum / (N * max)).

    python tools/band_balance.py [--world 8] [--config M]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "mitsuba3-amvpt_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import amvpt
    from amvpt import dist as adist
    s = amvpt.load_file(os.path.join(REPO, "scenes", "cbox_grid.xml"), res=1024, spp=64, gx=4, gy=2, reuse=8)
    sd, vd, p = s.describe(0, 0, 0)
    _, _, _, L = amvpt.plan(p)
    dev = amvpt.DeviceScene(sd)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    def shard_times(bounds, reps):
        ms = []
        for r in range(len(bounds) - 1):
            b, e = bounds[r], bounds[r + 1]
            dev.render(vd, p, film.data_ptr(), b, e, stream)   # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                dev.render(vd, p, film.data_ptr(), b, e, stream)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3 / reps)
        return ms

    for w in sorted({1, 2, 4, args.world}):
        bounds = [adist.lane_shard(L, r, w)[0] for r in range(w)] + [L]
        # equal lane counts, then bench.py's one-measurement rebalance (amvpt.dist.balanced_shards)
        for kind in ("equal", "balanced"):
            if kind == "balanced":
                if w == 1:
                    break
                bounds = adist.balanced_shards(bounds, ms, align=256)
            ms = shard_times(bounds, args.reps)
            print(json.dumps({"world": w, "partition": kind, "shard_ms": [round(x, 2) for x in ms],
                              "max_ms": round(max(ms), 2),
                              "efficiency_bound": round(sum(ms) / (w * max(ms)), 4)}), flush=True)


if __name__ == "__main__":
    main()
