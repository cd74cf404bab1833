"""A/B the BVH build shape (amvpt_set_bvh_build) on a scene: per-kernel HIP-event ms.

python tools/bvh_sweep.py [--scene cbox_grid.xml] [--res 512] [--spp 64]
"""
import argparse
import itertools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mitsuba3-amvpt_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cbox_grid.xml")
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--leaf", default="2,4,8,15")
    ap.add_argument("--cost", default="0,1,4")
    ap.add_argument("--traversal", default="0")
    args = ap.parse_args()
    import torch
    import amvpt
    kw = dict(res=args.res, spp=args.spp)
    if args.scene == "cbox_grid.xml":
        kw.update(gx=4, gy=2, reuse=8)
    s = amvpt.load_file(os.path.join(REPO, "scenes", args.scene), **kw)
    sd, vd, p = s.describe(0, 0, 0)
    film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
    for leaf, cost, trav in itertools.product([int(x) for x in args.leaf.split(",")],
                                              [float(x) for x in args.cost.split(",")],
                                              [int(x) for x in args.traversal.split(",")]):
        amvpt.set_bvh_build(leaf, cost)
        amvpt.set_traversal(trav)
        dev = amvpt.DeviceScene(sd)
        nodes, prims = dev.stats()
        best = None
        for _ in range(3):
            c = amvpt.Counters()
            film.zero_()
            dev.render(vd, p, film.data_ptr(), counters=c)
            torch.cuda.synchronize()
            d = c.as_dict()
            if best is None or d["total_ms"] < best["total_ms"]:
                best = d
        print(json.dumps({"leaf": leaf, "cost": cost, "traversal": trav, "nodes": nodes,
                          "primary": round(best["kernel_ms_primary"], 2), "bounce": round(best["kernel_ms_bounce"], 2),
                          "splat": round(best["kernel_ms_splat"], 2), "total": round(best["total_ms"], 2)}), flush=True)
        del dev
    amvpt.set_bvh_build(4, 0.0)
    amvpt.set_traversal(0)


if __name__ == "__main__":
    main()
