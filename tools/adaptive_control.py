"""Control experiment for the C5-shape energy shift.

The unbiasedness gate's c5_adaptive case (8 x 4 grid of 64^2 views, groups of 4, adaptive 3, 16 spp) read
its per-view means 0.12 % low on average against the reuse-off render.  This runs the same shape with the
fill off and on, at 16 and 64 spp, at 64^2 and 128^2 per view, with the Gaussian and the box filter, each
against a reuse-off reference of 512 spp, K seeds per variant, and prints the POOLED energy ratio (mean
over every view's interior pixels, frames as the independent units) with its standard error, the per-group
means and their signs.

  python tools/adaptive_control.py [--k 64] [--out gpurun_out/adaptive_control.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mitsuba3-amvpt_amd"))
sys.path.insert(0, REPO)
import amvpt  # noqa: E402

CBOX = os.path.join(REPO, "scenes", "cbox_grid.xml")
BASE = dict(gx=8, gy=4, reuse=4)


def frames(defines, seeds):
    """(developed frames (K, H, W, 3), ratio-of-means frame (1, H, W, 3)): the raw RGBW ImageBlocks are developed
    per frame as hdrfilm does (RGB / W, W = 0 -> 1), and also summed over the K frames before the divide -- a
    self-normalised estimator's ratio bias (E[sum wL / sum w] != E[sum wL] / E[sum w], O(1/n)) is in the first
    and not in the second"""
    s = amvpt.load_file(CBOX, **defines)
    raw = [amvpt.render(s, seed=k, raw=True).astype(np.float64) for k in seeds]
    dev = np.stack([r[..., :3] / np.where(r[..., 3:4] == 0.0, 1.0, r[..., 3:4]) for r in raw])
    tot = np.sum(raw, axis=0)
    rom = tot[..., :3] / np.where(tot[..., 3:4] == 0.0, 1.0, tot[..., 3:4])
    return dev, rom[None]


def tile_means(fr, res, gx, gy):
    """(K, gy, gx) mean over each view tile's interior (>= 2 px from the tile border)"""
    K, H, W, _ = fr.shape
    y, x = np.mgrid[0:H, 0:W]
    inner = ((y % res) >= 2) & ((y % res) < res - 2) & ((x % res) >= 2) & ((x % res) < res - 2)
    out = np.zeros((K, gy, gx))
    for ty in range(gy):
        for tx in range(gx):
            m = np.zeros((H, W), bool)
            m[ty * res:(ty + 1) * res, tx * res:(tx + 1) * res] = True
            out[:, ty, tx] = fr[:, m & inner].mean(axis=(1, 2))
    return out


def group_of_tiles(gx, gy, G):
    """view group of each quilt tile (grid.cpp: reverse_y defaults to true, so tile row ty is view row gy-1-ty)"""
    g = np.zeros((gy, gx), int)
    for ty in range(gy):
        for tx in range(gx):
            g[ty, tx] = ((gy - 1 - ty) * gx + tx) // G
    return g


def compare(test, ref, groups, test_rom=None, ref_rom=None):
    pt, pr = test.mean(axis=(1, 2)), ref.mean(axis=(1, 2))    # pooled per frame
    K1, K2 = len(pt), len(pr)
    r = pt.mean() / pr.mean()
    se = r * np.sqrt(pt.var(ddof=1) / (K1 * pt.mean() ** 2) + pr.var(ddof=1) / (K2 * pr.mean() ** 2))
    gm = []
    for gi in range(groups.max() + 1):
        sel = groups == gi
        gm.append(float(test[:, sel].mean() / ref[:, sel].mean()))
    out = dict(ratio=float(r), se=float(se), z=float((r - 1.0) / se), group_ratios=np.round(gm, 5).tolist(),
               groups_below=int(sum(g < 1.0 for g in gm)), n_groups=len(gm), pooled_frames=pt.tolist())
    if test_rom is not None:
        out["ratio_of_means"] = float(test_rom.mean() / ref_rom.mean())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "adaptive_control.json"))
    a = ap.parse_args()
    K = a.k
    variants = [
        # (name, res, defines relative to BASE)
        ("a0_s16", 64, dict(adaptive=0, spp=16)),
        ("a3_s16", 64, dict(adaptive=3, spp=16)),
        ("a0_s64", 64, dict(adaptive=0, spp=64)),
        ("a3_s64", 64, dict(adaptive=3, spp=64)),
        ("a0_s256", 64, dict(adaptive=0, spp=256)),
        ("g1_s16", 64, dict(reuse=1, spp=16)),            # the reuse-off side itself at 16 spp
        ("a0_s16_box", 64, dict(adaptive=0, spp=16, rfilter="box")),
        ("a3_s16_box", 64, dict(adaptive=3, spp=16, rfilter="box")),
        ("a0_s64_box", 64, dict(adaptive=0, spp=64, rfilter="box")),
        ("g1_s16_box", 64, dict(reuse=1, spp=16, rfilter="box")),
        ("a0_s16_r128", 128, dict(adaptive=0, spp=16)),
        ("a3_s16_r128", 128, dict(adaptive=3, spp=16)),
    ]
    refs = {}
    out = dict(K=K, shape=dict(BASE, scene="cbox_grid.xml"), variants={})
    t0 = time.time()
    groups = group_of_tiles(BASE["gx"], BASE["gy"], BASE["reuse"])
    for name, res, d in variants:
        rf = d.get("rfilter", "gaussian")
        key = (res, rf)
        if key not in refs:
            dd = dict(BASE, res=res, reuse=1, spp=512, rfilter=rf)
            dev, rom = frames(dd, range(1000, 1000 + K))
            refs[key] = (tile_means(dev, res, BASE["gx"], BASE["gy"]), tile_means(rom, res, BASE["gx"], BASE["gy"]))
            print("ref res=%d %s done (%.0f s)" % (res, rf, time.time() - t0), flush=True)
        dd = dict(BASE, res=res)
        dd.update(d)
        dev, rom = frames(dd, range(K))
        c = compare(tile_means(dev, res, BASE["gx"], BASE["gy"]), refs[key][0], groups,
                    tile_means(rom, res, BASE["gx"], BASE["gy"]), refs[key][1])
        c["defines"] = dd
        out["variants"][name] = c
        print("%-12s pooled ratio %.5f +- %.5f (z %+.2f), ratio of means %.5f; groups below 1: %d/%d %s (%.0f s)" % (
            name, c["ratio"], c["se"], c["z"], c["ratio_of_means"], c["groups_below"], c["n_groups"], c["group_ratios"],
            time.time() - t0), flush=True)
    # the fill alone: adaptive 3 against adaptive 0 of the same shape (same reference cancels)
    for a3, a0 in (("a3_s16", "a0_s16"), ("a3_s64", "a0_s64"), ("a3_s16_box", "a0_s16_box"),
                   ("a3_s16_r128", "a0_s16_r128")):
        r3, r0 = out["variants"][a3], out["variants"][a0]
        # paired by seed (the same K seeds: the fill's lanes are the only difference)
        q = np.array(r3["pooled_frames"]) / np.array(r0["pooled_frames"])
        d, se = q.mean(), q.std(ddof=1) / np.sqrt(len(q))
        out.setdefault("fill_vs_nofill", {})[a3] = dict(ratio=float(d), se=float(se), z=float((d - 1) / se))
        print("fill effect %-12s %.5f +- %.5f (z %+.2f)" % (a3, d, se, (d - 1) / se), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
