"""Control experiment for the cone-layout per-view energy shift (round 6).

The unbiasedness gate's cbox_g8_cone case (grid.cpp cone layout, 12 degrees, 8 views of 128^2, G = 8, 64 spp)
passes the per-pixel Z-test off the geometric edge mask but reads the central views' interior means up to 0.17 %
high against the reuse-off render.  This separates the candidate causes, per view, K seeds per side:
  * the per-view ratio over ALL interior pixels vs over the pixels OFF the edge mask (a footprint straddling a
    discontinuity is a differently weighted average in a self-normalised film -- does the shift live there?);
  * the Gaussian (5 x 5 footprint) vs the box filter (one pixel);
  * the developed mean vs the ratio of means (frames summed before the divide: the O(1/n) ratio bias);
  * the cone layout vs a plain cam_dir line through the same camera positions (no lens shift).

  python tools/cone_control.py [--k 24]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mitsuba3-amvpt_amd"), REPO, os.path.join(REPO, "tests")]
import amvpt  # noqa: E402
import test_gpu_unbiased as U  # noqa: E402

CONE = os.path.join(REPO, "scenes", "cbox_cone.xml")
CBOX = os.path.join(REPO, "scenes", "cbox_grid.xml")


def raw_frames(path, seeds, **d):
    s = amvpt.load_file(path, **d)
    return np.stack([amvpt.render(s, seed=k, raw=True).astype(np.float64) for k in seeds])


def dev(raw):
    return raw[..., :3] / np.where(raw[..., 3:4] == 0.0, 1.0, raw[..., 3:4])


def per_view(fr, mask, res):
    K, H, W, _ = fr.shape
    out = []
    for ty in range(H // res):
        for tx in range(W // res):
            m = np.zeros((H, W), bool)
            m[ty * res:(ty + 1) * res, tx * res:(tx + 1) * res] = True
            out.append(fr[:, m & mask].mean(axis=(1, 2)))
    return np.stack(out, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=24)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "cone_control.json"))
    a = ap.parse_args()
    K, res = a.k, 128
    base = dict(res=res, gx=4, gy=2)
    # the cone's camera x offsets are 3.9 tan((i/7 - 1/2) 12 deg): +-0.4099 at the ends; a cam_dir line of length
    # 0.8198 centred on the grid camera puts the cameras at the same offsets (evenly spaced: the tangents are
    # nearly linear over +-6 degrees), without the shear
    variants = [
        ("cone_gauss_64", CONE, dict(cone=12, spp=64)),
        ("cone_box_64", CONE, dict(cone=12, spp=64, rfilter="box")),
        ("cone_gauss_256", CONE, dict(cone=12, spp=256)),
        ("line_gauss_64", CBOX, dict(spp=64, reuse=8)),
    ]
    out = {"K": K, "variants": {}}
    t0 = time.time()
    for name, path, d in variants:
        dd = dict(base, **d)
        if path == CBOX:
            # cam_dist through a define is not in cbox_grid.xml: patch the XML text
            xml = open(CBOX).read().replace('<float name="cam_dist" value="0.4"/>', '<float name="cam_dist" value="0.8198"/>')
            tmp = os.path.join(REPO, "gpurun_out", "line_cam.xml")
            os.makedirs(os.path.dirname(tmp), exist_ok=True)
            open(tmp, "w").write(xml)
            path = tmp
        G, radius = 8, (1 if d.get("rfilter") == "box" else 2)
        test = raw_frames(path, range(K), **dd)
        ref = raw_frames(path, range(1000, 1000 + K), **dict(dd, reuse=1, spp=512))
        interior = U._interior(test.shape[1:3], res)
        edges = U._edge_mask(amvpt, path, dd, G, radius)
        r = {}
        for mname, mask in (("interior", interior), ("off_mask", interior & ~edges), ("edges", interior & edges)):
            vt, vr = per_view(dev(test), mask, res), per_view(dev(ref), mask, res)
            z = (vt.mean(0) - vr.mean(0)) / np.sqrt(vt.var(0, ddof=1) / K + vr.var(0, ddof=1) / K)
            # ratio of means per view: RGB and W sums over the frames, divided once per pixel, then averaged
            rom_t = per_view(dev(test.sum(0, keepdims=True)), mask, res)[0]
            rom_r = per_view(dev(ref.sum(0, keepdims=True)), mask, res)[0]
            r[mname] = dict(ratio=np.round(vt.mean(0) / vr.mean(0), 5).tolist(), z=np.round(z, 2).tolist(),
                            rom_ratio=np.round(rom_t / rom_r, 5).tolist(), pixels=int(mask.sum()))
            print("%-15s %-9s ratio %s\n%-25s z %s\n%-25s ratio of means %s" % (
                name, mname, r[mname]["ratio"], "", r[mname]["z"], "", r[mname]["rom_ratio"]), flush=True)
        out["variants"][name] = r
        print("(%.0f s)" % (time.time() - t0), flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
