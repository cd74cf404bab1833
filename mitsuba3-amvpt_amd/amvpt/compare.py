"""Image comparison for the parity / convergence gates.

Mirrors the reference's `cmp.py` comparison but on LINEAR RGB (no sqrt tonemap),
which is what the metric's "per-pixel RMSE < 1e-3" gate is stated on:

    python -m amvpt.compare a.exr b.exr [--width W --height H --channels 3]

  rmse    sqrt(mean((a - b)^2)) over all pixels and channels
  psnr    10 log10(peak^2 / mse), peak = max(b) (the reference image)
  relmse  mean((a - b)^2 / (b^2 + 1e-2))  (relative MSE, robust to HDR highlights)
  max_abs max |a - b|
"""
import argparse
import json
import math
import struct

import numpy as np


def metrics(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        raise ValueError("shape mismatch %s vs %s" % (a.shape, b.shape))
    d = a - b
    mse = float(np.mean(d * d))
    peak = float(np.max(b)) if b.size else 0.0
    return {
        "rmse": math.sqrt(mse),
        "psnr": (10.0 * math.log10(peak * peak / mse)) if mse > 0 and peak > 0 else float("inf"),
        "relmse": float(np.mean(d * d / (b * b + 1e-2))),
        "max_abs": float(np.max(np.abs(d))) if d.size else 0.0,
        "nan_mismatch": int(np.sum(np.isnan(a) != np.isnan(b))),
    }


def exr_size(path):
    """(width, height, channels) of an uncompressed scanline EXR written by amvpt.write_exr."""
    with open(path, "rb") as f:
        data = f.read(1 << 16)
    if data[:4] != b"\x76\x2f\x31\x01":
        raise ValueError("%s: not an OpenEXR file" % path)
    p, chans, win = 8, 0, None
    while data[p] != 0:
        name_end = data.index(b"\0", p)
        name = data[p:name_end].decode()
        type_end = data.index(b"\0", name_end + 1)
        size = struct.unpack("<i", data[type_end + 1:type_end + 5])[0]
        val = data[type_end + 5:type_end + 5 + size]
        if name == "channels":
            q = 0
            while val[q] != 0:
                q = val.index(b"\0", q) + 1 + 16
                chans += 1
        elif name == "dataWindow":
            win = struct.unpack("<4i", val)
        p = type_end + 5 + size
    return win[2] - win[0] + 1, win[3] - win[1] + 1, chans


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("a")
    ap.add_argument("b", help="reference image")
    ap.add_argument("--tolerance", type=float, default=None, help="exit 1 if rmse > tolerance")
    args = ap.parse_args(argv)
    import amvpt
    wa, ha, ca = exr_size(args.a)
    wb, hb, cb = exr_size(args.b)
    if (wa, ha, ca) != (wb, hb, cb):
        raise SystemExit("size mismatch: %s vs %s" % ((wa, ha, ca), (wb, hb, cb)))
    m = metrics(amvpt.read_exr(args.a, wa, ha, ca), amvpt.read_exr(args.b, wb, hb, cb))
    print(json.dumps(m))
    if args.tolerance is not None and not m["rmse"] <= args.tolerance:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
