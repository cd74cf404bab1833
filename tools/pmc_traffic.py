"""Per-launch HBM traffic of each kernel from two rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json>

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one
TCC pass on gfx950) and are reported by rocprofv3 in KiB.  Corrections per
/opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE
counts a wide coalesced streaming read at half its bytes on gfx950, so it is
doubled; WRITE_SIZE is exact for 16-B/lane stores and f32 atomics.  Our kernels
mix 16-B loads (view/lane records, float4) with narrower ones, so the doubled
figure is an upper bound for the narrow part -- stated in DESIGN.md.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_revision as revision  # noqa: E402  (the stamp bench.py checks)


def per_kernel(d, counter):
    acc = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        a = acc[k]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
    return acc


def main():
    fd, wd, out = sys.argv[1:4]
    config = sys.argv[4] if len(sys.argv) > 4 else "M"
    f = per_kernel(fd, "FETCH_SIZE")
    w = per_kernel(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        if "amvpt" not in k:
            continue
        nf, sf = f.get(k, [0, 0.0])
        nw, sw = w.get(k, [0, 0.0])
        fetch = 2.0 * sf * 1024 / max(nf, 1)
        write = sw * 1024 / max(nw, 1)
        res[k] = {"launches": max(nf, nw), "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                  "hbm_bytes_per_launch": fetch + write}
    # frames the profiled bench rendered: tools/gpu_run.sh runs `bench.py --steps 1 --warmup 0` (the timed frame and
    # the instrumented frame), so the per-frame traffic is the launches' sum / 2 (bench.py frame_pmc)
    frames = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    json.dump({"source": [fd, wd], "config": config, "source_revision": revision(), "frames_profiled": frames,
               "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 wide-read), WRITE_SIZE KiB x1024",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print("%-70s %6d launches  %.3e B/launch (fetch %.3e, write %.3e)" % (
            k[:70], v["launches"], v["hbm_bytes_per_launch"], v["fetch_bytes_per_launch"], v["write_bytes_per_launch"]))


if __name__ == "__main__":
    main()
