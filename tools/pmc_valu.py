"""Per-launch VALU issue of each kernel from a rocprofv3 SQ PMC pass (tools/pmc_sq.sh pass A:
SQ_WAVES, SQ_INSTS_VALU, SQ_INSTS_SALU, ...).  bench.py divides the per-launch VALU wave-instructions
by its own live launch time to report the VALU-issue fraction next to the HBM roofline.

    python tools/pmc_valu.py <sqA_dir> <out.json>

Peak VALU issue (MI355X_MICROARCH.md: a wave issues a VALU instruction over 2 cycles, 32 lanes per
cycle): 256 CUs x 4 SIMDs x 2.4 GHz / 2 = 1228.8 G wave-instructions/s.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_revision as revision  # noqa: E402  (the stamp bench.py checks)


def main():
    d, out = sys.argv[1], sys.argv[2]
    config = sys.argv[3] if len(sys.argv) > 3 else "M"
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
        k = r["Kernel_Name"]
        if "amvpt" not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 2   # bench.py --steps 1 --warmup 0: timed + instrumented frame
    res = {"source": d, "config": config, "source_revision": revision(), "peak_valu_ginst_s": 1228.8,
           "frames_profiled": frames, "kernels": {}}
    for k, c in acc.items():
        n = max(1, len(ids[k]))
        res["kernels"][k] = {"launches": n, "waves_per_launch": c["SQ_WAVES"] / n,
                             "valu_insts_per_launch": c["SQ_INSTS_VALU"] / n,
                             "salu_insts_per_launch": c["SQ_INSTS_SALU"] / n,
                             "valu_per_wave": c["SQ_INSTS_VALU"] / max(1.0, c["SQ_WAVES"])}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(res["kernels"].items()):
        print("%-70s %5d launches  %.3e VALU/launch  %7.0f VALU/wave" % (k[:70], v["launches"], v["valu_insts_per_launch"], v["valu_per_wave"]))


if __name__ == "__main__":
    main()
