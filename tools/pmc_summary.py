"""Per-kernel totals of every counter in one or more rocprofv3 PMC output dirs.

    python tools/pmc_summary.py <dir> [<dir> ...]
"""
import collections
import csv
import os
import sys


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
            k = r["Kernel_Name"]
            if "amvpt" not in k:
                continue
            k = k.split("(")[0].replace("void ", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for k, c in tot.items():
        print("== %s  (%d launches)" % (k, len(launches[k])))
        waves = c.get("SQ_WAVES", 0.0)
        for n in sorted(c):
            per = "  %.1f /wave" % (c[n] / waves) if waves and n.startswith("SQ_INSTS") else ""
            print("   %-24s %.4e%s" % (n, c[n], per))


if __name__ == "__main__":
    main()
