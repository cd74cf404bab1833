"""Per-kernel time per frame from a rocprofv3 --stats kernel_stats.csv.

    python tools/kstats.py <run_kernel_stats.csv> [frames]
"""
import csv
import sys

frames = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "")
    print("%-44s %6s calls  %8.1f ms/frame  avg %9.1f us" % (
        n[:44], r["Calls"], float(r["TotalDurationNs"]) / 1e6 / frames, float(r["AverageNs"]) / 1e3))
