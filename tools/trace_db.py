"""Per-kernel totals (and the first N dispatches in order) from a rocprofv3 kernel-trace results database.
    python tools/trace_db.py <run_results.db> [substring] [N]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
sub = sys.argv[2] if len(sys.argv) > 2 else ""
nseq = int(sys.argv[3]) if len(sys.argv) > 3 else 0
agg = collections.defaultdict(lambda: [0, 0.0])
seq = []
for name, start, end in db.execute("select name, start, end from kernels"):
    if sub not in name:
        continue
    short = name.split("(")[0].replace("void amvpt::", "")
    d = (end - start) / 1e3
    agg[short][0] += 1
    agg[short][1] += d
    seq.append((start, short, d))
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-60s %5d launches %9.2f ms %9.1f us avg" % (k, n, t / 1e3, t / n))
seq.sort()
for s in seq[:nseq]:
    print("  %-40s %8.1f us" % (s[1][-40:], s[2]))
