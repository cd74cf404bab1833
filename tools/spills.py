"""Spill / reload sites of one kernel in an AMDGPU .s file, by the loop depth of their basic block
(depth >= 1: every iteration of the kernel's loop pays them).
    python tools/spills.py /tmp/kprobe.s [kernel-substring]"""
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
depth, inkern, blk = 0, False, "?"
rows = []
for ln in open(path):
    m = re.match(r"^(\S+):\s*(;.*)?$", ln)
    if re.match(r"^_Z\S*:", ln):
        inkern = want in ln
        continue
    if m or ln.startswith("; %bb"):
        d = re.search(r"Depth=(\d+)", ln)
        depth = int(d.group(1)) if d else 0
        blk = (m.group(1) if m else ln.split()[1])
        continue
    if inkern and "scratch_" in ln:
        kind = "store" if "store" in ln else "load"
        w = re.search(r"dword(x\d)?", ln).group(0)
        n = int(w[-1]) if w[-1].isdigit() else 1
        rows.append((depth, kind, n, blk))
tot = {}
for d, k, n, b in rows:
    tot[(d, k)] = tot.get((d, k), 0) + n
for (d, k), n in sorted(tot.items()):
    print("depth %d %-5s %3d dwords" % (d, k, n))
