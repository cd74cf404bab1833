"""Loops of one kernel's assembly (backward branches) and the spill / hazard instructions inside each:
    python tools/isa_loops.py <kernel.s>   (one function's lines, e.g. cut from a hipcc -S dump)"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
labels = {}
for n, l in enumerate(lines):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = n
loops = []
for n, l in enumerate(lines):
    m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < n:
        loops.append((labels[m.group(2)], n))
for a, b in sorted(loops):
    body = [x.strip().split()[0] for x in lines[a:b + 1] if x.startswith("\t") and not x.strip().startswith((".", ";"))]
    cnt = lambda p: sum(1 for x in body if x.startswith(p))
    print("lines %5d-%5d  instrs %5d  readlane %3d  writelane %3d  s_nop %3d  scratch %3d  v_div_scale %3d" % (
        a, b, len(body), cnt("v_readlane"), cnt("v_writelane"), cnt("s_nop"), cnt("scratch_"), cnt("v_div_scale")))
