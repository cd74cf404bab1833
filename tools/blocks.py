"""Per-basic-block instruction counts of one kernel in an AMDGPU .s file, with loop nesting (the
compiler's "Loop Header: Depth=N" / "in Loop: Header=BBx Depth=N" comments): a static attribution of a
kernel's VALU work to its loops.
    python tools/blocks.py <file.s> <kernel-substring>"""
import re
import sys

path, want = sys.argv[1], sys.argv[2]
inkern = False
blocks = []   # (label, depth, header, counts)
cur = None
for ln in open(path):
    if re.match(r"^_Z\S*:", ln):
        if inkern:
            break
        inkern = want in ln
        if inkern:
            cur = ["entry", 0, "", {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0, "other": 0}]
            blocks.append(cur)
        continue
    if not inkern:
        continue
    m = re.match(r"^(\.LBB\S+|; %bb\.\d+):?\s*(;.*)?$", ln)
    if m:
        c = ln
        d = re.search(r"Depth=(\d+)", c)
        h = re.search(r"Header=(\S+)", c)
        lab = m.group(1)
        hdr = lab if "Loop Header" in c else (h.group(1) if h else "")
        cur = [lab, int(d.group(1)) if d else 0, hdr, {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0, "other": 0}]
        blocks.append(cur)
        continue
    t = ln.strip()
    if t.startswith(";") and ("Loop" in t) and cur is not None and sum(cur[3].values()) == 0:
        d = re.search(r"Depth=(\d+)", t)
        h = re.search(r"Header=(\S+)", t)
        cur[1] = int(d.group(1)) if d else cur[1]
        cur[2] = cur[0] if "Loop Header" in t else (h.group(1) if h else cur[2])
        continue
    if not t or t.startswith((";", ".")):
        continue
    op = t.split()[0]
    k = ("valu" if op.startswith("v_") else "smem" if op.startswith("s_load") or op.startswith("s_buffer") else
         "salu" if op.startswith("s_") else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else
         "lds" if op.startswith("ds_") else "other")
    cur[3][k] += 1
tot = {}
for lab, d, h, c in blocks:
    key = (d, h)
    t = tot.setdefault(key, {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0, "blocks": 0})
    for k in ("valu", "salu", "smem", "vmem", "lds"):
        t[k] += c[k]
    t["blocks"] += 1
print("depth header              blocks   valu   salu   smem   vmem    lds")
for (d, h), t in sorted(tot.items(), key=lambda x: (x[0][0], x[0][1])):
    print("%5d %-20s %6d %6d %6d %6d %6d %6d" % (d, h or "-", t["blocks"], t["valu"], t["salu"], t["smem"], t["vmem"], t["lds"]))
