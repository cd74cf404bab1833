"""Static instruction mix of one kernel in an assembly dump (hipcc -S):
    python tools/isa_mix.py <file.s> <mangled-name-substring> [top]"""
import collections
import sys

path, sub = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
body, on = [], False
for line in open(path):
    if not on and line.startswith("_ZN") and sub in line.split(":")[0]:
        on = True
        continue
    if on:
        if line.startswith(".Lfunc_end"):
            break
        t = line.strip()
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            body.append(t.split()[0])
ops = collections.Counter(body)
print("instructions", len(body))
for k, n in ops.most_common(top):
    print("  %-28s %6d" % (k, n))
