"""Instruction histogram of one kernel in a hipcc -S listing (tools for reading the ISA).

    python tools/ihist.py <file.s> <symbol-substring> [--dump]
"""
import collections
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_ZN") and key in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = [l for l in lines[start:end]]
    if "--dump" in sys.argv:
        print("\n".join(body))
        return
    ins = [l.strip().split()[0] for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ins)
    print(lines[start].split(":")[0], "instructions:", len(ins))
    for k, v in sorted(c.items(), key=lambda x: -x[1]):
        print("  %-28s %d" % (k, v))


if __name__ == "__main__":
    main()
