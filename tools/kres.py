"""Per-kernel resources of the built HIP library (scratch bytes per lane, VGPRs, SGPRs, code size),
read from the gfx950 code object inside lib/libamvpt_hip.so with the ROCm LLVM tools.

    python tools/kres.py [libdir] [substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(so):
    """Every gfx950 code object bundled in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, so,
                        os.path.join(d, "junk")], check=True, capture_output=True)
        blob = open(fat, "rb").read()
        # the section holds one offload bundle per translation unit, each 4096-aligned
        starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", blob)]
        outs = []
        for n, s in enumerate(starts):
            e = starts[n + 1] if n + 1 < len(starts) else len(blob)
            part = os.path.join(d, "b%d" % n)
            open(part, "wb").write(blob[s:e])
            co = part + ".co"
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + part, "--output=" + co],
                               capture_output=True)
            if r.returncode == 0 and os.path.getsize(co):
                outs.append(open(co, "rb").read())
        return outs


def kernels(so):
    res = {}
    for blob in code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(blob)
            f.flush()
            out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", "-W", f.name], check=True,
                                 capture_output=True, text=True).stdout
        for line in out.splitlines():
            p = line.split()
            if len(p) < 8:
                continue
            name, val, size = p[7], p[1], p[2]
            for suf, key in ((".private_seg_size", "scratch"), (".num_vgpr", "vgpr"), (".numbered_sgpr", "sgpr")):
                if name.endswith(suf):
                    res.setdefault(name[: -len(suf)], {})[key] = int(val, 16)
            if p[3] == "FUNC":
                res.setdefault(name, {})["code_bytes"] = int(size)
    return res


def main():
    args = sys.argv[1:]
    lib = args.pop(0) if args and not args[0].startswith("k_") else "lib"
    so = os.path.join(REPO, "mitsuba3-amvpt_amd", lib, "libamvpt_hip.so")
    for k, v in sorted(kernels(so).items()):
        if "vgpr" not in v or (args and not any(a in k for a in args)):
            continue
        print("%-90s vgpr %3d sgpr %3d scratch %3d code %6d" % (k[:90], v["vgpr"], v.get("sgpr", 0), v.get("scratch", 0),
                                                                 v.get("code_bytes", 0)))


if __name__ == "__main__":
    main()
