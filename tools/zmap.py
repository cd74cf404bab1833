"""Dump AMVPT vs reuse-off frame stacks (means / variances) for the Z-test gate analysis."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "mitsuba3-amvpt_amd"), os.path.join(R, "tests")]
import amvpt
K = int(os.environ.get("ZK", "24"))
path = os.path.join(R, "scenes", sys.argv[1])
tag = sys.argv[2]
defs = dict(res=32, spp=64, gx=2, gy=2, reuse=4)
extra = dict(a.split("=") for a in sys.argv[3:])
defs.update({k: (int(v) if v.isdigit() else v) for k, v in extra.items()})
def frames(seeds, **d):
    sc = amvpt.load_file(path, **d)
    return np.stack([amvpt.render(sc, seed=s)[..., :3].astype(np.float64) for s in seeds])
t = frames(range(K), **defs)
r = frames(range(1000, 1000 + K), **dict(defs, reuse=1, spp=512))
os.makedirs(os.path.join(R, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(R, "gpurun_out", "zmap_%s.npz" % tag), tm=t.mean(0), tv=t.var(0, ddof=1), rm=r.mean(0), rv=r.var(0, ddof=1), K=K)
print("saved", tag)
