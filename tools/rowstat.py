"""Measurement helper: one frame of a bench config through a library dir, printing the lane counters
(splat_fallback of an AMVPT_SPLAT_ROWSTAT=1 build counts the lanes of rows that take the per-lane splat path).
    AB_CONFIG=M python tools/rowstat.py <libdir>"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["AMVPT_LIB_DIR"] = os.path.join(REPO, "mitsuba3-amvpt_amd", sys.argv[1])
sys.path[:0] = [REPO, os.path.join(REPO, "mitsuba3-amvpt_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402
import amvpt  # noqa: E402
from ab_value import CONFIGS  # noqa: E402

cfg = dict(CONFIGS[os.environ.get("AB_CONFIG", "M")])
scene = cfg.pop("scene")
s = amvpt.load_file(os.path.join(REPO, "scenes", scene), **cfg)
sd, vd, p = s.describe(0, 0, 0)
dev = amvpt.DeviceScene(sd)
film = torch.zeros((p.film_height, p.film_width, 4), dtype=torch.float32, device="cuda")
c = amvpt.Counters()
dev.render(vd, p, film.data_ptr(), counters=c)
torch.cuda.synchronize()
d = c.as_dict()
print(json.dumps({"config": os.environ.get("AB_CONFIG", "M"), "lib": sys.argv[1], "lanes": d["lanes"],
                  "view_splats": d["view_splats"], "splat_fallback": d["splat_fallback"],
                  "frac_of_splats": d["splat_fallback"] / max(1, d["view_splats"])}))
