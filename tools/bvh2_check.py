"""Two-box BVH of the mesh scene: node count and depth (amvpt_scene_bvh2)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mitsuba3-amvpt_amd")]
import amvpt  # noqa: E402

for name in ("cbox_mesh.xml", "cbox_grid.xml", "veach_grid.xml"):
    s = amvpt.load_file(os.path.join(REPO, "scenes", name), res=16, spp=16)
    sd, vd, p = s.describe(0, 0, 0)
    d = amvpt.DeviceScene(sd)
    print(name, "nodes/prims", d.stats(), "bvh2 (nodes, depth)", d.bvh2(), flush=True)
