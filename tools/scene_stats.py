"""BVH node / primitive counts of a scene as built on the device (amvpt_scene_stats).

    python tools/scene_stats.py scenes/cbox_mesh.xml [key=value ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mitsuba3-amvpt_amd")]


def main():
    import amvpt
    kw = {}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        kw[k] = int(v) if v.isdigit() else v
    s = amvpt.load_file(sys.argv[1], **kw)
    sd, vd, p = s.describe(0, 0, 0)
    dev = amvpt.DeviceScene(sd)
    nn, npr = dev.stats()
    print("%s nodes %d (%d KB at 32 B) prims %d (%d KB at 64 B)" % (os.path.basename(sys.argv[1]), nn,
          nn * 32 // 1024, npr, npr * 64 // 1024))


if __name__ == "__main__":
    main()
