"""The C++ host's multi-GPU entry (amvpt_host_render_multi: one thread per device, lane shards,
ncclReduce of the RGBW ImageBlocks, develop on devices[0]) on the GPUs this box has.  With one
device the reduce is RCCL's single-rank path and the result must equal amvpt_host_render up to the
film's float-atomic summation order (relative 1e-5 of the film scale);
the partition itself is checked against amvpt.dist on CPU (test_multirank.py)."""
import os

import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene,defines", [
    ("cbox_grid.xml", dict(res=32, spp=32, gx=4, gy=2, reuse=8)),
    ("cbox_grid.xml", dict(res=32, spp=16, reuse=4, adaptive=3)),
    ("cbox_env.xml", dict(res=32, spp=16, reuse=4, lw=3)),
], ids=["g8", "g4_adaptive", "env_weighted"])
def test_render_multi_single_device_equals_render(gpu_ready, amvpt_mod, scene, defines):
    s = amvpt_mod.load_file(os.path.join(SCENES, scene), **defines)
    c1, c2 = amvpt_mod.Counters(), amvpt_mod.Counters()
    ref = amvpt_mod.render(s, raw=True, counters=c1)
    out = amvpt_mod.render_multi(s, [0], raw=True, counters=c2)
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()
    assert c1.lanes == c2.lanes and c1.vertices == c2.vertices and c1.view_splats == c2.view_splats
    dev, img = amvpt_mod.render_multi(s, [0]), amvpt_mod.render(s)
    assert np.abs(dev - img).max() <= 1e-4 * max(1.0, np.abs(img).max())
