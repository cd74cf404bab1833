"""amvpt.compare: the RMSE / PSNR gate tool (CPU)."""
import json
import subprocess
import sys

import numpy as np

from conftest import PKG


def test_metrics_values():
    from amvpt.compare import metrics
    b = np.ones((4, 4, 3), np.float32)
    a = b.copy()
    a[0, 0, 0] = 1.5
    m = metrics(a, b)
    assert np.isclose(m["rmse"], np.sqrt(0.25 / 48))
    assert np.isclose(m["max_abs"], 0.5)
    assert m["psnr"] > 0 and m["nan_mismatch"] == 0
    assert metrics(b, b)["rmse"] == 0.0


def test_cli_on_exr_files(amvpt_mod, tmp_path):
    rng = np.random.default_rng(0)
    b = rng.random((9, 13, 3)).astype(np.float32)
    a = b + np.float32(1e-4)
    pa, pb = str(tmp_path / "a.exr"), str(tmp_path / "b.exr")
    amvpt_mod.write_exr(pa, a)
    amvpt_mod.write_exr(pb, b)
    out = subprocess.run([sys.executable, "-m", "amvpt.compare", pa, pb, "--tolerance", "1e-3"], cwd=PKG,
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    m = json.loads(out.stdout)
    assert abs(m["rmse"] - 1e-4) < 1e-6
    bad = subprocess.run([sys.executable, "-m", "amvpt.compare", pa, pb, "--tolerance", "1e-5"], cwd=PKG,
                         capture_output=True, text=True)
    assert bad.returncode == 1
