"""bench.py end to end on a reduced config-M shape: the driver's JSON contract (one line, the keys
the round-end bench reads, roofline + RMSE window objects).  Runs in a child process like the driver."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config", ["M", "mesh"])
def test_bench_line_contract(gpu_ready, config):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--config", config, "--steps", "1", "--warmup", "0",
           "--res", "64", "--spp", "16", "--no-cpu-baseline", "--rmse-lanes", "4096"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert out["value"] > 0 and out["scaling"] == "strong" and out["n_gpus"] == 1
    assert out["roofline"]["achieved"] > 0 and 0 < out["roofline"]["frac"] < 1
    assert out["rmse_vs_oracle"]["rmse"] < 1e-4
    assert out["config"]["workload"].startswith(config + ":")
