"""The CPU oracle under AddressSanitizer + UBSan (oracle/Makefile `asan`, oracle/asan_driver.cpp).

Every scene family the parity tests use is rendered once by the instrumented oracle (whole frame,
per-lane records): an out-of-bounds access, use-after-free or undefined behaviour (signed
overflow, misaligned load, bad shift ...) aborts the driver with a sanitizer report.
"""
import os
import subprocess

import pytest

from conftest import REPO, SCENES

DRIVER = os.path.join(REPO, "oracle", "build", "asan_driver")


@pytest.fixture(scope="module")
def asan_driver():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"])
    syms = subprocess.run(["nm", DRIVER], capture_output=True, text=True).stdout
    assert "__asan_init" in syms and "__ubsan" in syms, "driver is not instrumented"
    return DRIVER


@pytest.mark.parametrize("scene,defines", [
    ("cbox_grid.xml", dict(res=16, spp=16, gx=4, gy=2, reuse=8)),
    ("cbox_grid.xml", dict(res=16, spp=8, reuse=4, adaptive=3, cam="thinlens")),
    ("cbox_env.xml", dict(res=16, spp=8, reuse=4, adaptive=2, lw=3, ew=0.5)),
    ("veach_grid.xml", dict(res=12, spp=8, w0=0.25, w3=4)),
    ("cbox_mesh.xml", dict(res=12, spp=4)),
    ("cbox_path.xml", dict(res=16, spp=8)),
    ("cbox_batch.xml", dict(res=12, spp=8)),
])
def test_oracle_clean_under_asan(asan_driver, scene, defines):
    args = [asan_driver, os.path.join(SCENES, scene)] + ["%s=%s" % kv for kv in defines.items()]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(args, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "non-finite film values 0" in r.stdout
