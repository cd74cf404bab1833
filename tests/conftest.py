"""pytest configuration: markers, import paths and shared fixtures.

`-m "not gpu"` runs the oracle golden tests, host-framework tests, C-ABI
export checks and multi-rank (gloo) tests on CPU; `-m gpu` runs the HIP
parity tests through the C-ABI on an MI355X.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mitsuba3-amvpt_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

SCENES = os.path.join(REPO, "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through the C-ABI")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def amvpt_mod():
    import amvpt
    return amvpt


@pytest.fixture(scope="session")
def gpu_ready(amvpt_mod):
    n = amvpt_mod.device_count()
    if n <= 0:
        pytest.fail("no HIP device visible for a @gpu test")
    return n
