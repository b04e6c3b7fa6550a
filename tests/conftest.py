import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mcmc-for-nested-data_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu_lib():
    """The loaded HIP library; GPU tests fail loudly (never skip to CPU) without it."""
    from nestmc import _lib
    lib = _lib.load()
    n = _lib.device_count()
    assert n >= 1, "no HIP device visible"
    return lib
