import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "astro-sph-tools_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG_ROOT, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size property tests")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def asp():
    import asp_amd
    from asp_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return asp_amd


@pytest.fixture(scope="session")
def gpu(asp):
    """The GPU tests must run the native path: fail loudly if it cannot load."""
    from asp_amd import _lib
    L = _lib.lib()
    if L.asp_device_count() < 1:
        pytest.fail("no HIP device visible for a -m gpu test")
    return asp
