"""Shared test setup: the `gpu` marker, the oracle (checker only) and fixtures."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmipx.so on the device)")
    config.addinivalue_line("markers", "slow: full-size property checks")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def gpu():
    """libmipx with a live device; GPU tests fail loudly if the device or the .so is missing."""
    import imaginary_amd as ia
    n = ia.device_count()
    assert n > 0, "no HIP device visible to libmipx.so"
    return ia


@pytest.fixture
def rng():
    return np.random.default_rng(20241220)


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
