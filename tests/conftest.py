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


@pytest.fixture(params=["corner", "centre"])
def convention(request, oracle, gpu):
    """Both settings of PARITY_ASSUMPTIONS.md row 1 (libvips reduce sampling: X = o * s
    or X = (o + 0.5) * s - 0.5), in the engine (mipx_set_reduce_sampling) and in the
    oracle; the defaults come back afterwards."""
    prev_engine, prev_oracle = gpu.reduce_sampling(), oracle.get_switch("reduce_centre")
    gpu.set_reduce_sampling(request.param)
    oracle.set_switch("reduce_centre", int(request.param == "centre"))
    yield request.param
    gpu.set_reduce_sampling(prev_engine)
    oracle.set_switch("reduce_centre", prev_oracle)


@pytest.fixture
def rng():
    return np.random.default_rng(20241220)


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
