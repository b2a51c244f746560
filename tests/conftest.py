import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "video-style-transfer_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP extension calls)")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
        return cache[name]

    return load


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(params=["f32", "bf16x6"])
def step_policy(request):
    """The fp32-class GEMM policies a whole training step must pass the reference's golden bar
    under: exact fp32 MFMA (the library default) and bf16x6 everywhere (bench.py's headline)."""
    from vst import ops

    old = ops.POLICY_NAME[0] or ops.DEFAULT_POLICY
    ops.use_policy(request.param)
    yield request.param
    ops.use_policy(old if old in ops.POLICIES else ops.DEFAULT_POLICY)
