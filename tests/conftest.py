import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import pgdist  # noqa: E402,F401  (registers the package under its importable name)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def dev():
    import torch
    return torch.device("cuda", 0)


@pytest.fixture
def deterministic():
    """fixed-order BN statistics (no float atomics) for bitwise comparisons"""
    from pgdist.ops import kernels as K
    K.set_deterministic(True)
    yield
    K.set_deterministic(False)
