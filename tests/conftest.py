import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def native_lib():
    """The built libgcg_spmm.so (built in-tree if missing; never a fallback)."""
    from graphconvgeo_amd import _build, _native
    _build.build_native()
    return _native.load()


@pytest.fixture(scope="session")
def cuda(native_lib):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch.device("cuda:0")
