import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu_lib():
    """The HIP library, loaded once; GPU tests fail loudly if it is missing."""
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    from zonos_vibes_amd import _lib
    return _lib.lib()
