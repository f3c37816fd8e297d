import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def hip():
    """The HIP library; GPU tests fail loudly if it or the GPU is missing."""
    import torch
    from posecnn_amd import _lib
    assert torch.cuda.is_available(), "gpu-marked test needs a GPU"
    return _lib.load()
