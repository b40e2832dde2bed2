import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libsiren_hip.so")


@pytest.fixture(scope="session")
def lib():
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def dev(lib):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")
