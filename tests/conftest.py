import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def hjd():
    import ocljpegdecoder_amd
    return ocljpegdecoder_amd


@pytest.fixture(scope="session")
def ctx(hjd):
    import torch
    assert torch.cuda.is_available(), "GPU test needs a HIP device"
    c = hjd.Context(0)
    yield c
    c.close()
