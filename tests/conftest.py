import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on the MI355X box)")
    config.addinivalue_line("markers", "slow: large configuration")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def leo():
    """The product library, initialised on the GPU."""
    import leopard_amd
    res = leopard_amd.leo_init()
    assert res == leopard_amd.LeopardResult.Success, (res, leopard_amd.last_error())
    return leopard_amd
