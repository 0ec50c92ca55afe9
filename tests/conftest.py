import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libaiyagari on cuda:0)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """GPU tests must run the HIP path; skipping is not allowed on a GPU box, and off a
    GPU box the -m gpu selection is never run."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    from aiyagari_hark_amd import build, _lib
    build.build(verbose=False)
    _lib.load()
    return torch.device("cuda:0")
