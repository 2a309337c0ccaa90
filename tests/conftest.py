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
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: full-size property tests")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """The GPU tests share one process between PyTorch-ROCm (its own bundled HIP runtime) and
    libksqldb_hip.so (/opt/rocm's).  Initialise torch's runtime before the library's first
    call, the order bench.py uses."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
        except ImportError:
            return
        if torch.cuda.is_available():
            torch.cuda.init()
