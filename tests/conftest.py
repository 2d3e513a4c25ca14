import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")


@pytest.fixture(scope="session")
def hip():
    """The loaded C-ABI library; GPU tests only."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from physics_informed_image_segmentation_amd import _hip
    return _hip.lib()
