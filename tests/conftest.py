import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.hookimpl(trylast=True)   # after `-m` deselection
def pytest_collection_modifyitems(session, config, items):
    """torch's wheel carries its own HIP runtime: when a GPU test also uses torch (device buffers, RCCL),
    torch must initialise the GPU before libsiddhi_gfx's runtime does, or torch finds no device.  So a
    session with GPU tests initialises torch's runtime first (no-op without a GPU)."""
    if not any(it.get_closest_marker("gpu") for it in items):
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # noqa: BLE001  (torch missing or no device: the tests skip or fail on their own)
        pass
