import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwgaead on the device)")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first():
    """Initialise torch's HIP runtime before libwgaead's: torch ships its own
    libamdhip64 beside /opt/rocm's, and the one that starts second in a process
    must find the device already set up by the first (torch second reports no
    device). bench.py and smoke() touch torch.cuda first for the same reason."""
    try:
        import torch
        torch.cuda.is_available()
    except ImportError:
        pass
    yield


@pytest.fixture(scope="session")
def engine():
    """One device engine for the whole GPU session (tests run in a single process on the box)."""
    from wgtest import wg
    e = wg().Engine(0, key_slots=4096)
    yield e
    e.close()
