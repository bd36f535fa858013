import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwgaead on the device)")


@pytest.fixture(scope="session")
def engine():
    """One device engine for the whole GPU session (tests run in a single process on the box)."""
    from wgtest import wg
    e = wg().Engine(0, key_slots=4096)
    yield e
    e.close()
