import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "adaptive-compression_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_present():
    return os.path.exists("/dev/kfd")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def hip_lib():
    """The product C-ABI library, loaded through the product loader."""
    if not gpu_present():
        pytest.skip("no GPU (/dev/kfd) in this container")
    from ambc import _lib
    return _lib.load()
