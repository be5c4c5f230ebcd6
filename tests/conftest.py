"""pytest configuration: markers, import paths, and shared fixtures."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "shadow-1_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def shd():
    import shdgpu
    shdgpu.lib()
    return shdgpu


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    return oracle_ffi
