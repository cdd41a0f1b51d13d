import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def wgt():
    import webgputracer_amd

    return webgputracer_amd


@pytest.fixture(scope="session")
def ctx(wgt):
    """One HIP context for the whole GPU session (tests re-upload scenes)."""
    c = wgt.Context(0)
    yield c
    c.close()
