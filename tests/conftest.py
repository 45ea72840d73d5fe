import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running exhaustive check")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def engine_lib():
    from ggrs_amd import build
    build.build()
    from ggrs_amd import _lib
    return _lib.lib()
