import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def lib():
    import __graft_entry__ as g
    g.build_lib()
    from dslabs_amd import _lib
    return _lib.load()
