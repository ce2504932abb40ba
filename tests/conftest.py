import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def engine():
    from hypermerge_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def engine_general():
    """every document through the general (workgroup-per-document) kernel"""
    from hypermerge_amd.engine import Engine, GENERAL_ONLY
    e = Engine(0, GENERAL_ONLY)
    yield e
    e.close()
