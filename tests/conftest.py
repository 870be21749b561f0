import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """Builds libvhx.so / liboracle.so when they are missing (the GPU box receives them prebuilt)."""
    import __graft_entry__ as g
    g.ensure_built()
    yield


@pytest.fixture(scope="session")
def oracle():
    from tests._oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu():
    from voxelhex_amd import Raytracer
    rt = Raytracer(0)
    yield rt
    rt.close()
