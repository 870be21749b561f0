import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Per-frame contexts in flight (tests/test_gpu_inflight.py and the ordering tests: up to 16 shared contexts, each on its
# own stream -- the shape of bench.py --batch 0, which the N > 1 ranks and --shadows run) need a hardware queue per
# stream, and HIP reads GPU_MAX_HW_QUEUES once, when it initialises -- so it is raised here, before any test imports
# torch or loads libvhx (bench.py's hw_queues rule, F + 4). The N = 1 default bench (batches of 7 on 3 contexts) needs
# no raise; the batch tests pass either way.
try:
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 20:
        os.environ["GPU_MAX_HW_QUEUES"] = "20"
except ValueError:
    os.environ["GPU_MAX_HW_QUEUES"] = "20"


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
