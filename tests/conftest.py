import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgvrt.so on cuda:0)")
    config.addinivalue_line("markers", "slow: large CPU-oracle cases")


@pytest.fixture(scope="session")
def gv():
    return importlib.import_module("3dgvrt_lightfield_amd")


@pytest.fixture(scope="session")
def O():
    import oracle  # test infrastructure (oracle/oracle.py)
    return oracle


@pytest.fixture(scope="session")
def renderer(gv):
    if gv.device_count() == 0:
        pytest.fail("gpu test on a machine without a HIP device")
    r = gv.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="session")
def config1(gv):
    return gv.scene.config1()


@pytest.fixture(scope="session")
def config1_enc(O, config1):
    return O.enclose(config1)
