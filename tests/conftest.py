import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmppi_hip.so")


@pytest.fixture(scope="session")
def scene_c3():
    from helpers import c3_scene
    return c3_scene()
