import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "mpas-regent_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libmpasdyn.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def x1_2562():
    from mpasdyn import mesh
    return mesh.load_x1_2562()
