import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "self-play-racing_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    from tests.golden_util import Golden
    return Golden()


@pytest.fixture(scope="session")
def oracle():
    from oracle.orc import Oracle
    return Oracle(device_libm=False)


@pytest.fixture(scope="session")
def oracle_dev():
    from oracle.orc import Oracle
    return Oracle(device_libm=True)
