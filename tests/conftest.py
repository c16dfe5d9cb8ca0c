import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "phase-based-motion-manipulation_amd")
for p in (HERE, PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: large-size case")


@pytest.fixture(scope="session", autouse=True)
def _oracle_built():
    import oracle_py
    oracle_py.build()
    yield
