import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def engine():
    from ccka.engine import Engine

    # CCKA_TEST_LIB: run the suite against a variant build (A/B parity of a build switch)
    e = Engine(0, lib_path=os.environ.get("CCKA_TEST_LIB") or None)
    yield e
    e.close()
