import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "clustering-driven-replication-strategy_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libcdr.so")


@pytest.fixture(scope="session")
def ctx():
    import _cdr

    c = _cdr.Context(int(os.environ.get("CDR_DEVICE", "0")))
    yield c
    c.close()
