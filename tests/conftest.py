import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "scalecube-cluster_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs libswimhip.so kernels)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session", autouse=True)
def _built():
    import __graft_entry__

    __graft_entry__.build()
