import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mini-kvstore-v2_amd")
for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: full-size workload")


@pytest.fixture(scope="session", autouse=True)
def _built():
    import build  # mini-kvstore-v2_amd/build.py (rebuilds only if sources are newer)
    build.build()
    yield


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gctx():
    import kvreplay
    ctx = kvreplay.Context(0)
    yield ctx
    ctx.close()
