import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the device)")


@pytest.fixture(scope="session")
def O():
    from oracle import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def engine():
    from redisson_amd import SketchEngine

    e = SketchEngine(device=0)
    yield e
    e.close()


@pytest.fixture()
def client():
    from redisson_amd import Config, Redisson

    r = Redisson.create(Config(device=0))
    yield r
    r.shutdown()
