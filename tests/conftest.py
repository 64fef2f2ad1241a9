import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _paths  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through the C ABI")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def og():
    import okvisgpu
    return okvisgpu


@pytest.fixture(scope="session")
def oracle():
    import _oracle
    return _oracle


@pytest.fixture(scope="session")
def gpu_ctx(og):
    if og.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu tests must run on the MI355X box")
    ctx = og.Context(0)
    yield ctx
    ctx.close()
