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


# ---- achieved parity errors ------------------------------------------------------------------
# Parity tests record the worst GPU-vs-oracle deviation they measured next to the bound they
# assert; with OKVISGPU_PARITY_REPORT=<path> the session writes them as JSON (profiles/ keeps the
# round's copy, DESIGN.md §6 quotes it).
_PARITY = {}


@pytest.fixture(scope="session")
def parity():
    def record(name, achieved, bound):
        achieved = float(achieved)
        prev = _PARITY.get(name)
        if prev is None or achieved > prev["achieved"]:
            _PARITY[name] = {"achieved": achieved, "bound": float(bound)}
        print(f"parity {name}: achieved {achieved:.3e} (bound {bound:.1e})")
        assert achieved <= bound, f"{name}: {achieved:.3e} > {bound:.1e}"
    return record


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("OKVISGPU_PARITY_REPORT")
    if path and _PARITY:
        import json
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(dict(sorted(_PARITY.items())), f, indent=1)
