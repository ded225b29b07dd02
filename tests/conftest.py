import asyncio
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")
    # native artefacts are not versioned: (re)build whatever is missing or stale (no-op when fresh)
    from native import build as nb
    nb.build(sanitize=True)


def run(coro, timeout=60):
    """Run a coroutine to completion on a fresh event loop (no pytest-asyncio here)."""
    return asyncio.run(asyncio.wait_for(coro, timeout))


@pytest.fixture
def arun():
    return run


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    """`async def test_*` runs on a fresh event loop with a 120 s cap."""
    if asyncio.iscoroutinefunction(pyfuncitem.obj):
        args = {k: pyfuncitem.funcargs[k] for k in pyfuncitem._fixtureinfo.argnames}
        run(pyfuncitem.obj(**args), timeout=120)
        return True
    return None
