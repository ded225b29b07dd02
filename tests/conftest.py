import asyncio
import gc
import logging
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


# Shutdown hygiene: every component's stop() awaits its tasks and closes its sessions. asyncio
# reports a leak through its logger (the loop's default exception handler); any such report
# during a test fails it.
_LEAK_MARKS = ("Task was destroyed but it is pending", "Unclosed client session", "Unclosed connector")


class _LeakRecorder(logging.Handler):
    def __init__(self):
        super().__init__(logging.ERROR)
        self.seen: list[str] = []

    def emit(self, record):
        msg = record.getMessage()
        if msg.startswith(_LEAK_MARKS):
            self.seen.append(msg.splitlines()[0] + " " + " ".join(msg.splitlines()[1:2])[:200])


_LEAKS = _LeakRecorder()
logging.getLogger("asyncio").addHandler(_LEAKS)


@pytest.fixture(autouse=True)
def no_leaked_tasks_or_sessions():
    _LEAKS.seen.clear()
    yield
    gc.collect()
    if _LEAKS.seen:
        found, _LEAKS.seen[:] = list(_LEAKS.seen), []
        pytest.fail("asyncio leak (a stop() that does not await its tasks or close its sessions):\n  " + "\n  ".join(found))


def run(coro, timeout=60):
    """Run a coroutine to completion on a fresh event loop (no pytest-asyncio here)."""
    return asyncio.run(asyncio.wait_for(coro, timeout))


def log_text(path: str) -> str:
    """A container's output from its log file (the CRI records the log pump writes, decoded)."""
    from amdkube.kubelet.logs import read_text
    return read_text(path)


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
