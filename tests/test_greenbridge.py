"""utils/greenbridge.py: synchronous code that waits on coroutines from inside run_sync."""
import asyncio
import contextvars

import pytest

from amdkube.utils import greenbridge as gb

pytestmark = pytest.mark.skipif(not gb.available(), reason="greenlet not importable")
VAR = contextvars.ContextVar("gb_test", default="unset")


def _sync_body(log, n):
    assert gb.bridged()
    total = 0
    for i in range(n):
        total += gb.await_only(_slow(i))
        log.append(i)
    return total


async def _slow(i):
    await asyncio.sleep(0.01)
    return i


async def test_bridged_calls_interleave_on_the_loop():
    log_a, log_b = [], []
    a, b = await asyncio.gather(gb.run_sync(_sync_body, log_a, 5), gb.run_sync(_sync_body, log_b, 5))
    assert a == b == 10 and log_a == log_b == list(range(5))
    assert not gb.bridged()


async def test_errors_cross_the_bridge_both_ways():
    async def boom():
        raise KeyError("inner")

    def body():
        try:
            gb.await_only(boom())
        except KeyError as e:
            raise ValueError(f"caught {e}") from None

    with pytest.raises(ValueError, match="caught 'inner'"):
        await gb.run_sync(body)
    with pytest.raises(RuntimeError):
        gb.await_only(_slow(0))                      # not bridged: refused


async def test_context_and_cancellation():
    VAR.set("outer")
    seen = []

    def body():
        seen.append(VAR.get())
        gb.await_only(asyncio.sleep(10))
        seen.append("not reached")

    t = asyncio.create_task(gb.run_sync(body))
    await asyncio.sleep(0.05)
    t.cancel()
    with pytest.raises(asyncio.CancelledError):
        await t
    assert seen == ["outer"]


async def test_plain_functions_pass_through():
    assert await gb.run_sync(lambda x, y=1: x + y, 2, y=3) == 5
