"""Run synchronous code on the event loop with points where it may wait on a coroutine.

The apiserver's registry and storage layers are synchronous: over the embedded MVCC store a
write returns at once. Over a remote store (Etcd3Store) a write is a network round trip, and
a blocking call there stalls every other request on the loop for that long, so concurrent
writes could never share a round trip. `run_sync` runs such a call in a greenlet; where the
store would block, `await_only(coro)` suspends the greenlet and hands the coroutine to the
loop, and the call resumes with its result. Everything else stays ordinary synchronous code
on the loop thread (no locks, no threads), and the same code still runs unbridged, blocking,
where no loop drives it (bootstrap, tests, tools).

The reference needs none of this: Go's apiserver runs each request on its own goroutine and
etcd3/store.go blocks that goroutine in the client (staging/src/k8s.io/apiserver/pkg/storage/
etcd3/store.go:152 Create -> s.client.KV.Txn). A suspended greenlet is the equivalent of that
parked goroutine.
"""
from __future__ import annotations

import contextvars
import sys

try:
    import greenlet
except ImportError:           # blocking stores then simply block
    greenlet = None


if greenlet is not None:
    class _Bridge(greenlet.greenlet):
        """A greenlet whose parent is the coroutine driving it (see run_sync)."""
        __slots__ = ("driver",)

        def __init__(self, fn, driver):
            super().__init__(fn, driver)
            self.driver = driver


def available() -> bool:
    return greenlet is not None


def bridged() -> bool:
    """True inside run_sync: await_only may be called."""
    return greenlet is not None and isinstance(greenlet.getcurrent(), _Bridge)


def await_only(aw):
    """From synchronous code running under run_sync: wait for `aw` on the loop."""
    cur = greenlet.getcurrent()
    if not isinstance(cur, _Bridge):
        if hasattr(aw, "close"):
            aw.close()
        raise RuntimeError("await_only outside run_sync")
    return cur.driver.switch(aw)


async def run_sync(fn, *args, **kwargs):
    """Call fn(*args, **kwargs); each await_only inside it is awaited here."""
    if greenlet is None:
        return fn(*args, **kwargs)
    g = _Bridge(fn, greenlet.getcurrent())
    g.gr_context = contextvars.copy_context()
    result = g.switch(*args, **kwargs)
    while not g.dead:
        try:
            value = await result
        except BaseException:         # the waited coroutine's error surfaces at the await_only
            result = g.throw(*sys.exc_info())
        else:
            result = g.switch(value)
    return result
