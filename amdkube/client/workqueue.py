"""Work queues and Parallelize (client-go util/workqueue).

Reference: util/workqueue/queue.go:33 (dirty/processing sets: an item is never processed
concurrently and re-adds while processing are coalesced), delaying_queue.go,
rate_limitting_queue.go + default_rate_limiters.go (per-item exponential 5ms→1000s),
parallelizer.go:29 (Parallelize(workers, pieces, fn)).
"""
from __future__ import annotations

import asyncio
import collections
import heapq
import itertools
from concurrent.futures import ThreadPoolExecutor


class ShutDown(Exception):
    pass


class WorkQueue:
    def __init__(self, name: str = ""):
        self.name = name
        self._queue: collections.deque = collections.deque()
        self._dirty: set = set()
        self._processing: set = set()
        self._waiters: collections.deque = collections.deque()
        self._shutdown = False
        self.adds = 0

    def add(self, item):
        if self._shutdown or item in self._dirty:
            return
        self.adds += 1
        self._dirty.add(item)
        if item in self._processing:
            return
        self._queue.append(item)
        self._wake_one()

    def _wake_one(self):
        while self._waiters:
            f = self._waiters.popleft()
            if not f.done():
                f.set_result(None)
                return

    def __len__(self):
        return len(self._queue)

    async def get(self):
        """Next item (raises ShutDown once shut down and drained)."""
        while not self._queue:
            if self._shutdown:
                raise ShutDown()
            f = asyncio.get_running_loop().create_future()
            self._waiters.append(f)
            await f
        item = self._queue.popleft()
        self._processing.add(item)
        self._dirty.discard(item)
        return item

    def get_nowait(self):
        if not self._queue:
            return None
        item = self._queue.popleft()
        self._processing.add(item)
        self._dirty.discard(item)
        return item

    def done(self, item):
        self._processing.discard(item)
        if item in self._dirty:
            self._queue.append(item)
            self._wake_one()

    def shutdown(self):
        self._shutdown = True
        while self._waiters:
            f = self._waiters.popleft()
            if not f.done():
                f.set_result(None)

    @property
    def shutting_down(self):
        return self._shutdown


class DelayingQueue(WorkQueue):
    def __init__(self, name=""):
        super().__init__(name)
        self._heap: list = []
        self._seq = itertools.count()
        self._timer: asyncio.TimerHandle | None = None

    def add_after(self, item, delay: float):
        if delay <= 0:
            self.add(item)
            return
        loop = asyncio.get_running_loop()
        when = loop.time() + delay
        heapq.heappush(self._heap, (when, next(self._seq), item))
        self._arm()

    def _arm(self):
        loop = asyncio.get_running_loop()
        if self._timer is not None:
            self._timer.cancel()
        if self._heap:
            self._timer = loop.call_at(self._heap[0][0], self._fire)

    def _fire(self):
        loop = asyncio.get_running_loop()
        now = loop.time()
        while self._heap and self._heap[0][0] <= now:
            _, _, item = heapq.heappop(self._heap)
            self.add(item)
        self._timer = None
        self._arm()


class ItemExponentialFailureRateLimiter:
    def __init__(self, base=0.005, cap=1000.0):
        self.base, self.cap = base, cap
        self.failures: dict = {}

    def when(self, item) -> float:
        n = self.failures.get(item, 0)
        self.failures[item] = n + 1
        return min(self.cap, self.base * (2 ** n))

    def forget(self, item):
        self.failures.pop(item, None)

    def num_requeues(self, item) -> int:
        return self.failures.get(item, 0)


class RateLimitingQueue(DelayingQueue):
    def __init__(self, name="", limiter=None):
        super().__init__(name)
        self.limiter = limiter or ItemExponentialFailureRateLimiter()

    def add_rate_limited(self, item):
        self.add_after(item, self.limiter.when(item))

    def forget(self, item):
        self.limiter.forget(item)

    def num_requeues(self, item):
        return self.limiter.num_requeues(item)


_POOL: ThreadPoolExecutor | None = None


def parallelize(workers: int, pieces: int, fn) -> None:
    """Run fn(i) for i in range(pieces) on up to `workers` threads (Parallelize semantics).

    The scheduler's per-node checks are native (C++) or short Python; for pure-Python
    pieces the GIL makes threads pointless, so small piece counts run inline.
    """
    global _POOL
    if pieces <= 0:
        return
    if workers <= 1 or pieces < 64:
        for i in range(pieces):
            fn(i)
        return
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=16, thread_name_prefix="parallelize")
    list(_POOL.map(fn, range(pieces)))


async def parallelize_async(workers: int, pieces: int, afn) -> None:
    sem = asyncio.Semaphore(workers)

    async def one(i):
        async with sem:
            await afn(i)
    await asyncio.gather(*(one(i) for i in range(pieces)))
