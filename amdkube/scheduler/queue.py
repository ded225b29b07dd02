"""Scheduling queue: PriorityQueue with an unschedulable sub-queue.

Reference: plugin/pkg/scheduler/core/scheduling_queue.go:64,163 — activeQ ordered by pod
priority (then arrival), unschedulableQ parked until a cluster event (node add/update,
assigned pod deleted/terminated) calls MoveAllToActiveQueue; FIFO fallback without the
PodPriority gate. Unschedulable pods are also retried on a timer so nothing is stranded.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools

from ..api import meta as m


class SchedulingQueue:
    def __init__(self, use_priority: bool = True, unschedulable_retry: float = 30.0):
        self.use_priority = use_priority
        self.heap: list = []
        self.items: dict[str, dict] = {}
        self.unschedulable: dict[str, dict] = {}
        self.seq = itertools.count()
        self._waiters: list[asyncio.Future] = []
        self.retry = unschedulable_retry
        self.received_move = False

    def __len__(self):
        return len(self.items)

    def _prio(self, pod):
        return -int((pod.get("spec") or {}).get("priority") or 0) if self.use_priority else 0

    def add(self, pod: dict):
        key = m.key_of(pod)
        self.unschedulable.pop(key, None)
        if key in self.items:
            self.items[key] = pod
            return
        self.items[key] = pod
        heapq.heappush(self.heap, (self._prio(pod), next(self.seq), key))
        self._wake()

    def update(self, pod: dict):
        key = m.key_of(pod)
        if key in self.items:
            self.items[key] = pod
        elif key in self.unschedulable:
            self.unschedulable.pop(key)
            self.add(pod)
        else:
            self.add(pod)

    def delete(self, pod: dict):
        key = m.key_of(pod)
        self.items.pop(key, None)
        self.unschedulable.pop(key, None)

    def add_unschedulable(self, pod: dict):
        key = m.key_of(pod)
        if self.received_move:
            self.received_move = False
            self.add(pod)
            return
        self.unschedulable[key] = pod
        asyncio.get_running_loop().call_later(self.retry, self._retry_one, key)

    def _retry_one(self, key):
        pod = self.unschedulable.pop(key, None)
        if pod is not None:
            self.add(pod)

    def move_all_to_active(self):
        if not self.unschedulable:
            self.received_move = True
            return
        pods = list(self.unschedulable.values())
        self.unschedulable.clear()
        for p in pods:
            self.add(p)

    def _wake(self):
        while self._waiters:
            f = self._waiters.pop()
            if not f.done():
                f.set_result(None)
                return

    def pop_nowait(self):
        while self.heap:
            _, _, key = heapq.heappop(self.heap)
            pod = self.items.pop(key, None)
            if pod is not None:
                return pod
        return None

    async def pop(self) -> dict:
        while True:
            pod = self.pop_nowait()
            if pod is not None:
                self.received_move = False
                return pod
            f = asyncio.get_running_loop().create_future()
            self._waiters.append(f)
            await f
