"""Per-item exponential back-off keyed by an event time.

Reference: staging/src/k8s.io/client-go/util/flowcontrol/backoff.go (Backoff: Next,
IsInBackOffSince, IsInBackOffSinceUpdate, GC, hasExpired). The kubelet keeps one of these for
container restarts (kubelet.go:859, 10 s doubling to MaxContainerBackOff = 300 s) and
kuberuntime_manager.go doBackOff consults it with the finish time of the container's last
exited instance.

Times are float seconds on whatever clock `clock` returns (wall clock by default, because the
event times handed in are container finish timestamps from the runtime).
"""
from __future__ import annotations

import threading
import time


class Backoff:
    __slots__ = ("clock", "default", "max", "_items", "_lock")

    def __init__(self, initial: float, maximum: float, clock=time.time):
        self.clock = clock
        self.default, self.max = float(initial), float(maximum)
        self._items: dict[str, list[float]] = {}     # id -> [backoff, last_update]
        self._lock = threading.Lock()

    def get(self, key: str) -> float:
        with self._lock:
            e = self._items.get(key)
            return e[0] if e else 0.0

    def _expired(self, event_time: float, last_update: float) -> bool:
        # stable once the item has been fine for twice the maximum back-off
        return event_time - last_update > self.max * 2

    def next(self, key: str, event_time: float):
        with self._lock:
            e = self._items.get(key)
            if e is None or self._expired(event_time, e[1]):
                e = self._items[key] = [self.default, 0.0]
            else:
                e[0] = min(e[0] * 2, self.max)
            e[1] = self.clock()

    def reset(self, key: str):
        with self._lock:
            self._items.pop(key, None)

    delete_entry = reset

    def is_in_backoff_since(self, key: str, event_time: float) -> bool:
        with self._lock:
            e = self._items.get(key)
            if e is None or self._expired(event_time, e[1]):
                return False
            return self.clock() - event_time < e[0]

    def is_in_backoff_since_update(self, key: str, event_time: float) -> bool:
        with self._lock:
            e = self._items.get(key)
            if e is None or self._expired(event_time, e[1]):
                return False
            return event_time - e[1] < e[0]

    def remaining(self, key: str, event_time: float) -> float:
        """Seconds until is_in_backoff_since(key, event_time) turns False (0 when not in back-off)."""
        with self._lock:
            e = self._items.get(key)
            if e is None or self._expired(event_time, e[1]):
                return 0.0
            return max(0.0, event_time + e[0] - self.clock())

    def gc(self):
        with self._lock:
            now = self.clock()
            for k in [k for k, e in self._items.items() if now - e[1] > self.max * 2]:
                del self._items[k]

    def drop_prefix_containing(self, part: str):
        """Forget every item whose key contains `part` (e.g. all containers of one pod uid)."""
        with self._lock:
            for k in [k for k in self._items if part in k]:
                del self._items[k]

    def clear(self):
        with self._lock:
            self._items.clear()

    def __len__(self):
        return len(self._items)
