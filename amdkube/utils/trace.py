"""utiltrace: step timers that log only when the whole operation was slow.

Reference: staging/src/k8s.io/apiserver/pkg/util/trace/trace.go; the scheduler wraps
Schedule in `trace.LogIfLong(100ms)` with steps "Computing predicates", "Prioritizing",
"Selecting host" (plugin/pkg/scheduler/core/generic_scheduler.go:110-154).
"""
from __future__ import annotations

import logging
import time

log = logging.getLogger("amdkube.trace")


class Trace:
    __slots__ = ("name", "start", "steps")

    def __init__(self, name: str):
        self.name = name
        self.start = time.perf_counter()
        self.steps: list[tuple[float, str]] = []

    def step(self, msg: str):
        self.steps.append((time.perf_counter(), msg))

    def total(self) -> float:
        return time.perf_counter() - self.start

    def format(self) -> str:
        out = [f'Trace "{self.name}" (total {self.total() * 1000:.1f}ms):']
        last = self.start
        for t, msg in self.steps:
            out.append(f"  [{(t - self.start) * 1000:.1f}ms] [{(t - last) * 1000:.1f}ms] {msg}")
            last = t
        return "\n".join(out)

    def log_if_long(self, threshold_s: float) -> bool:
        if self.total() >= threshold_s:
            log.info(self.format())
            return True
        return False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
