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


class PodStageTracer:
    """Pod-startup stage timestamps, one JSON line per (pod uid, stage, wall time), written when
    AMDKUBE_POD_TRACE names a file. Every component appends to its own file (<path>.<pid>);
    hack/pod_timeline.py joins them into per-stage latency percentiles. Wall-clock times
    (time.time) so processes on one node line up."""

    def __init__(self, path: str | None = None):
        import os
        path = path if path is not None else os.environ.get("AMDKUBE_POD_TRACE")
        self.f = open(f"{path}.{os.getpid()}", "a", buffering=1 << 16) if path else None

    def __call__(self, uid: str, stage: str, t: float | None = None):
        if self.f is not None:
            self.f.write(f'{{"uid":"{uid}","stage":"{stage}","t":{time.time() if t is None else t:.6f}}}\n')

    def flush(self):
        if self.f is not None:
            self.f.flush()


POD_TRACE = PodStageTracer()
