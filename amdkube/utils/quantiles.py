"""Prometheus Summary with quantile objectives over a sliding time window.

`prometheus_client.Summary` exports only `_sum`/`_count`. The reference's Go client exports
`{quantile="0.5|0.9|0.99"}` series for every Summary (prometheus/client_golang summary.go:
DefObjectives {0.5: 0.05, 0.9: 0.01, 0.99: 0.001}, DefMaxAge 10 min, DefAgeBuckets 5,
DefBufCap 500), and those are what the e2e metrics checks and dashboards read
(test/e2e/framework/metrics_util.go:264-270; pkg/kubelet/metrics/metrics.go:53-152).

Each quantile stream is the biased/targeted-quantile summary of Cormode, Korn, Muthukrishnan and
Srivastava ("Effective computation of biased quantiles over data streams", ICDE 2005): a sorted
list of (value, width, delta) tuples compressed under the targeted invariant
f(r, n) = min over objectives (q, e) of 2e*r/q when r >= q*n, else 2e*(n-r)/(1-q), so the rank
error at quantile q stays within e*n. Observations are buffered (500) and merged sorted.

The per-label-set state is native (amdkube._native._quantile over native/quantile_core.h, one
shared sorted buffer merged into every age-bucket stream); the pure-Python streams below are
the same algorithm, used when the extension is not built.

Windowing follows the Go client: AGE_BUCKETS streams, every observation goes into all of them,
and every max_age/AGE_BUCKETS the oldest stream is reset and becomes the newest. Quantiles are
read from the oldest, which covers the last max_age. `_sum` and `_count` are cumulative.
"""
from __future__ import annotations

import math
import threading
import time

from prometheus_client.metrics_core import Metric

DEF_OBJECTIVES = {0.5: 0.05, 0.9: 0.01, 0.99: 0.001}
DEF_MAX_AGE = 600.0
DEF_AGE_BUCKETS = 5
BUF_CAP = 500


class TargetedStream:
    """One CKMS targeted-quantile stream."""
    __slots__ = ("targets", "vals", "widths", "deltas", "n", "buf")

    def __init__(self, targets: dict[float, float]):
        self.targets = sorted(targets.items())
        self.vals: list[float] = []
        self.widths: list[float] = []
        self.deltas: list[float] = []
        self.n = 0.0
        self.buf: list[float] = []

    def _invariant(self, r: float) -> float:
        m = math.inf
        n = self.n
        for q, e in self.targets:
            f = 2 * e * r / q if q * n <= r else 2 * e * (n - r) / (1 - q)
            if f < m:
                m = f
        return m

    def insert(self, v: float):
        self.buf.append(v)
        if len(self.buf) >= BUF_CAP:
            self.flush()

    def flush(self):
        if not self.buf:
            return
        self.buf.sort()
        vals, widths, deltas = self.vals, self.widths, self.deltas
        r = 0.0
        i = 0
        for v in self.buf:
            while i < len(vals) and vals[i] <= v:
                r += widths[i]
                i += 1
            delta = 0.0 if i == 0 or i == len(vals) else max(0.0, math.floor(self._invariant(r)) - 1)
            vals.insert(i, v)
            widths.insert(i, 1.0)
            deltas.insert(i, delta)
            self.n += 1
            r += 1
            i += 1
        self.buf = []
        self._compress()

    def _compress(self):
        vals, widths, deltas = self.vals, self.widths, self.deltas
        if len(vals) < 2:
            return
        xi = len(vals) - 1
        r = self.n - 1 - widths[xi]
        for i in range(len(vals) - 2, -1, -1):
            cw = widths[i]
            if cw + widths[xi] + deltas[xi] <= self._invariant(r):
                widths[xi] += cw
                del vals[i], widths[i], deltas[i]
                xi -= 1
            else:
                xi = i
            r -= cw

    def query(self, q: float) -> float:
        self.flush()
        if not self.vals:
            return math.nan
        t = math.ceil(q * self.n)
        t += math.ceil(self._invariant(t) / 2)
        r = 0.0
        prev = self.vals[0]
        pw = self.widths[0]
        for j in range(1, len(self.vals)):
            r += pw
            if r + self.widths[j] + self.deltas[j] > t:
                return prev
            prev, pw = self.vals[j], self.widths[j]
        return prev

    def reset(self):
        self.vals, self.widths, self.deltas, self.buf = [], [], [], []
        self.n = 0.0


try:
    from .._native import _quantile as _NATIVE
except ImportError:          # CPU checkouts without the native build: same algorithm in Python
    _NATIVE = None


class _NativeChild:
    __slots__ = ("_owner", "_s", "_qs")

    def __init__(self, owner: "QuantileSummary"):
        self._owner = owner
        self._qs = sorted(owner.objectives)
        self._s = _NATIVE.Summary(sorted(owner.objectives.items()), owner.max_age, owner.age_buckets, owner.clock())

    def observe(self, v: float):
        self._s.observe(float(v), self._owner.clock())

    def quantiles(self) -> dict[float, float]:
        return dict(zip(self._qs, self._s.quantiles(self._owner.clock())))

    @property
    def sum(self) -> float:
        return self._s.sum

    @property
    def count(self) -> int:
        return self._s.count

    def time(self):
        return _Timer(self)


class _Timer:
    __slots__ = ("child", "t0")

    def __init__(self, child):
        self.child = child

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.child.observe(time.perf_counter() - self.t0)


class _Child:
    __slots__ = ("_owner", "_streams", "_head", "_next_rotate", "sum", "count", "_lock")

    def __init__(self, owner: "QuantileSummary"):
        self._owner = owner
        self._streams = [TargetedStream(owner.objectives) for _ in range(owner.age_buckets)]
        self._head = 0
        self._next_rotate = owner.clock() + owner.max_age / owner.age_buckets
        self.sum = 0.0
        self.count = 0
        self._lock = threading.Lock()

    def _rotate(self, now: float):
        step = self._owner.max_age / self._owner.age_buckets
        while now >= self._next_rotate:
            self._streams[self._head].reset()
            self._head = (self._head + 1) % len(self._streams)
            self._next_rotate += step

    def observe(self, v: float):
        with self._lock:
            self._rotate(self._owner.clock())
            self.sum += v
            self.count += 1
            for s in self._streams:
                s.insert(v)

    def quantiles(self) -> dict[float, float]:
        with self._lock:
            self._rotate(self._owner.clock())
            head = self._streams[self._head]
            return {q: head.query(q) for q in sorted(self._owner.objectives)}

    def time(self):
        return _Timer(self)


class QuantileSummary:
    """Drop-in for the prometheus_client Summary surface the components use (`labels(...)`,
    `observe`, `time`), registered as a collector in a CollectorRegistry."""

    def __init__(self, name: str, documentation: str, labelnames=(), registry=None,
                 objectives: dict[float, float] | None = None, max_age: float = DEF_MAX_AGE,
                 age_buckets: int = DEF_AGE_BUCKETS, clock=time.monotonic, native: bool | None = None):
        self.name, self.documentation = name, documentation
        self.labelnames = tuple(labelnames)
        self.objectives = dict(DEF_OBJECTIVES if objectives is None else objectives)
        self.max_age, self.age_buckets, self.clock = float(max_age), int(age_buckets), clock
        self._children: dict[tuple, _Child] = {}
        self._lock = threading.Lock()
        use_native = _NATIVE is not None if native is None else native
        self._child_cls = _NativeChild if use_native else _Child
        if registry is not None:
            registry.register(self)

    def labels(self, *values, **kw) -> _Child:
        if kw:
            values = tuple(str(kw[n]) for n in self.labelnames)
        else:
            values = tuple(str(v) for v in values)
        if len(values) != len(self.labelnames):
            raise ValueError(f"{self.name}: expected labels {self.labelnames}, got {values}")
        with self._lock:
            ch = self._children.get(values)
            if ch is None:
                ch = self._children[values] = self._child_cls(self)
            return ch

    def clear(self):
        """Drop every child (prometheus Vec Reset)."""
        with self._lock:
            self._children.clear()

    def observe(self, v: float):
        if self.labelnames:
            raise ValueError(f"{self.name} has labels {self.labelnames}; use .labels(...)")
        self.labels().observe(v)

    def time(self):
        return self.labels().time()

    def describe(self):
        return [Metric(self.name, self.documentation, "summary")]

    def collect(self):
        fam = Metric(self.name, self.documentation, "summary")
        with self._lock:
            children = list(self._children.items())
        if not self.labelnames and not children:
            children = [((), self._child_cls(self))]
        for values, ch in children:
            lbl = dict(zip(self.labelnames, values))
            for q, v in ch.quantiles().items():
                fam.add_sample(self.name, {**lbl, "quantile": _fmt_q(q)}, v)
            fam.add_sample(self.name + "_sum", lbl, ch.sum)
            fam.add_sample(self.name + "_count", lbl, float(ch.count))
        return [fam]

    # read access for in-process consumers (bench, tests)
    def quantile(self, q: float, *values) -> float:
        return self.labels(*values).quantiles().get(q, math.nan)


def _fmt_q(q: float) -> str:
    return repr(float(q)).rstrip("0").rstrip(".") if q != int(q) else str(int(q))
