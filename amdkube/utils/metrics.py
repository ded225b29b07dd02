"""Per-component Prometheus registries.

Every component owns a CollectorRegistry so several components can live in one test
process without metric-name collisions; `/metrics` handlers render their own registry.
Metric names follow the reference.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, Summary, generate_latest  # noqa: F401

CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"

# exponential buckets in microseconds (1ms .. ~16s), like the reference's ExponentialBuckets(1000, 2, 15)
MICRO_BUCKETS = tuple(1000 * 2 ** i for i in range(15))


def new_registry() -> CollectorRegistry:
    return CollectorRegistry(auto_describe=True)


def render(registry: CollectorRegistry) -> bytes:
    return generate_latest(registry)
