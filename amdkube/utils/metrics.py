"""Per-component Prometheus registries and the reference's exposition names.

Every component owns a CollectorRegistry so several components can live in one test
process without metric-name collisions; `/metrics` handlers render their own registry.
Metric names follow the reference.

`render` writes the text format the reference's Go client (client_golang 0.8, vendored by
the reference) writes: a counter is exported under its declared name (`apiserver_request_count`,
not prometheus_client's OpenMetrics-style `apiserver_request_count_total`), and no `_created`
series are emitted. Those are the names the e2e framework, dashboards and alerts query
(test/e2e/framework/metrics_util.go:330-331).
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, Summary  # noqa: F401
from prometheus_client.utils import floatToGoString

CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"

# exponential buckets in microseconds (1ms .. ~16s), like the reference's ExponentialBuckets(1000, 2, 15)
MICRO_BUCKETS = tuple(1000 * 2 ** i for i in range(15))


def new_registry() -> CollectorRegistry:
    return CollectorRegistry(auto_describe=True)


def _esc_help(s: str) -> str:
    return s.replace("\\", r"\\").replace("\n", r"\n")


def _esc_label(s: str) -> str:
    return s.replace("\\", r"\\").replace("\n", r"\n").replace('"', r'\"')


def render(registry: CollectorRegistry) -> bytes:
    out: list[str] = []
    for fam in registry.collect():
        name, typ = fam.name, fam.type
        samples = [s for s in fam.samples if not s.name.endswith("_created")]
        if typ == "counter":
            # prometheus_client strips a declared `_total` and re-adds it to the sample; the Go
            # client exports the declared name as is
            samples = [s._replace(name=name) if s.name == name + "_total" else s for s in samples]
        elif typ in ("unknown", "info", "stateset", "gaugehistogram"):
            typ = "untyped" if typ == "unknown" else "gauge"
        out.append(f"# HELP {name} {_esc_help(fam.documentation)}")
        out.append(f"# TYPE {name} {typ}")
        for s in samples:
            if s.labels:
                lab = ",".join(f'{k}="{_esc_label(str(v))}"' for k, v in s.labels.items())
                out.append(f"{s.name}{{{lab}}} {floatToGoString(s.value)}")
            else:
                out.append(f"{s.name} {floatToGoString(s.value)}")
    return ("\n".join(out) + "\n").encode() if out else b""
