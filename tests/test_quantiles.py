"""Prometheus Summary quantiles (amdkube.utils.quantiles, native/quantile_core.h).

Parity target: prometheus/client_golang summary.go as linked by the reference (DefObjectives
0.5/0.05, 0.9/0.01, 0.99/0.001; DefMaxAge 10 min over 5 age buckets; exposition
`name{quantile="0.5"}` plus `_sum`/`_count`), the shape pkg/kubelet/metrics/metrics.go:53-152 and
staging/src/k8s.io/apiserver/pkg/endpoints/metrics/metrics.go:55-70 export.
"""
from __future__ import annotations

import bisect
import math
import os
import random
import subprocess

import pytest
from prometheus_client.parser import text_string_to_metric_families

from amdkube.utils import quantiles as Q
from amdkube.utils.metrics import new_registry, render

BOTH = [False] + ([True] if Q._NATIVE is not None else [])


@pytest.mark.parametrize("native", BOTH)
def test_rank_error_within_objectives(native):
    s = Q.QuantileSummary("lat_us", "h", registry=None, native=native)
    rnd = random.Random(3)
    xs = [rnd.lognormvariate(8, 1.5) for _ in range(60000)]
    for x in xs:
        s.observe(x)
    xs.sort()
    for q, eps in Q.DEF_OBJECTIVES.items():
        v = s.quantile(q)
        rank = bisect.bisect_left(xs, v) / len(xs)
        assert abs(rank - q) <= eps, (q, rank)


def test_native_and_python_streams_agree():
    if Q._NATIVE is None:
        pytest.skip("native _quantile not built")
    a = Q.QuantileSummary("a", "h", native=True)
    b = Q.QuantileSummary("b", "h", native=False)
    rnd = random.Random(5)
    for _ in range(12345):
        x = rnd.random() * 1e6
        a.observe(x)
        b.observe(x)
    assert a.labels().quantiles() == b.labels().quantiles()
    assert a.labels().count == b.labels().count == 12345


@pytest.mark.parametrize("native", BOTH)
def test_window_forgets_after_max_age(native):
    now = [0.0]
    s = Q.QuantileSummary("w", "h", ["op"], clock=lambda: now[0], native=native)
    for _ in range(1000):
        s.labels("x").observe(5.0)
    now[0] = 300.0                                   # half the window: old samples still count
    assert s.quantile(0.5, "x") == 5.0
    for _ in range(10):
        s.labels("x").observe(9.0)
    now[0] = 601.0                                   # the 5.0s are older than max_age now
    assert s.quantile(0.5, "x") == 9.0
    now[0] = 2000.0                                  # nothing observed in the last 10 minutes
    assert math.isnan(s.quantile(0.5, "x"))
    assert s.labels("x").count == 1010               # _count and _sum stay cumulative


def test_exposition_matches_go_client_shape():
    r = new_registry()
    s = Q.QuantileSummary("kubelet_device_plugin_alloc_latency_microseconds", "h", ["resource_name"], registry=r)
    for v in (10, 20, 30):
        s.labels("amd.com/gpu").observe(v)
    text = render(r).decode()
    # (three samples: the targeted query's rank slack lands every quantile on 30, as in Go)
    assert 'kubelet_device_plugin_alloc_latency_microseconds{resource_name="amd.com/gpu",quantile="0.5"} 30.0' in text
    fams = {f.name: f for f in text_string_to_metric_families(text)}
    fam = fams["kubelet_device_plugin_alloc_latency_microseconds"]
    assert fam.type == "summary"
    qs = sorted(smp.labels["quantile"] for smp in fam.samples if "quantile" in smp.labels)
    assert qs == ["0.5", "0.9", "0.99"]
    assert any(smp.name.endswith("_count") and smp.value == 3 for smp in fam.samples)
    # an unlabelled summary with no observations still exports NaN quantiles and zero count
    r2 = new_registry()
    Q.QuantileSummary("kubelet_pod_start_latency_microseconds", "h", registry=r2)
    assert 'kubelet_pod_start_latency_microseconds{quantile="0.99"} NaN' in render(r2).decode()


def test_native_selftest_under_asan():
    exe = os.path.join(os.path.dirname(Q.__file__), "..", "_native", "bin", "quantile-selftest-asan")
    if not os.path.exists(exe):
        pytest.skip("sanitizer build not present (python native/build.py --sanitize)")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "OK" in out.stdout, out.stdout + out.stderr
