"""deploy/monitoring/* against a live scrape (BASELINE config 5).

Every metric name that a Grafana panel or a Prometheus alert in deploy/monitoring queries must be
exported by some component of a running cluster: the apiserver, the kubelet (/metrics and
/metrics/cadvisor), the scheduler and the amd-smi exporter. The reference's names are the
targets: pkg/kubelet/metrics/metrics.go:53-152 (Summaries with quantiles),
staging/src/k8s.io/apiserver/pkg/endpoints/metrics/metrics.go:37-70,
plugin/pkg/scheduler/metrics/metrics.go:34-50, cadvisor's container_accelerator_* series.
"""
from __future__ import annotations

import json
import os
import re

import aiohttp
import yaml
from prometheus_client.parser import text_string_to_metric_families

from amdkube.api import meta as m
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.monitoring.exporter import Exporter
from tests.conftest import run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MON = os.path.join(ROOT, "deploy", "monitoring")
PROMQL_WORDS = {"sum", "rate", "irate", "max", "min", "avg", "count", "by", "without", "histogram_quantile",
                "increase", "on", "ignoring", "and", "or", "unless", "delta", "deriv", "topk", "bottomk", "abs",
                "clamp_min", "clamp_max", "offset", "bool", "e"}


def promql_metrics(expr: str) -> set[str]:
    """Metric names referenced by a PromQL expression (selectors, ranges and grouping removed)."""
    e = re.sub(r"\{[^}]*\}", " ", expr)
    e = re.sub(r"\[[^\]]*\]", " ", e)
    e = re.sub(r"\b(by|without|on|ignoring)\s*\([^)]*\)", " ", e)
    e = re.sub(r'"[^"]*"', " ", e)
    e = re.sub(r"\b\d+(\.\d+)?([eE][+-]?\d+)?\b", " ", e)          # numbers (1e6)
    names = set(re.findall(r"[a-zA-Z_:][a-zA-Z0-9_:]*", e))
    return {n for n in names if n not in PROMQL_WORDS}


def manifest_queries() -> list[tuple[str, str]]:
    out = []
    dash = json.load(open(os.path.join(MON, "grafana-dashboard.json")))
    for p in dash["panels"]:
        for t in p.get("targets") or []:
            out.append((f"panel {p['title']!r}", t["expr"]))
    rules = yaml.safe_load(open(os.path.join(MON, "alerts.yml")))
    for g in rules["groups"]:
        for r in g["rules"]:
            out.append((f"alert {r['alert']}", str(r["expr"])))
    return out


def test_promql_name_extraction():
    assert promql_metrics('max(kubelet_pod_start_latency_microseconds{quantile="0.5"}) / 1e6') == \
        {"kubelet_pod_start_latency_microseconds"}
    assert promql_metrics('sum by (node, gpu) (rate(amd_gpu_xgmi_link_read_bytes_total{node=~"$node"}[1m]))') == \
        {"amd_gpu_xgmi_link_read_bytes_total"}


def test_every_dashboard_and_alert_metric_is_scraped():
    async def go():
        async with LocalCluster(gpus="fake", relist_period=0.2, scheduler_kw={"port": 0}) as lc:
            c = lc.client
            await lc.wait_gpus(8)
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "mon", "namespace": "default"},
                            "spec": {"restartPolicy": "Never", "containers": [{
                                "name": "c", "image": "busybox", "command": ["sh", "-c", "sleep 30"],
                                "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            pod = await wait_pod(c, "default", "mon", ("Running",), 30)
            assert m.name_of(pod) == "mon"
            kport = lc.kubelet.server.port
            ex = Exporter(lc.backend, node=lc.node_name, kubelet_url=f"http://127.0.0.1:{kport}")
            await ex.start("127.0.0.1", 0)
            bodies = {}
            try:
                async with aiohttp.ClientSession() as s:
                    for name, url in (("exporter", f"http://127.0.0.1:{ex.port}/metrics"),
                                      ("kubelet", f"http://127.0.0.1:{kport}/metrics"),
                                      ("cadvisor", f"http://127.0.0.1:{kport}/metrics/cadvisor"),
                                      ("scheduler", f"http://127.0.0.1:{lc.scheduler.port}/metrics")):
                        async with s.get(url) as r:
                            assert r.status == 200, (name, r.status)
                            bodies[name] = await r.text()
                bodies["apiserver"] = (await c.request("GET", "/metrics", raw=True)).decode()
            finally:
                await ex.stop()
            return bodies

    bodies = run(go(), 90)
    exported: set[str] = set()
    for text in bodies.values():
        for fam in text_string_to_metric_families(text):
            exported.add(fam.name)
            exported.update(s.name for s in fam.samples)
    missing = []
    for where, expr in manifest_queries():
        for name in promql_metrics(expr):
            if name not in exported:
                missing.append(f"{where}: {name}")
    assert not missing, "queried but never exported:\n  " + "\n  ".join(missing)
    # the Summary quantile series the dashboard's device-plugin and pod-startup panels read
    kub = bodies["kubelet"]
    assert re.search(r'kubelet_device_plugin_alloc_latency_microseconds\{resource_name="amd.com/gpu",quantile="0.5"\} [0-9.e+]+', kub), kub
    assert re.search(r'kubelet_pod_start_latency_microseconds\{quantile="0.99"\} [0-9.e+]+', kub)
    assert re.search(r'apiserver_request_latencies_summary\{verb="POST",resource="pods",subresource="",scope="namespace",quantile="0.99"\} [0-9.e+]+',
                     bodies["apiserver"])
    # counters carry the reference's (Go client) names, with no `_total`/`_created` series
    assert "apiserver_request_count{" in bodies["apiserver"] and "apiserver_request_count_total" not in bodies["apiserver"]
    assert "_created" not in bodies["apiserver"]


def test_api_responsiveness_reads_the_latency_summary():
    """metrics_util.go readLatencyMetrics/HighLatencyRequests over an exposition: events and
    WATCH/CONNECT are ignored, counts are summed over client/contentType/code, quantiles are
    microseconds, LIST limits rise to 5 s / 10 s only in clusters of more than 500 nodes."""
    from amdkube.benchmark import apiresp
    text = "\n".join([
        "# TYPE apiserver_request_latencies_summary summary",
        'apiserver_request_latencies_summary{verb="POST",resource="pods",subresource="",scope="namespace",quantile="0.5"} 1500',
        'apiserver_request_latencies_summary{verb="POST",resource="pods",subresource="",scope="namespace",quantile="0.99"} 1.2e+06',
        'apiserver_request_latencies_summary{verb="LIST",resource="nodes",subresource="",scope="cluster",quantile="0.99"} 7e+06',
        'apiserver_request_latencies_summary{verb="WATCH",resource="pods",subresource="",scope="cluster",quantile="0.99"} 9e+09',
        'apiserver_request_latencies_summary{verb="POST",resource="events",subresource="",scope="namespace",quantile="0.99"} 9e+09',
        "# TYPE apiserver_request_count counter",
        'apiserver_request_count{verb="POST",resource="pods",subresource="",scope="namespace",client="a",contentType="application/json",code="201"} 3',
        'apiserver_request_count{verb="POST",resource="pods",subresource="",scope="namespace",client="b",contentType="application/json",code="409"} 2',
        'apiserver_request_count{verb="LIST",resource="nodes",subresource="",scope="cluster",client="a",contentType="application/json",code="200"} 1',
        ""])
    calls = apiresp.parse_latency_metrics(text)
    assert {(c.verb, c.resource) for c in calls} == {("POST", "pods"), ("LIST", "nodes")}
    post = [c for c in calls if c.verb == "POST"][0]
    assert post.count == 5 and post.perc50_s == 0.0015 and post.perc99_s == 1.2
    bad, _ = apiresp.high_latency_requests(calls, node_count=100)
    assert bad == 2                          # POST over 1 s; LIST over 1 s in a small cluster
    bad, _ = apiresp.high_latency_requests(calls, node_count=600)
    assert bad == 1                          # LIST cluster-scope limit 10 s in a big cluster
    s = apiresp.summarize(calls)
    assert s["api_p99_ms"] == 1200.0 and s["api_list_p99_ms"] == 7000.0
