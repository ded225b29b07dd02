"""API responsiveness as the reference's e2e framework measures it.

Reference: test/e2e/framework/metrics_util.go
  * ResetMetrics (:423-431): DELETE /metrics on the apiserver before the measured phase;
  * readLatencyMetrics (:309-358): scrape /metrics, keep `apiserver_request_latencies_summary`
    quantile samples (microseconds) and `apiserver_request_count`, ignoring resource `events`
    and verbs WATCH/WATCHLIST/PROXY/proxy/CONNECT, grouped by (resource, subresource, verb, scope);
  * HighLatencyRequests (:363-398): a call is bad when its p99 exceeds 1 s
    (apiCallLatencyThreshold, :52); LISTs in a cluster of more than 500 nodes get 5 s, or 10 s when
    cluster-scoped (:57-59).
"""
from __future__ import annotations

from dataclasses import dataclass, field

from prometheus_client.parser import text_string_to_metric_families

API_CALL_LATENCY_THRESHOLD_S = 1.0
API_LIST_CALL_LATENCY_THRESHOLD_S = 5.0
API_CLUSTER_SCOPE_LIST_CALL_THRESHOLD_S = 10.0
BIG_CLUSTER_NODE_COUNT_THRESHOLD = 500
IGNORED_RESOURCES = {"events"}
IGNORED_VERBS = {"WATCH", "WATCHLIST", "PROXY", "proxy", "CONNECT"}


@dataclass
class APICall:
    resource: str
    subresource: str
    verb: str
    scope: str
    perc50_s: float = 0.0
    perc90_s: float = 0.0
    perc99_s: float = 0.0
    count: int = 0
    bad: bool = field(default=False)

    def as_dict(self) -> dict:
        return {"resource": self.resource, "subresource": self.subresource, "verb": self.verb, "scope": self.scope,
                "count": self.count, "p50_ms": round(self.perc50_s * 1e3, 3), "p90_ms": round(self.perc90_s * 1e3, 3),
                "p99_ms": round(self.perc99_s * 1e3, 3)}


def parse_latency_metrics(text: str) -> list[APICall]:
    """readLatencyMetrics over one /metrics body."""
    calls: dict[tuple, APICall] = {}

    def call(lb) -> APICall | None:
        res, verb = lb.get("resource", ""), lb.get("verb", "")
        if res in IGNORED_RESOURCES or verb in IGNORED_VERBS:
            return None
        key = (res, lb.get("subresource", ""), verb, lb.get("scope", ""))
        c = calls.get(key)
        if c is None:
            c = calls[key] = APICall(*key)
        return c

    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            if s.name == "apiserver_request_latencies_summary" and "quantile" in s.labels:
                c = call(s.labels)
                if c is None or s.value != s.value:        # NaN: no observation in the window
                    continue
                # time.Duration(int64(latency)) * time.Microsecond
                lat = int(s.value) * 1e-6
                q = float(s.labels["quantile"])
                if q == 0.5:
                    c.perc50_s = lat
                elif q == 0.9:
                    c.perc90_s = lat
                elif q == 0.99:
                    c.perc99_s = lat
            elif s.name in ("apiserver_request_count", "apiserver_request_count_total"):
                c = call(s.labels)
                if c is not None:
                    c.count += int(s.value)
    return list(calls.values())


def high_latency_requests(calls: list[APICall], node_count: int) -> tuple[int, list[APICall]]:
    """(number of bad calls, calls sorted by p99 descending with `bad` set)."""
    big = node_count > BIG_CLUSTER_NODE_COUNT_THRESHOLD
    bad = 0
    for c in calls:
        limit = API_CALL_LATENCY_THRESHOLD_S
        if c.verb == "LIST" and big:
            limit = API_CLUSTER_SCOPE_LIST_CALL_THRESHOLD_S if c.scope == "cluster" else API_LIST_CALL_LATENCY_THRESHOLD_S
        c.bad = c.perc99_s > limit
        bad += c.bad
    return bad, sorted(calls, key=lambda c: -c.perc99_s)


async def reset_metrics(client):
    """ResetMetrics: DELETE /metrics."""
    await client.request("DELETE", "/metrics", raw=True)


async def read_latency_metrics(client) -> list[APICall]:
    body = await client.request("GET", "/metrics", raw=True)
    return parse_latency_metrics(body.decode())


def summarize(calls: list[APICall], node_count: int = 1) -> dict:
    """The density report's API fields: worst non-LIST p99, worst LIST p99, bad-call count."""
    bad, ordered = high_latency_requests(calls, node_count)
    nonlist = [c for c in ordered if c.verb != "LIST" and c.count]
    lists = [c for c in ordered if c.verb == "LIST" and c.count]
    return {"api_p99_ms": round(nonlist[0].perc99_s * 1e3, 3) if nonlist else None,
            "api_list_p99_ms": round(lists[0].perc99_s * 1e3, 3) if lists else None,
            "api_bad_calls": bad, "calls": sum(c.count for c in ordered),
            "worst": [c.as_dict() for c in ordered[:5]], "source": "apiserver_request_latencies_summary"}
