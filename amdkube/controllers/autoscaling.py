"""HorizontalPodAutoscaler controller, with a GPU-utilization target for MI355X workloads.

Reference: pkg/controller/podautoscaler/horizontal.go + replica_calculator.go (1.9,
autoscaling/v1): every --horizontal-pod-autoscaler-sync-period (30 s) read the target's
scale; utilization = Σ usage / Σ requests over the target's ready pods that report
metrics; usageRatio = utilization / target; inside the 10 % tolerance nothing changes,
else desired = ceil(usageRatio × pods-with-metrics). Pods without metrics count as at target
on a scale-down and idle on a scale-up, unready pods as idle on a scale-up, and a rebalanced
ratio that flips direction keeps the count (replica_calculator.go, integer milli-units); clamp to [minReplicas, maxReplicas]
and to the scale-up limit max(2 × current, 4); a scale-up needs 3 min and a scale-down 5 min
since the last rescale (--horizontal-pod-autoscaler-{upscale,downscale}-delay); status
carries currentReplicas / desiredReplicas / currentCPUUtilizationPercentage / lastScaleTime.

autoscaling/v2beta1 (horizontal.go computeReplicasForMetrics, 1.9): spec.metrics may list
Resource (cpu/memory, targetAverageUtilization or targetAverageValue), Pods (a per-pod custom
metric averaged over the target's pods, targetAverageValue) and Object (one custom metric of
another object, targetValue) sources; each proposes a replica count and the largest wins. The
v1 storage object carries the extra metrics, currentMetrics and the AbleToScale /
ScalingActive / ScalingLimited conditions in annotations (api/autoscaling.py); the controller
writes status through the v2beta1 status subresource.

MI355X extensions: the custom metrics API of `amdkube metrics-server` serves gpu_utilization /
gpu_memory_used_bytes / gpu_count per pod, so a Pods metric on gpu_utilization scales on MI355X
activity. The older annotation `autoscaling.amd.com/target-gpu-utilization: "<pct>"` adds the
same signal read from the resource metrics source, without the custom metrics API.

Resource metrics come from the resource metrics API (metrics.k8s.io, the metrics-server) when it
is registered, else straight from the kubelets' /stats/summary, where CPU usage is the rate
between two successive cumulative samples.
"""
from __future__ import annotations

import asyncio
import json
import math
import time

import aiohttp

from ..api import autoscaling as api_autoscaling
from ..api import meta as m
from ..api.helpers import is_pod_ready
from ..api.labels import selector_from_label_selector, selector_from_set
from ..api.quantity import Quantity
from .base import Controller, split_key

GPU_TARGET_ANNOTATION = "autoscaling.amd.com/target-gpu-utilization"
TOLERANCE = 0.1
SCALE_TARGETS = {"Deployment": "deployments", "ReplicaSet": "replicasets", "ReplicationController": "replicationcontrollers",
                 "StatefulSet": "statefulsets"}


class KubeletSummaryMetrics:
    """Pod CPU (millicores) and GPU activity (%) from every node's kubelet /stats/summary."""

    def __init__(self, client):
        self.client = client
        self._prev: dict[tuple, tuple[float, int]] = {}
        self._http: aiohttp.ClientSession | None = None

    async def pod_metrics(self, ns: str) -> dict[str, dict]:
        if self._http is None:
            self._http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5))
        out: dict[str, dict] = {}
        nodes, _ = await self.client.list("nodes")
        for node in nodes:
            st = node.get("status") or {}
            port = ((st.get("daemonEndpoints") or {}).get("kubeletEndpoint") or {}).get("Port")
            addr = next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "InternalIP"), None)
            if not port or not addr:
                continue
            try:
                async with self._http.get(f"http://{addr}:{port}/stats/summary") as r:
                    summary = await r.json()
            except (aiohttp.ClientError, asyncio.TimeoutError, ValueError):
                continue
            now = time.time()
            for p in summary.get("pods") or []:
                ref = p.get("podRef") or {}
                if ref.get("namespace") != ns:
                    continue
                cpu_milli, gpu, ngpu, mem = 0.0, 0.0, 0, 0
                have_cpu = True
                for c in p.get("containers") or []:
                    key = (ref.get("uid"), c.get("name"))
                    cur = int(((c.get("cpu") or {}).get("usageCoreNanoSeconds")) or 0)
                    prev = self._prev.get(key)
                    self._prev[key] = (now, cur)
                    if prev is None or now <= prev[0]:
                        have_cpu = False
                    else:
                        cpu_milli += max(0, cur - prev[1]) / (now - prev[0]) / 1e6
                    mem += int(((c.get("memory") or {}).get("workingSetBytes")) or 0)
                    for a in c.get("accelerators") or []:
                        gpu += float(a.get("dutyCycle", 0))
                        ngpu += 1
                ent = {}
                if have_cpu:
                    ent["cpu_milli"] = cpu_milli
                if ngpu:
                    ent["gpu_util"] = gpu / ngpu
                if mem:
                    ent["memory_bytes"] = mem
                out[ref.get("name")] = ent
        return out

    async def close(self):
        if self._http:
            await self._http.close()


class ResourceMetricsAPI:
    """metrics/rest_metrics_client.go resourceMetricsClient: pod CPU from the resource metrics API
    (metrics.k8s.io/v1beta1 PodMetrics, served by the metrics-server behind the aggregator) — the
    reference 1.9 default (--horizontal-pod-autoscaler-use-rest-clients). GPU activity rides in
    the metrics-server's amd.com/gpu-duty-cycle annotation. When the group is not served (no
    metrics-server registered) the kubelet-summary source answers instead."""

    def __init__(self, client, fallback=None):
        self.client = client
        self.fallback = fallback or KubeletSummaryMetrics(client)

    async def _served(self) -> bool:
        try:
            groups = (await self.client.request("GET", "/apis")).get("groups") or []
        except Exception:
            return False
        return any(g.get("name") == "metrics.k8s.io" for g in groups)

    async def pod_metrics(self, ns: str) -> dict[str, dict]:
        if not await self._served():
            return await self.fallback.pod_metrics(ns)
        try:
            items = (await self.client.request("GET", f"/apis/metrics.k8s.io/v1beta1/namespaces/{ns}/pods")).get("items") or []
        except Exception:
            return await self.fallback.pod_metrics(ns)
        out = {}
        for pm in items:
            cts = pm.get("containers") or []
            ent = {"cpu_milli": float(sum(Quantity(ct["usage"]["cpu"]).as_fraction() * 1000 for ct in cts))}
            if any("memory" in ct.get("usage", {}) for ct in cts):
                ent["memory_bytes"] = int(sum(Quantity(ct["usage"].get("memory", "0")).value() for ct in cts))
            duty = ((pm.get("metadata") or {}).get("annotations") or {}).get("amd.com/gpu-duty-cycle")
            if duty is not None:
                ent["gpu_util"] = float(duty)
            out[m.name_of(pm)] = ent
        return out

    async def close(self):
        await self.fallback.close()


class CustomMetricsAPI:
    """metrics/rest_metrics_client.go customMetricsClient: Pods and Object metrics from the custom
    metrics API (custom.metrics.k8s.io/v1beta1, behind the aggregator; `amdkube metrics-server`
    serves gpu_utilization / gpu_memory_used_bytes / gpu_count)."""

    def __init__(self, client):
        self.client = client

    async def pod_metric(self, ns: str, metric: str, selector: str) -> dict[str, float]:
        d = await self.client.request("GET", f"/apis/{CMG}/namespaces/{_seg(ns)}/pods/*/{_seg(metric)}",
                                      params={"labelSelector": selector} if selector else None)
        return {(it.get("describedObject") or {}).get("name"): _num(it.get("value"))
                for it in (d or {}).get("items") or []}

    async def object_metric(self, ns: str, target: dict, metric: str) -> float:
        plural = OBJECT_PLURALS.get(target.get("kind"), (target.get("kind") or "").lower() + "s")
        # every segment comes from the HPA's spec: quoted so none can step out of the metrics API
        d = await self.client.request("GET", f"/apis/{CMG}/namespaces/{_seg(ns)}/{_seg(plural)}/{_seg(target.get('name') or '')}/"
                                             f"{_seg(metric)}")
        items = (d or {}).get("items") or []
        if not items:
            raise LookupError(f"no value for {metric} of {target.get('kind')}/{target.get('name')}")
        return _num(items[0].get("value"))


CMG = "custom.metrics.k8s.io/v1beta1"


def _seg(v: str) -> str:
    """One URL path segment: '/', '..' and the like cannot change the request's path."""
    from urllib.parse import quote
    v = str(v)
    if v in ("", ".", ".."):
        raise LookupError(f"invalid metric path segment {v!r}")
    return quote(v, safe="")
OBJECT_PLURALS = {"Pod": "pods", "Service": "services", "Deployment": "deployments", "Node": "nodes",
                  "Ingress": "ingresses", "ReplicaSet": "replicasets", "StatefulSet": "statefulsets"}


def _num(q) -> float:
    return float(Quantity(str(q)).as_fraction()) if q is not None else 0.0


def _fmt(v: float) -> str:
    """A float as the canonical quantity string the reference writes (milli-units below 1000 × int)."""
    return _fmt_milli(int(round(v * 1000)))


def _fmt_milli(mv: int) -> str:
    """resource.NewMilliQuantity(mv, DecimalSI).String() for the values the controller writes."""
    return str(mv // 1000) if mv % 1000 == 0 else f"{mv}m"


_USAGE_KEY = {"cpu": "cpu_milli", "memory": "memory_bytes"}


def _ratio_replicas(ratio: float, n: int, current: int) -> int:
    return current if abs(ratio - 1.0) <= TOLERANCE else int(math.ceil(ratio * n))


# ---- replica calculator (replica_calculator.go, metrics/utilization.go), in integer milli-units
def resource_utilization_ratio(metrics: dict, requests: dict, target: int) -> tuple[float, int, int]:
    """GetResourceUtilizationRatio: metrics of pods with no known request are extraneous; the
    utilization is an integer percentage and the raw average an integer milli-value."""
    total = req = n = 0
    for name, v in metrics.items():
        if name not in requests:
            continue
        total, req, n = total + v, req + requests[name], n + 1
    if req == 0:
        raise LookupError("no metrics returned matched known pods")
    util = total * 100 // req
    return util / target, util, total // n


def metric_utilization_ratio(metrics: dict, target: int) -> tuple[float, int]:
    """GetMetricUtilizationRatio: every metric counts, superfluous ones included."""
    util = sum(metrics.values()) // len(metrics)
    return util / target, util


def _classify(pods, metrics) -> tuple[int, set, set]:
    """Pods not Running-and-Ready are unready (their metrics dropped); ready pods without a metric
    are missing; the rest count."""
    ready, unready, missing = 0, set(), set()
    for p in pods:
        name = m.name_of(p)
        if (p.get("status") or {}).get("phase") != "Running" or not is_pod_ready(p):
            unready.add(name)
            metrics.pop(name, None)
        elif name not in metrics:
            missing.add(name)
        else:
            ready += 1
    return ready, unready, missing


def _replicas_from(current, ratio, ready, unready, missing, metrics, missing_down, zero_missing_at_one, recompute,
                   tolerance=TOLERANCE) -> int:
    """The shared tail of GetResourceReplicas and calcPlainMetricReplicas: with no unready pods on a
    scale-up and nothing missing, ceil(ratio × ready pods) outside the tolerance. Otherwise missing
    pods count as at target on a scale-down and idle on a scale-up, unready pods as idle on a
    scale-up, and a recomputed ratio that falls inside the tolerance or flips direction keeps the
    current count."""
    rebalance = bool(unready) and ratio > 1.0
    if not rebalance and not missing:
        return current if abs(1.0 - ratio) <= tolerance else int(math.ceil(ratio * ready))
    if missing:
        if ratio < 1.0:
            for name in missing:
                metrics[name] = missing_down(name)
        elif ratio > 1.0 or zero_missing_at_one:
            for name in missing:
                metrics[name] = 0
    if rebalance:
        for name in unready:
            metrics[name] = 0
    new = recompute(metrics)
    if abs(1.0 - new) <= tolerance or (ratio < 1.0 < new) or (ratio > 1.0 > new):
        return current
    return int(math.ceil(new * len(metrics)))


def get_resource_replicas(current: int, target_util: int, resource: str, pods, metrics: dict, ns: str = "",
                          tolerance: float = TOLERANCE) -> tuple[int, int, int]:
    """GetResourceReplicas: (replicas, utilization %, raw average milli-value). `metrics` maps pod
    name → Σ container usage in milli-units; every container of every pod needs a request."""
    if not metrics:
        raise LookupError(f"unable to get metrics for resource {resource}: no metrics returned from heapster")
    if not pods:
        raise LookupError("no pods returned by selector while calculating replica count")
    metrics, requests = dict(metrics), {}
    for p in pods:
        total = 0
        for c in (p.get("spec") or {}).get("containers") or []:
            q = ((c.get("resources") or {}).get("requests") or {}).get(resource)
            if q is None:
                raise LookupError(f"missing request for {resource} on container {c.get('name', '')} in pod {ns}/{m.name_of(p)}")
            total += Quantity(str(q)).milli_value()
        requests[m.name_of(p)] = total
    ready, unready, missing = _classify(pods, metrics)
    if not metrics:
        raise LookupError("did not receive metrics for any ready pods")
    ratio, util, raw = resource_utilization_ratio(metrics, requests, target_util)
    rep = _replicas_from(current, ratio, ready, unready, missing, metrics, requests.__getitem__, False,
                         lambda mt: resource_utilization_ratio(mt, requests, target_util)[0], tolerance)
    return rep, util, raw


def get_plain_metric_replicas(current: int, target: int, pods, metrics: dict, tolerance: float = TOLERANCE) -> tuple[int, int]:
    """calcPlainMetricReplicas (GetRawResourceReplicas / GetMetricReplicas): (replicas, average
    milli-value) against a per-pod target milli-value."""
    if not pods:
        raise LookupError("no pods returned by selector while calculating replica count")
    metrics = dict(metrics)
    ready, unready, missing = _classify(pods, metrics)
    if not metrics:
        raise LookupError("did not receive metrics for any ready pods")
    ratio, util = metric_utilization_ratio(metrics, target)
    rep = _replicas_from(current, ratio, ready, unready, missing, metrics, lambda _: target, True,
                         lambda mt: metric_utilization_ratio(mt, target)[0], tolerance)
    return rep, util


def get_object_metric_replicas(current: int, target: int, value: int, tolerance: float = TOLERANCE) -> int:
    """GetObjectMetricReplicas: one object's milli-value against the target, scaled over the
    current replica count."""
    ratio = value / target
    return current if abs(1.0 - ratio) <= tolerance else int(math.ceil(ratio * current))


def _milli(v) -> int:
    """A metric source's base-unit float as the integer milli-value the calculator works in."""
    return int(round(v * 1000))


def resource_metrics_milli(raw: dict, resource: str) -> dict:
    """Pod → Σ usage in milli-units from a resource metrics source (cpu_milli is already milli)."""
    key = _USAGE_KEY.get(resource)
    if key is None:
        return {}
    return {name: int(round(mt[key])) if resource == "cpu" else int(mt[key]) * 1000
            for name, mt in raw.items() if key in mt}


def gpu_proposal(pods, metrics, target_pct, current) -> tuple[int | None, float | None]:
    vals = [(metrics.get(m.name_of(p)) or {}).get("gpu_util") for p in pods]
    vals = [v for v in vals if v is not None]
    if not vals:
        return None, None
    util = sum(vals) / len(vals)
    return _ratio_replicas(util / float(target_pct), len(vals), current), util


def _set_condition(conds: list, typ: str, status: str, reason: str, message: str, now: str):
    """horizontal.go setCondition: lastTransitionTime moves only when the status flips."""
    for c in conds:
        if c.get("type") == typ:
            if c.get("status") != status:
                c["lastTransitionTime"] = now
            c.update(status=status, reason=reason, message=message)
            return
    conds.append({"type": typ, "status": status, "lastTransitionTime": now, "reason": reason, "message": message})


class HorizontalPodAutoscalerController(Controller):
    """horizontal.go reconcileAutoscaler over the autoscaling/v2beta1 metric list (read from the
    stored v1 object's annotations, api/autoscaling.py): every metric proposes a replica count,
    the largest wins (computeReplicasForMetrics); status gets currentMetrics and the
    AbleToScale / ScalingActive / ScalingLimited conditions, written through the v2beta1
    status subresource so the apiserver folds them back into the v1 annotations."""
    name = "horizontalpodautoscaling"
    workers = 1

    def __init__(self, mgr, metrics=None, sync_period: float = 30.0, upscale_delay: float = 180.0,
                 downscale_delay: float = 300.0, clock=time.time):
        super().__init__(mgr)
        self.metrics = metrics or ResourceMetricsAPI(mgr.client)
        self.custom = self.metrics if hasattr(self.metrics, "pod_metric") else CustomMetricsAPI(mgr.client)
        self.sync_period, self.upscale_delay, self.downscale_delay = sync_period, upscale_delay, downscale_delay
        self.clock = clock
        self._poll = None

    def setup(self):
        self.hpa_inf = self.mgr.factory.informer("horizontalpodautoscalers")
        self.pod_inf = self.mgr.pods
        self.hpa_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))

    async def start(self):
        await super().start()
        self._poll = asyncio.create_task(self._loop(), name="hpa-poll")

    async def stop(self):
        if self._poll:
            self._poll.cancel()
        if hasattr(self.metrics, "close"):
            await self.metrics.close()
        await super().stop()

    async def _loop(self):
        while True:
            await asyncio.sleep(self.sync_period)
            for h in self.hpa_inf.list():
                self.enqueue(h)

    def _event(self, hpa, typ, reason, msg):
        rec = getattr(self.mgr, "recorder", None)
        if rec is not None:
            rec.event(hpa, typ, reason, msg)

    async def _metric_proposals(self, hpa, ns, pods, selector_str, current):
        """computeReplicasForMetrics: [(replicas, metric name, status entry)] plus the first
        failure (reason, message) if any metric could not be read."""
        specs = api_autoscaling.metrics_of(hpa)
        ann = m.annotations_of(hpa)
        explicit_cpu = (hpa.get("spec") or {}).get("targetCPUUtilizationPercentage") is not None
        if GPU_TARGET_ANNOTATION in ann and not explicit_cpu and api_autoscaling.METRICS_ANNOTATION not in ann:
            specs = []      # the GPU annotation alone replaces the defaulted 80 % CPU target
        out, failure, resource_metrics = [], None, None
        for ms in specs:
            typ = ms.get("type")
            try:
                if typ == "Resource":
                    if resource_metrics is None:
                        resource_metrics = await self.metrics.pod_metrics(ns)
                    r = ms.get("resource") or {}
                    rname = r.get("name")
                    tu, tv = r.get("targetAverageUtilization"), r.get("targetAverageValue")
                    # the metrics API is asked with the target's selector: metrics of other pods never arrive
                    names = {m.name_of(p) for p in pods}
                    mt = {k: v for k, v in resource_metrics_milli(resource_metrics, rname).items() if k in names}
                    if tu is not None:
                        rep, util, raw = get_resource_replicas(current, int(tu), rname, pods, mt, ns)
                        cur = {"name": rname, "currentAverageUtilization": util, "currentAverageValue": _fmt_milli(raw)}
                    else:
                        if not mt:
                            raise LookupError(f"unable to get metrics for resource {rname}: no metrics returned from heapster")
                        rep, raw = get_plain_metric_replicas(current, Quantity(str(tv)).milli_value(), pods, mt)
                        cur = {"name": rname, "currentAverageValue": _fmt_milli(raw)}
                    out.append((rep, f"{rname} resource" + (" utilization (percentage of request)" if tu is not None else ""),
                                {"type": "Resource", "resource": cur}))
                elif typ == "Pods":
                    pm = ms.get("pods") or {}
                    vals = await self.custom.pod_metric(ns, pm.get("metricName"), selector_str)
                    if not vals:
                        raise LookupError(f"unable to get metric {pm.get('metricName')}: no metrics returned from custom metrics API")
                    rep, avg = get_plain_metric_replicas(current, Quantity(str(pm.get("targetAverageValue"))).milli_value(), pods,
                                                         {k: _milli(v) for k, v in vals.items()})
                    out.append((rep, f"pods metric {pm.get('metricName')}",
                                {"type": "Pods", "pods": {"metricName": pm.get("metricName"), "currentAverageValue": _fmt_milli(avg)}}))
                elif typ == "Object":
                    om = ms.get("object") or {}
                    val = _milli(await self.custom.object_metric(ns, om.get("target") or {}, om.get("metricName")))
                    rep = get_object_metric_replicas(current, Quantity(str(om.get("targetValue"))).milli_value(), val)
                    out.append((rep, f"{om.get('metricName')} metric on {(om.get('target') or {}).get('kind')}",
                                {"type": "Object", "object": {"target": om.get("target"), "metricName": om.get("metricName"),
                                                              "currentValue": _fmt_milli(val)}}))
                else:
                    raise LookupError(f"unknown metric source type {typ!r}")
            except (LookupError, m.StatusError, aiohttp.ClientError, asyncio.TimeoutError, ZeroDivisionError, ValueError) as e:
                if failure is None:
                    failure = (f"FailedGet{typ}Metric", f"the HPA was unable to compute the replica count: {e}")
        gt = ann.get(GPU_TARGET_ANNOTATION)
        gpu_util = None
        if gt:
            if resource_metrics is None:
                resource_metrics = await self.metrics.pod_metrics(ns)
            rep, gpu_util = gpu_proposal(pods, resource_metrics, float(gt), current)
            if rep is not None:
                out.append((rep, "MI355X gpu utilization", None))
        return out, failure, gpu_util

    async def sync(self, key):
        hpa = self.hpa_inf.get(key)
        if hpa is None:
            return
        ns, name = split_key(key)
        spec, st = hpa.get("spec") or {}, hpa.get("status") or {}
        ann = m.annotations_of(hpa)
        conds = api_autoscaling._load(ann.get(api_autoscaling.CONDITIONS_ANNOTATION))
        now = self.clock()
        stamp = m.format_time(now)
        ref = spec.get("scaleTargetRef") or {}
        plural = SCALE_TARGETS.get(ref.get("kind"))
        target = await self.client.get_or_none(plural, ref.get("name", ""), ns) if plural else None
        if target is None:
            _set_condition(conds, "AbleToScale", "False", "FailedGetScale",
                           f"the HPA controller was unable to get the target's current scale: {ref.get('kind')}/{ref.get('name')}", stamp)
            self._event(hpa, "Warning", "FailedGetScale", f"unable to get the scale of {ref.get('kind')}/{ref.get('name')}")
            await self._write_status(hpa, ns, name, {"currentReplicas": st.get("currentReplicas", 0),
                                                     "desiredReplicas": st.get("desiredReplicas", 0)}, None, conds)
            return
        _set_condition(conds, "AbleToScale", "True", "SucceededGetScale",
                       "the HPA controller was able to get the target's current scale", stamp)
        tspec = target.get("spec") or {}
        current = int(tspec.get("replicas", 1))
        sel = tspec.get("selector") or {}
        selector = selector_from_set(sel) if ref.get("kind") == "ReplicationController" else selector_from_label_selector(sel)
        selector_str = ",".join(f"{k}={v}" for k, v in sorted(sel.items())) if ref.get("kind") == "ReplicationController" \
            else _selector_string(sel)
        # every pod the selector matches, as the reference's pod list: the calculator itself sets
        # unready (not Running and Ready) and metric-less pods aside
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == ns and selector.matches(m.labels_of(p))]
        lo, hi = int(spec.get("minReplicas", 1)), int(spec.get("maxReplicas", current))
        current_metrics, gpu_util, reason = None, None, ""
        if current == 0:
            desired = 0     # autoscaling is disabled for a target scaled to zero
            _set_condition(conds, "ScalingActive", "False", "ScalingDisabled",
                           "scaling is disabled since the replica count of the target is zero", stamp)
        else:
            proposals, failure, gpu_util = await self._metric_proposals(hpa, ns, pods, selector_str, current)
            current_metrics = [p[2] for p in proposals if p[2] is not None]
            if proposals:
                desired, reason = max((p[0], p[1]) for p in proposals)
                _set_condition(conds, "ScalingActive", "True", "ValidMetricFound",
                               f"the HPA was able to successfully calculate a replica count from {reason}", stamp)
            else:
                desired = current
                if failure is not None:
                    _set_condition(conds, "ScalingActive", "False", failure[0], failure[1], stamp)
                    self._event(hpa, "Warning", failure[0], failure[1])
            bounded = max(lo, min(hi, desired, max(2 * current, 4)))
            if desired > hi or (bounded < desired and bounded == max(2 * current, 4)):
                limit = ("TooManyReplicas", "the desired replica count is more than the maximum replica count") \
                    if desired > hi else ("ScaleUpLimit", "the desired replica count is increasing faster than the maximum scale rate")
                _set_condition(conds, "ScalingLimited", "True", *limit, stamp)
            elif desired < lo:
                _set_condition(conds, "ScalingLimited", "True", "TooFewReplicas",
                               "the desired replica count is less than the minimum replica count", stamp)
            else:
                _set_condition(conds, "ScalingLimited", "False", "DesiredWithinRange",
                               "the desired count is within the acceptable range", stamp)
            desired = bounded
        last = m.parse_time(st.get("lastScaleTime"))
        rescale = desired != current
        if rescale and last is not None:
            up_blocked = desired > current and now - last < self.upscale_delay
            down_blocked = desired < current and now - last < self.downscale_delay
            if up_blocked or down_blocked:
                rescale = False
                _set_condition(conds, "AbleToScale", "False", "BackoffUpscale" if up_blocked else "BackoffDownscale",
                               "the time since the previous scale is still within the "
                               f"{'upscale' if up_blocked else 'downscale'} forbidden window", stamp)
        new_st = {"currentReplicas": current, "desiredReplicas": desired if rescale else current,
                  "observedGeneration": (hpa.get("metadata") or {}).get("generation", 1)}
        if rescale:
            await self.client.patch(plural, ref["name"], {"spec": {"replicas": desired}}, ns)
            new_st["lastScaleTime"] = stamp
            _set_condition(conds, "AbleToScale", "True", "SucceededRescale",
                           f"the HPA controller was able to update the target scale to {desired}", stamp)
            self._event(hpa, "Normal", "SuccessfulRescale", f"New size: {desired}; reason: {reason} above target"
                        if desired > current else f"New size: {desired}; reason: All metrics below target")
        elif st.get("lastScaleTime"):
            new_st["lastScaleTime"] = st["lastScaleTime"]
        await self._write_status(hpa, ns, name, new_st, current_metrics, conds)
        if gpu_util is not None:
            v = f"{gpu_util:.1f}"
            if ann.get("autoscaling.amd.com/current-gpu-utilization") != v:
                await self.client.patch("horizontalpodautoscalers", name,
                                        {"metadata": {"annotations": {"autoscaling.amd.com/current-gpu-utilization": v}}}, ns)

    async def _write_status(self, hpa, ns, name, new_st, current_metrics, conds):
        """Through the v2beta1 status subresource; skipped when nothing but timestamps would change."""
        old = api_autoscaling.v1_to_v2(json.loads(json.dumps(hpa))).get("status") or {}
        body = dict(new_st)
        if current_metrics is not None:
            body["currentMetrics"] = current_metrics
        body["conditions"] = conds
        same = all(old.get(k) == v for k, v in new_st.items()) and \
            (current_metrics is None or old.get("currentMetrics", []) == current_metrics) and \
            [{k: c.get(k) for k in ("type", "status", "reason", "message")} for c in old.get("conditions") or []] == \
            [{k: c.get(k) for k in ("type", "status", "reason", "message")} for c in conds]
        if same:
            return
        await self.client.request("PATCH", f"/apis/autoscaling/v2beta1/namespaces/{ns}/horizontalpodautoscalers/{name}/status",
                                  body={"status": body}, content_type="application/merge-patch+json")


def _selector_string(sel: dict) -> str:
    parts = [f"{k}={v}" for k, v in sorted((sel.get("matchLabels") or {}).items())]
    for e in sel.get("matchExpressions") or []:
        op, vals = e.get("operator"), ",".join(e.get("values") or [])
        parts.append({"In": f"{e['key']} in ({vals})", "NotIn": f"{e['key']} notin ({vals})",
                      "Exists": e["key"], "DoesNotExist": f"!{e['key']}"}.get(op, e["key"]))
    return ",".join(parts)
