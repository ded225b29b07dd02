"""HorizontalPodAutoscaler controller, with a GPU-utilization target for MI355X workloads.

Reference: pkg/controller/podautoscaler/horizontal.go + replica_calculator.go (1.9,
autoscaling/v1): every --horizontal-pod-autoscaler-sync-period (30 s) read the target's
scale; utilization = Σ usage / Σ requests over the target's running pods that report
metrics; usageRatio = utilization / target; inside the 10 % tolerance nothing changes,
else desired = ceil(usageRatio × pods-with-metrics); clamp to [minReplicas, maxReplicas]
and to the scale-up limit max(2 × current, 4); a scale-up needs 3 min and a scale-down 5 min
since the last rescale (--horizontal-pod-autoscaler-{upscale,downscale}-delay); status
carries currentReplicas / desiredReplicas / currentCPUUtilizationPercentage / lastScaleTime.

MI355X extension: the annotation `autoscaling.amd.com/target-gpu-utilization: "<pct>"` adds
a second metric, the mean MI355X activity (amd-smi duty cycle, exported per container by
the kubelet's accelerator stats) of the pods' assigned GPUs. The larger of the two
proposals wins (the multi-metric rule of autoscaling/v2).

Metrics come from the resource metrics API (metrics.k8s.io, the metrics-server) when it is
registered, else straight from the kubelets' /stats/summary, where CPU usage is the rate between
two successive cumulative samples.
"""
from __future__ import annotations

import asyncio
import math
import time

import aiohttp

from ..api import meta as m
from ..api.helpers import is_pod_terminal
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
                cpu_milli, gpu, ngpu = 0.0, 0.0, 0
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
                    for a in c.get("accelerators") or []:
                        gpu += float(a.get("dutyCycle", 0))
                        ngpu += 1
                ent = {}
                if have_cpu:
                    ent["cpu_milli"] = cpu_milli
                if ngpu:
                    ent["gpu_util"] = gpu / ngpu
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
            ent = {"cpu_milli": float(sum(Quantity(ct["usage"]["cpu"]).as_fraction() * 1000
                                          for ct in pm.get("containers") or []))}
            duty = ((pm.get("metadata") or {}).get("annotations") or {}).get("amd.com/gpu-duty-cycle")
            if duty is not None:
                ent["gpu_util"] = float(duty)
            out[m.name_of(pm)] = ent
        return out

    async def close(self):
        await self.fallback.close()


def _cpu_request_milli(pod) -> int:
    total = 0
    for c in (pod.get("spec") or {}).get("containers") or []:
        v = ((c.get("resources") or {}).get("requests") or {}).get("cpu")
        if v is None:
            return 0  # reference: a pod missing a CPU request makes CPU utilization undefined
        total += Quantity(v).milli_value()
    return total


def cpu_proposal(pods, metrics, target_pct, current) -> tuple[int | None, int | None]:
    usage = req = 0
    n = 0
    for p in pods:
        mt = metrics.get(m.name_of(p)) or {}
        r = _cpu_request_milli(p)
        if "cpu_milli" not in mt or r <= 0:
            continue
        usage += mt["cpu_milli"]
        req += r
        n += 1
    if n == 0 or req == 0:
        return None, None
    util = int(round(usage * 100.0 / req))
    ratio = util / float(target_pct)
    if abs(ratio - 1.0) <= TOLERANCE:
        return current, util
    return int(math.ceil(ratio * n)), util


def gpu_proposal(pods, metrics, target_pct, current) -> tuple[int | None, float | None]:
    vals = [(metrics.get(m.name_of(p)) or {}).get("gpu_util") for p in pods]
    vals = [v for v in vals if v is not None]
    if not vals:
        return None, None
    util = sum(vals) / len(vals)
    ratio = util / float(target_pct)
    if abs(ratio - 1.0) <= TOLERANCE:
        return current, util
    return int(math.ceil(ratio * len(vals))), util


class HorizontalPodAutoscalerController(Controller):
    name = "horizontalpodautoscaling"
    workers = 1

    def __init__(self, mgr, metrics=None, sync_period: float = 30.0, upscale_delay: float = 180.0,
                 downscale_delay: float = 300.0, clock=time.time):
        super().__init__(mgr)
        self.metrics = metrics or ResourceMetricsAPI(mgr.client)
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

    async def sync(self, key):
        hpa = self.hpa_inf.get(key)
        if hpa is None:
            return
        ns, name = split_key(key)
        spec, st = hpa.get("spec") or {}, hpa.get("status") or {}
        ref = spec.get("scaleTargetRef") or {}
        plural = SCALE_TARGETS.get(ref.get("kind"))
        if plural is None:
            return
        target = await self.client.get_or_none(plural, ref.get("name", ""), ns)
        if target is None:
            return
        tspec = target.get("spec") or {}
        current = int(tspec.get("replicas", 1))
        sel = tspec.get("selector") or {}
        selector = selector_from_set(sel) if ref.get("kind") == "ReplicationController" else selector_from_label_selector(sel)
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == ns and selector.matches(m.labels_of(p))
                and not is_pod_terminal(p) and not (p.get("metadata") or {}).get("deletionTimestamp")
                and (p.get("status") or {}).get("phase") == "Running"]
        metrics = await self.metrics.pod_metrics(ns)
        proposals = []
        cpu_target = spec.get("targetCPUUtilizationPercentage", 80 if GPU_TARGET_ANNOTATION not in m.annotations_of(hpa) else None)
        cpu_util = gpu_util = None
        if cpu_target:
            r, cpu_util = cpu_proposal(pods, metrics, cpu_target, current)
            if r is not None:
                proposals.append(r)
        gt = m.annotations_of(hpa).get(GPU_TARGET_ANNOTATION)
        if gt:
            r, gpu_util = gpu_proposal(pods, metrics, float(gt), current)
            if r is not None:
                proposals.append(r)
        desired = max(proposals) if proposals else current
        lo, hi = int(spec.get("minReplicas", 1)), int(spec.get("maxReplicas", current))
        desired = max(lo, min(hi, desired, max(2 * current, 4)))
        now = self.clock()
        last = m.parse_time(st.get("lastScaleTime"))
        rescale = desired != current
        if rescale and last is not None:
            if desired > current and now - last < self.upscale_delay:
                rescale = False
            if desired < current and now - last < self.downscale_delay:
                rescale = False
        new_st = {"currentReplicas": current, "desiredReplicas": desired if rescale else current,
                  "observedGeneration": (hpa.get("metadata") or {}).get("generation", 1)}
        if cpu_util is not None:
            new_st["currentCPUUtilizationPercentage"] = cpu_util
        if rescale:
            await self.client.patch(plural, ref["name"], {"spec": {"replicas": desired}}, ns)
            new_st["lastScaleTime"] = m.format_time(now)
        elif st.get("lastScaleTime"):
            new_st["lastScaleTime"] = st["lastScaleTime"]
        ann = {}
        if gpu_util is not None:
            ann["autoscaling.amd.com/current-gpu-utilization"] = f"{gpu_util:.1f}"
        if {k: st.get(k) for k in new_st} != new_st:
            await self.client.patch("horizontalpodautoscalers", name, {"status": new_st}, ns, sub="status")
        if ann and any(m.annotations_of(hpa).get(k) != v for k, v in ann.items()):
            await self.client.patch("horizontalpodautoscalers", name, {"metadata": {"annotations": ann}}, ns)
