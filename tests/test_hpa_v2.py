"""HorizontalPodAutoscaler autoscaling/v2beta1 and the custom metrics API.

Reference tests mirrored: pkg/apis/autoscaling/v1/conversion_test.go (v2beta1 metrics and
status round-trip through the v1 annotations), pkg/controller/podautoscaler/horizontal_test.go
(TestScaleUpCMUnreadyLessScale-style Pods metrics, TestConditionFailedGetMetrics,
TestScaleUpRCExceedMaxReplicas conditions, Object metrics), and the custom-metrics-apiserver's
MetricValueList shape. The e2e test drives the whole path on MI355X-shaped fake devices:
amd-smi duty cycle → kubelet summary → metrics-server custom.metrics.k8s.io → aggregator →
HPA Pods metric gpu_utilization → Deployment scale."""
from __future__ import annotations

import copy
import json

import pytest

from amdkube.api import autoscaling as A
from amdkube.api import meta as m
from amdkube.controllers.autoscaling import (_fmt, _selector_string, get_plain_metric_replicas, get_resource_replicas,
                                             resource_metrics_milli)
from amdkube.localcluster import LocalCluster
from amdkube.metrics import MetricsServer
from tests.test_controllers_ext import _replicas, _status_ready, pod_tpl, until

V2 = "/apis/autoscaling/v2beta1/namespaces/default/horizontalpodautoscalers"


def _hpa_v2(name="infer", metrics=None, lo=1, hi=4, kind="Deployment"):
    return {"apiVersion": "autoscaling/v2beta1", "kind": "HorizontalPodAutoscaler", "metadata": {"name": name},
            "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": kind, "name": name},
                     "minReplicas": lo, "maxReplicas": hi, "metrics": metrics or []}}


# ------------------------------------------------------------------------ conversion
def test_v2beta1_round_trips_through_v1_annotations():
    metrics = [{"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 70}},
               {"type": "Pods", "pods": {"metricName": "gpu_utilization", "targetAverageValue": "50"}},
               {"type": "Resource", "resource": {"name": "memory", "targetAverageValue": "1Gi"}}]
    v2 = _hpa_v2(metrics=metrics)
    v2["status"] = {"currentReplicas": 2, "desiredReplicas": 3,
                    "currentMetrics": [{"type": "Resource", "resource": {"name": "cpu", "currentAverageUtilization": 91}},
                                       {"type": "Pods", "pods": {"metricName": "gpu_utilization", "currentAverageValue": "88"}}],
                    "conditions": [{"type": "ScalingActive", "status": "True", "reason": "ValidMetricFound", "message": "x"}]}
    v1 = A.v2_to_v1(copy.deepcopy(v2))
    ann = v1["metadata"]["annotations"]
    assert v1["spec"]["targetCPUUtilizationPercentage"] == 70 and "metrics" not in v1["spec"]
    assert [x["type"] for x in json.loads(ann[A.METRICS_ANNOTATION])] == ["Pods", "Resource"]
    assert v1["status"]["currentCPUUtilizationPercentage"] == 91
    assert set(ann) == {A.METRICS_ANNOTATION, A.CURRENT_METRICS_ANNOTATION, A.CONDITIONS_ANNOTATION}
    back = A.v1_to_v2(copy.deepcopy(v1))
    assert back["spec"]["metrics"] == metrics
    assert back["status"]["currentMetrics"] == v2["status"]["currentMetrics"]
    assert back["status"]["conditions"] == v2["status"]["conditions"]
    assert "annotations" not in back["metadata"]
    # a v1 object with no metric at all reads as the defaulted 80 % CPU target
    bare = {"metadata": {"name": "x"}, "spec": {"maxReplicas": 2}}
    assert A.metrics_of(bare) == [{"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 80}}]
    # no CPU metric but a Pods metric: no defaulted CPU target appears
    only_pods = A.v2_to_v1(_hpa_v2(metrics=metrics[1:2]))
    assert "targetCPUUtilizationPercentage" not in only_pods["spec"] and A.metrics_of(only_pods) == metrics[1:2]


def test_replica_calculator_units():
    pods = [{"metadata": {"name": f"p{i}"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "500m", "memory": "1Gi"}}}]},
             "status": {"phase": "Running", "conditions": [{"type": "Ready", "status": "True"}]}} for i in range(2)]
    mt = {"p0": {"cpu_milli": 900.0, "memory_bytes": 3 << 30}, "p1": {"cpu_milli": 300.0, "memory_bytes": 1 << 30}}
    cpu, mem = resource_metrics_milli(mt, "cpu"), resource_metrics_milli(mt, "memory")
    # cpu utilization: 1200m of 1000m = 120 % vs 60 % → ceil(2 × 2) = 4; raw average 600m
    assert get_resource_replicas(2, 60, "cpu", pods, cpu) == (4, 120, 600)
    # raw memory average 2 Gi vs 1 Gi → 4; utilization 200 % vs 190 % is inside the 10 % tolerance
    assert get_plain_metric_replicas(2, (1 << 30) * 1000, pods, mem) == (4, (2 << 30) * 1000)
    assert get_resource_replicas(2, 190, "memory", pods, mem)[:2] == (2, 200)
    # a container without a request makes the utilization undefined: the reference errors out
    del pods[1]["spec"]["containers"][0]["resources"]["requests"]["cpu"]
    with pytest.raises(LookupError, match="missing request for cpu"):
        get_resource_replicas(2, 60, "cpu", pods, cpu)
    assert _fmt(0.6) == "600m" and _fmt(88.0) == "88" and _fmt(1.25) == "1250m"
    assert _selector_string({"matchLabels": {"b": "2", "a": "1"},
                             "matchExpressions": [{"key": "t", "operator": "In", "values": ["x", "y"]}]}) == "a=1,b=2,t in (x,y)"


# ------------------------------------------------------------------------ apiserver
async def test_v2beta1_served_next_to_v1():
    async with LocalCluster(gpus="none", with_controllers=False, relist_period=0.2) as lc:
        c = lc.client
        metrics = [{"type": "Pods", "pods": {"metricName": "gpu_utilization", "targetAverageValue": "50"}},
                   {"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 70}}]
        made = await c.request("POST", V2, body=_hpa_v2(metrics=metrics))
        assert made["apiVersion"] == "autoscaling/v2beta1"
        assert sorted(x["type"] for x in made["spec"]["metrics"]) == ["Pods", "Resource"]
        v1 = await c.get("horizontalpodautoscalers", "infer", "default")
        assert v1["apiVersion"] == "autoscaling/v1" and v1["spec"]["targetCPUUtilizationPercentage"] == 70
        assert "gpu_utilization" in v1["metadata"]["annotations"][A.METRICS_ANNOTATION]
        # merge patch against the v2beta1 view replaces the metric list
        await c.request("PATCH", V2 + "/infer", body={"spec": {"metrics": metrics[:1], "maxReplicas": 6}},
                        content_type="application/merge-patch+json")
        v1 = await c.get("horizontalpodautoscalers", "infer", "default")
        assert "targetCPUUtilizationPercentage" not in v1["spec"] and v1["spec"]["maxReplicas"] == 6
        # status through the v2beta1 status subresource lands in the v1 annotations
        await c.request("PATCH", V2 + "/infer/status", content_type="application/merge-patch+json", body={"status": {
            "currentReplicas": 1, "desiredReplicas": 2,
            "currentMetrics": [{"type": "Pods", "pods": {"metricName": "gpu_utilization", "currentAverageValue": "90"}}],
            "conditions": [{"type": "AbleToScale", "status": "True", "reason": "SucceededRescale", "message": "m"}]}})
        v1 = await c.get("horizontalpodautoscalers", "infer", "default")
        ann = v1["metadata"]["annotations"]
        assert v1["status"]["desiredReplicas"] == 2 and '"90"' in ann[A.CURRENT_METRICS_ANNOTATION]
        assert "SucceededRescale" in ann[A.CONDITIONS_ANNOTATION]
        # a v1 spec update keeps what the status writer put in the annotations
        await c.patch("horizontalpodautoscalers", "infer", {"spec": {"minReplicas": 2}}, "default")
        v2 = await c.request("GET", V2 + "/infer")
        assert v2["spec"]["minReplicas"] == 2 and v2["status"]["currentMetrics"][0]["pods"]["currentAverageValue"] == "90"
        assert v2["status"]["conditions"][0]["reason"] == "SucceededRescale"
        lst = await c.request("GET", V2)
        assert lst["kind"] == "HorizontalPodAutoscalerList" and lst["items"][0]["spec"]["metrics"] == metrics[:1]


# ------------------------------------------------------------------------ controller
class FakeSources:
    """Resource metrics (pod_metrics) plus the custom metrics API (pod_metric / object_metric)."""

    def __init__(self):
        self.resource, self.pods, self.objects = {}, {}, {}
        self.selectors = []

    async def pod_metrics(self, ns):
        return dict(self.resource)

    async def pod_metric(self, ns, metric, selector):
        self.selectors.append(selector)
        return dict(self.pods.get(metric, {}))

    async def object_metric(self, ns, target, metric):
        key = (target.get("kind"), target.get("name"), metric)
        if key not in self.objects:
            raise LookupError(f"no {metric} for {key}")
        return self.objects[key]


async def _v2(c, name="infer"):
    return await c.request("GET", f"{V2}/{name}")


def _cond(h, typ):
    return next((x for x in (h.get("status") or {}).get("conditions") or [] if x["type"] == typ), {})


async def test_hpa_v2_pods_object_and_conditions():
    src = FakeSources()
    kw = {"hpa_metrics": src, "hpa_sync_period": 0.2, "hpa_upscale_delay": 0.0, "hpa_downscale_delay": 0.0}
    async with LocalCluster(gpus="none", controllers_kw=kw, relist_period=0.2) as lc:
        c = lc.client
        await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "infer"},
                        "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "infer"}}, "template": pod_tpl({"app": "infer"})}},
                       "default")
        await until(lambda: _status_ready(c, "deployments", "infer", 1), 30)
        # only an Object metric, which cannot be read → ScalingActive False, nothing moves
        await c.request("POST", V2, body=_hpa_v2(hi=3, metrics=[
            {"type": "Object", "object": {"target": {"kind": "Service", "name": "front"}, "metricName": "requests_per_second",
                                          "targetValue": "100"}}]))

        async def failed():
            return _cond(await _v2(c), "ScalingActive").get("reason") == "FailedGetObjectMetric"
        await until(failed)
        assert (await c.get("deployments", "infer", "default"))["spec"]["replicas"] == 1
        # the object now reports 250 rps against 100 → ceil(2.5 × 1) = 3
        src.objects[("Service", "front", "requests_per_second")] = 250.0
        await until(lambda: _replicas(c, "infer", 3))
        h = await _v2(c)
        assert _cond(h, "ScalingActive")["reason"] == "ValidMetricFound"
        assert h["status"]["currentMetrics"][0]["object"]["currentValue"] == "250"
        await until(lambda: _status_ready(c, "deployments", "infer", 3), 30)
        # switch to the Pods metric gpu_utilization: 3 pods at 90 vs target 40 → ceil(2.25 × 3) = 7 → capped at 3
        pods = (await c.list("pods", "default", label_selector="app=infer"))[0]
        src.pods["gpu_utilization"] = {m.name_of(p): 90.0 for p in pods}
        await c.request("PATCH", V2 + "/infer", content_type="application/merge-patch+json", body={"spec": {"metrics": [
            {"type": "Pods", "pods": {"metricName": "gpu_utilization", "targetAverageValue": "40"}}]}})

        async def limited():
            h = await _v2(c)
            pods_read = [x["type"] for x in h["status"].get("currentMetrics") or []] == ["Pods"]
            return pods_read and _cond(h, "ScalingLimited").get("reason") == "TooManyReplicas" and h
        h = await until(limited)
        assert h["status"]["currentMetrics"] == [{"type": "Pods", "pods": {"metricName": "gpu_utilization", "currentAverageValue": "90"}}]
        assert "app=infer" in src.selectors
        # idle GPUs → all metrics below target → down to minReplicas, the range condition clears
        src.pods["gpu_utilization"] = {m.name_of(p): 2.0 for p in pods}
        await until(lambda: _replicas(c, "infer", 1))

        async def in_range():
            return _cond(await _v2(c), "ScalingLimited").get("reason") in ("DesiredWithinRange", "TooFewReplicas")
        await until(in_range)
        evs, _ = await c.list("events", "default")
        assert any(e.get("reason") == "SuccessfulRescale" and "New size: 3" in e.get("message", "") for e in evs)


# ------------------------------------------------------------------------ e2e through the custom metrics API
async def test_custom_metrics_api_drives_gpu_hpa(tmp_path):
    from tests.test_metrics_server import _ca, _leaf
    d = str(tmp_path)
    _ca(d, "serving-ca")
    scert, skey = _leaf(d, "serving-ca", "metrics", "metrics-server", server=True)
    kw = {"hpa_sync_period": 0.2, "hpa_upscale_delay": 0.0, "hpa_downscale_delay": 0.0}
    async with LocalCluster(gpus="fake", n_gpus=4, controllers_kw=kw, relist_period=0.2) as lc:
        c = lc.client
        ms = await MetricsServer(c, resolution=0.2, tls_cert=scert, tls_key=skey, authorize=False).start()
        try:
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "metrics-server", "namespace": "kube-system"},
                            "spec": {"ports": [{"port": 443, "targetPort": ms.port}]}})
            await c.create({"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "metrics-server", "namespace": "kube-system"},
                            "subsets": [{"addresses": [{"ip": "127.0.0.1"}], "ports": [{"port": ms.port}]}]})
            for grp in ("metrics.k8s.io", "custom.metrics.k8s.io"):
                await c.create({"apiVersion": "apiregistration.k8s.io/v1beta1", "kind": "APIService",
                                "metadata": {"name": f"v1beta1.{grp}"},
                                "spec": {"group": grp, "version": "v1beta1", "groupPriorityMinimum": 100, "versionPriority": 100,
                                         "insecureSkipTLSVerify": True, "service": {"namespace": "kube-system", "name": "metrics-server"}}})
            tpl = pod_tpl({"app": "infer"})
            tpl["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": "1"}}
            await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "infer"},
                            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "infer"}}, "template": tpl}}, "default")
            await until(lambda: _status_ready(c, "deployments", "infer", 1), 30)
            for i in range(4):
                lc.backend.set_sample(i, gfx_activity=90)
            base = "/apis/custom.metrics.k8s.io/v1beta1"
            disc = await c.request("GET", base)
            assert {"pods/gpu_utilization", "nodes/gpu_count"} <= {r["name"] for r in disc["resources"]}

            async def busy():
                try:
                    d = await c.request("GET", f"{base}/namespaces/default/pods/*/gpu_utilization", params={"labelSelector": "app=infer"})
                except m.StatusError:
                    return None
                return d if d["items"] and float(d["items"][0]["value"]) == 90 else None
            vals = await until(busy)
            it = vals["items"][0]
            assert vals["kind"] == "MetricValueList" and it["describedObject"]["kind"] == "Pod" and it["metricName"] == "gpu_utilization"
            one = await c.request("GET", f"{base}/namespaces/default/pods/{it['describedObject']['name']}/gpu_count")
            assert one["items"][0]["value"] == "1"
            node = await c.request("GET", f"{base}/nodes/{lc.node_name}/gpu_count")
            assert node["items"][0]["value"] == "4"
            try:
                await c.request("GET", f"{base}/namespaces/default/pods/*/not_a_metric")
                raise AssertionError("unknown metric served")
            except m.StatusError as e:
                assert e.code == 404
            # the HPA reads gpu_utilization through the aggregator: 90 vs 45 → 2 replicas
            await c.request("POST", V2, body=_hpa_v2(hi=2, metrics=[
                {"type": "Pods", "pods": {"metricName": "gpu_utilization", "targetAverageValue": "45"}}]))
            await until(lambda: _replicas(c, "infer", 2), 30)
            h = await _v2(c)
            assert _cond(h, "ScalingActive")["reason"] == "ValidMetricFound"
            await until(lambda: _status_ready(c, "deployments", "infer", 2), 30)
        finally:
            await ms.stop()


def test_metrics_server_help_mentions_custom_metrics():
    from amdkube.cmd import components
    assert "custom.metrics.k8s.io" in components.metrics_server.__doc__


def test_custom_metrics_paths_stay_inside_the_metrics_api():
    """Object-metric targets come from the HPA's spec: a name such as '../../api/v1/secrets'
    must not turn the controller's request into a read of another API path."""
    import asyncio as _asyncio

    import pytest as _pytest

    from amdkube.controllers.autoscaling import CustomMetricsAPI
    seen = []

    class C:
        async def request(self, method, path, **kw):
            seen.append(path)
            return {"items": [{"value": "3"}]}

    async def go():
        api = CustomMetricsAPI(C())
        assert await api.object_metric("ml", {"kind": "Service", "name": "../../../api/v1/secrets"}, "qps") == 3.0
        with _pytest.raises(LookupError):
            await api.object_metric("ml", {"kind": "Service", "name": ".."}, "qps")
        await api.pod_metric("ml", "gpu/../x", "app=a")
    _asyncio.run(go())
    assert seen[0] == "/apis/custom.metrics.k8s.io/v1beta1/namespaces/ml/services/..%2F..%2F..%2Fapi%2Fv1%2Fsecrets/qps"
    assert seen[1].endswith("/pods/*/gpu%2F..%2Fx")
