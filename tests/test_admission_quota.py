"""LimitRanger and ResourceQuota admission at the reference's semantics.

* LimitRanger: the TestPodLimitFunc / TestPersistentVolumeClaimLimitFunc tables of
  plugin/pkg/admission/limitranger/admission_test.go, extracted by
  hack/extract_limitranger_cases.py into tests/fixtures/limitranger_cases.json, plus
  TestDefaultContainerResourceRequirements, TestMergePodResourceRequirements,
  TestPodLimitFuncApplyDefault and TestLimitRangerIgnoresSubresource (ported).
* ResourceQuota: plugin/pkg/admission/resourcequota/admission_test.go's tests ported over an
  in-memory context (quota status, the CAS'd status update the admission writes), and the
  evaluators of pkg/quota/evaluator/core against the quota controller in a cluster.
* The round-4 probes through a live apiserver, and 40 concurrent creates against `pods: 5`
  over --etcd-servers with group commit.
"""
from __future__ import annotations

import asyncio
import copy
import json
import os

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import admission as adm
from tests.conftest import run

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "limitranger_cases.json")))


class Ctx:
    """The admission context: objects by (plural, ns, name), with the storage CAS the quota
    admission uses (every call recorded as an action)."""

    def __init__(self, *objs):
        self.objs = {}
        self.actions = []
        for o in objs:
            self.put(o)

    @staticmethod
    def _plural(o):
        return {"LimitRange": "limitranges", "ResourceQuota": "resourcequotas"}[o["kind"]]

    def put(self, o):
        o = copy.deepcopy(o)
        o.setdefault("apiVersion", "v1")
        self.objs[(self._plural(o), m.namespace_of(o), m.name_of(o))] = o

    def list_objects(self, plural, ns, group=""):
        return [copy.deepcopy(o) for (p, n, _), o in self.objs.items() if p == plural and n == ns]

    def guaranteed_update_object(self, plural, ns, name, fn, group=""):
        cur = self.objs.get((plural, ns, name))
        new = fn(copy.deepcopy(cur))
        if new is not None:
            self.objs[(plural, ns, name)] = new
            self.actions.append(("update", plural, "status", name))
        return new or cur


def _attrs(obj, op=adm.CREATE, resource="pods", sub="", old=None):
    return adm.Attributes(op, resource, sub, m.namespace_of(obj) or "test", m.name_of(obj), obj, old, None,
                          obj.get("kind", ""))


def _lr_run(obj, lr, resource="pods"):
    plug = adm.LimitRanger()
    ctx = Ctx(lr)
    a = _attrs(copy.deepcopy(obj), resource=resource)
    plug.admit(a, ctx)
    plug.validate(a, ctx)
    return a.obj


# --------------------------------------------------------------------- LimitRanger tables
@pytest.mark.parametrize("case", FIX["pod"]["successCases"], ids=lambda c: c["name"])
def test_pod_limit_func_success_cases(case):
    _lr_run(case["object"], case["limitRange"])


@pytest.mark.parametrize("case", FIX["pod"]["errorCases"], ids=lambda c: c["name"])
def test_pod_limit_func_error_cases(case):
    with pytest.raises(m.StatusError) as ei:
        _lr_run(case["object"], case["limitRange"])
    assert ei.value.code == 403 and f'pods "{case["name"]}" is forbidden' in str(ei.value)


@pytest.mark.parametrize("case", FIX["pvc"]["successCases"], ids=lambda c: c["name"])
def test_pvc_limit_func_success_cases(case):
    _lr_run(case["object"], case["limitRange"], resource="persistentvolumeclaims")


@pytest.mark.parametrize("case", FIX["pvc"]["errorCases"], ids=lambda c: c["name"])
def test_pvc_limit_func_error_cases(case):
    with pytest.raises(m.StatusError):
        _lr_run(case["object"], case["limitRange"], resource="persistentvolumeclaims")


def _pod(name, n, requests=None, limits=None, init=()):
    res = {}
    if requests is not None:
        res["requests"] = dict(requests)
    if limits is not None:
        res["limits"] = dict(limits)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "test"},
           "spec": {"containers": [{"name": f"foo-{i}", "image": f"foo:V{i}", "resources": copy.deepcopy(res)}
                                   for i in range(n)]}}
    for i, r in enumerate(init):
        pod["spec"].setdefault("initContainers", []).append({"name": f"foo-{i}", "image": f"foo:V{i}",
                                                             "resources": copy.deepcopy(r)})
    return pod


def test_default_container_resource_requirements():
    """admission_test.go:162 TestDefaultContainerResourceRequirements."""
    reqs, lims = adm.default_container_requirements(FIX["validLimitRange"])
    assert reqs == {"cpu": "50m", "memory": "5Mi"} and lims == {"cpu": "75m", "memory": "10Mi"}


def test_merge_pod_resource_requirements_and_annotation():
    """admission_test.go:193 TestMergePodResourceRequirements."""
    plug, lr = adm.LimitRanger(), FIX["validLimitRange"]
    a = _attrs(_pod("empty-resources", 1))
    plug.admit(a, Ctx(lr))
    assert a.obj["spec"]["containers"][0]["resources"] == {"requests": {"cpu": "50m", "memory": "5Mi"},
                                                          "limits": {"cpu": "75m", "memory": "10Mi"}}
    assert a.obj["metadata"]["annotations"][adm.LIMIT_RANGER_ANNOTATION] == \
        "LimitRanger plugin set: cpu, memory request for container foo-0; cpu, memory limit for container foo-0"
    inp = {"requests": {"memory": "512Mi"}}
    a = _attrs(_pod("limit-memory", 1, requests={"memory": "512Mi"}, init=[inp]))
    plug.admit(a, Ctx(lr))
    want = {"requests": {"cpu": "50m", "memory": "512Mi"}, "limits": {"cpu": "75m", "memory": "10Mi"}}
    assert a.obj["spec"]["containers"][0]["resources"] == want and a.obj["spec"]["initContainers"][0]["resources"] == want
    # the init container's defaults are recorded under the "init container" prefix (the Go test
    # checks only the container half of the annotation; amdkube records both)
    assert a.obj["metadata"]["annotations"][adm.LIMIT_RANGER_ANNOTATION].startswith(
        "LimitRanger plugin set: cpu request for container foo-0; cpu, memory limit for container foo-0")
    full = {"requests": {"cpu": "100m", "memory": "512Mi"}, "limits": {"cpu": "200m", "memory": "1G"}}
    init_full = {"requests": {"cpu": "200m", "memory": "1G"}, "limits": {"cpu": "400m", "memory": "2G"}}
    a = _attrs(_pod("limit-memory", 1, full["requests"], full["limits"], init=[init_full]))
    plug.admit(a, Ctx(lr))
    assert a.obj["spec"]["containers"][0]["resources"] == full and a.obj["spec"]["initContainers"][0]["resources"] == init_full
    assert adm.LIMIT_RANGER_ANNOTATION not in (a.obj["metadata"].get("annotations") or {})


def test_pod_limit_func_apply_default():
    """admission_test.go:636 TestPodLimitFuncApplyDefault (containers and init containers)."""
    a = _attrs(_pod("foo", 1, {}, {}, init=[{}]))
    adm.LimitRanger().admit(a, Ctx(FIX["validLimitRange"]))
    for c in a.obj["spec"]["containers"] + a.obj["spec"]["initContainers"]:
        assert c["resources"] == {"limits": {"cpu": "75m", "memory": "10Mi"}, "requests": {"cpu": "50m", "memory": "5Mi"}}


def test_limit_ranger_ignores_subresource_and_checks_updates():
    """admission_test.go:687/713: an UPDATE without limits is refused; a status update is not checked."""
    plug, ctx = adm.LimitRanger(), Ctx(FIX["validLimitRangeNoDefaults"])
    pod = _pod("testPod", 1)
    a = _attrs(pod, op=adm.UPDATE)
    plug.admit(a, ctx)
    with pytest.raises(m.StatusError):
        plug.validate(a, ctx)
    plug.validate(_attrs(pod, op=adm.UPDATE, sub="status"), ctx)


def test_limit_range_defaulting_on_store():
    """SetDefaults_LimitRangeItem: a Container item's default comes from max and its
    defaultRequest from default, then min; so a stored LimitRange with only min/max still
    defaults pods."""
    from amdkube.api import SCHEME
    lr = {"apiVersion": "v1", "kind": "LimitRange", "metadata": {"name": "l", "namespace": "test"},
          "spec": {"limits": [{"type": "Container", "max": {"cpu": "2"}, "min": {"memory": "64Mi"}}]}}
    SCHEME.default(lr)
    item = lr["spec"]["limits"][0]
    assert item["default"] == {"cpu": "2"} and item["defaultRequest"] == {"cpu": "2", "memory": "64Mi"}


# --------------------------------------------------------------------- ResourceQuota
def _quota(name, hard, used, scopes=None, ns="test"):
    q = {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": name, "namespace": ns, "resourceVersion": "124"},
         "spec": {"hard": dict(hard)}, "status": {"hard": dict(hard), "used": dict(used)}}
    if scopes:
        q["spec"]["scopes"] = list(scopes)
    return q


CPU_MEM_PODS = ({"cpu": "3", "memory": "100Gi", "pods": "5"}, {"cpu": "1", "memory": "50Gi", "pods": "3"})


def _quota_validate(ctx, obj, op=adm.CREATE, resource="pods", old=None, sub=""):
    adm.ResourceQuota().validate(_attrs(obj, op=op, resource=resource, old=old, sub=sub), ctx)


def test_admission_ignores_delete_and_subresources():
    """admission_test.go:125,152."""
    ctx = Ctx(_quota("quota", {"memory": "100Mi"}, {"memory": "90Mi"}))
    plug = adm.ResourceQuota()
    assert adm.DELETE not in plug.operations
    pod = _pod("123", 1, {"memory": "100Mi"}, {})
    with pytest.raises(m.StatusError):
        _quota_validate(ctx, pod)
    _quota_validate(ctx, pod, sub="status")


def test_admit_below_quota_limit_updates_status():
    """admission_test.go:191 TestAdmitBelowQuotaLimit: used becomes cpu=1100m, memory=52Gi, pods=4,
    written with an update of resourcequotas/status."""
    ctx = Ctx(_quota("quota", *CPU_MEM_PODS))
    _quota_validate(ctx, _pod("allowed-pod", 1, {"cpu": "100m", "memory": "2Gi"}, {}))
    assert ("update", "resourcequotas", "status", "quota") in ctx.actions
    used = ctx.objs[("resourcequotas", "test", "quota")]["status"]["used"]
    assert (used["cpu"], used["memory"], used["pods"]) == ("1100m", "52Gi", "4")


def test_admit_handles_old_objects():
    """admission_test.go:272: LoadBalancer -> NodePort(1 port) charges only the new nodeport."""
    ctx = Ctx(_quota("quota", {"services": "10", "services.loadbalancers": "10", "services.nodeports": "10"},
                     {"services": "1", "services.loadbalancers": "1", "services.nodeports": "0"}))
    old = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "service", "namespace": "test", "resourceVersion": "1"},
           "spec": {"type": "LoadBalancer"}}
    new = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "service", "namespace": "test"},
           "spec": {"type": "NodePort", "ports": [{"port": 1234}]}}
    _quota_validate(ctx, new, op=adm.UPDATE, resource="services", old=old)
    used = ctx.objs[("resourcequotas", "test", "quota")]["status"]["used"]
    assert used == {"services": "1", "services.loadbalancers": "1", "services.nodeports": "1"}


def test_admit_exceed_quota_limit():
    """admission_test.go:643."""
    ctx = Ctx(_quota("quota", *CPU_MEM_PODS))
    with pytest.raises(m.StatusError) as ei:
        _quota_validate(ctx, _pod("not-allowed-pod", 1, {"cpu": "3", "memory": "2Gi"}, {}))
    assert "exceeded quota: quota, requested: cpu=3, used: cpu=1, limited: cpu=3" in str(ei.value)
    assert not ctx.actions


def test_admit_enforce_quota_constraints():
    """admission_test.go:686: limits.memory is limited, so every container must set it; and a
    limit below its request is refused."""
    hard = {"cpu": "3", "memory": "100Gi", "limits.memory": "200Gi", "pods": "5"}
    used = {"cpu": "1", "memory": "50Gi", "limits.memory": "100Gi", "pods": "3"}
    ctx = Ctx(_quota("quota", hard, used))
    with pytest.raises(m.StatusError) as ei:
        _quota_validate(ctx, _pod("not-allowed-pod", 1, {"cpu": "100m", "memory": "2Gi"}, {"cpu": "200m"}))
    assert "failed quota: quota: must specify limits.memory" in str(ei.value)
    with pytest.raises(m.StatusError):
        _quota_validate(ctx, _pod("not-allowed-pod", 1, {"cpu": "200m", "memory": "2Gi"}, {"cpu": "100m", "memory": "1Gi"}))


def test_admit_pod_in_namespace_without_quota():
    """admission_test.go:736."""
    hard = {"cpu": "3", "memory": "100Gi", "limits.memory": "200Gi", "pods": "5"}
    ctx = Ctx(_quota("quota", hard, {"cpu": "1", "memory": "50Gi", "limits.memory": "100Gi", "pods": "3"}, ns="other"))
    _quota_validate(ctx, _pod("not-allowed-pod", 1, {"cpu": "100m", "memory": "2Gi"}, {"cpu": "200m"}))


def test_admit_below_terminating_quota_limit():
    """admission_test.go:789: a pod with activeDeadlineSeconds is charged only to the
    Terminating-scoped quota."""
    ctx = Ctx(_quota("quota-non-terminating", *CPU_MEM_PODS, scopes=["NotTerminating"]),
              _quota("quota-terminating", *CPU_MEM_PODS, scopes=["Terminating"]))
    pod = _pod("allowed-pod", 1, {"cpu": "100m", "memory": "2Gi"}, {})
    pod["spec"]["activeDeadlineSeconds"] = 30
    _quota_validate(ctx, pod)
    assert [a[3] for a in ctx.actions] == ["quota-terminating"]
    used = ctx.objs[("resourcequotas", "test", "quota-terminating")]["status"]["used"]
    assert (used["cpu"], used["memory"], used["pods"]) == ("1100m", "52Gi", "4")


def test_admit_best_effort_scopes():
    """admission_test.go:903 / :1010: a BestEffort pod charges the BestEffort quota only; a
    Burstable pod is ignored by a BestEffort-scoped quota."""
    ctx = Ctx(_quota("quota-besteffort", {"pods": "5"}, {"pods": "3"}, scopes=["BestEffort"]),
              _quota("quota-not-besteffort", {"pods": "5"}, {"pods": "3"}, scopes=["NotBestEffort"]))
    _quota_validate(ctx, _pod("allowed-pod", 1))
    assert [a[3] for a in ctx.actions] == ["quota-besteffort"]
    assert ctx.objs[("resourcequotas", "test", "quota-besteffort")]["status"]["used"]["pods"] == "4"
    ctx2 = Ctx(_quota("quota-besteffort", {"pods": "5"}, {"pods": "3"}, scopes=["BestEffort"]))
    _quota_validate(ctx2, _pod("allowed-pod", 1, {"cpu": "100m", "memory": "1Gi"}, {}))
    assert not ctx2.actions


def test_has_usage_stats_and_unknown_status():
    """admission_test.go:1054 TestHasUsageStats; a quota the controller has not filled in yet
    refuses admission ("status unknown")."""
    from amdkube import quota as Q
    assert not Q.has_usage_stats({"status": {}})
    assert not Q.has_usage_stats({"status": {"hard": {"cpu": "1"}, "used": {}}})
    assert Q.has_usage_stats({"status": {"hard": {"cpu": "1"}, "used": {"cpu": "0"}}})
    q = _quota("quota", {"pods": "5"}, {})
    q["status"]["used"] = {}
    with pytest.raises(m.StatusError) as ei:
        _quota_validate(Ctx(q), _pod("p", 1))
    assert "status unknown for quota: quota" in str(ei.value)


def test_admit_rejects_negative_usage():
    """admission_test.go:1143."""
    ctx = Ctx(_quota("quota", {"persistentvolumeclaims": "3", "requests.storage": "100Gi"},
                     {"persistentvolumeclaims": "1", "requests.storage": "10Gi"}))
    pvc = {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "pvc", "namespace": "test"},
           "spec": {"resources": {"requests": {"storage": "-1Gi"}}}}
    with pytest.raises(m.StatusError) as ei:
        _quota_validate(ctx, pvc, resource="persistentvolumeclaims")
    assert "quota usage is negative" in str(ei.value)
    pvc["spec"]["resources"]["requests"]["storage"] = "1Gi"
    _quota_validate(ctx, pvc, resource="persistentvolumeclaims")


def test_admit_when_unrelated_resource_exceeds_quota():
    """admission_test.go:1190: services over quota do not block a pod."""
    ctx = Ctx(_quota("quota", {"services": "3", "pods": "4"}, {"services": "4", "pods": "1"}))
    _quota_validate(ctx, _pod("allowed-pod", 1, {"cpu": "100m", "memory": "2Gi"}, {}))


def test_object_counts_and_storage_class_quota():
    ctx = Ctx(_quota("quota", {"configmaps": "1", "count/secrets": "0", "gold.storageclass.storage.k8s.io/requests.storage": "10Gi"},
                     {"configmaps": "1", "count/secrets": "0", "gold.storageclass.storage.k8s.io/requests.storage": "0"}))
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c", "namespace": "test"}}
    with pytest.raises(m.StatusError, match="configmaps=1"):
        _quota_validate(ctx, cm, resource="configmaps")
    with pytest.raises(m.StatusError, match="count/secrets"):
        _quota_validate(ctx, {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "s", "namespace": "test"}},
                        resource="secrets")
    pvc = {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "pvc", "namespace": "test"},
           "spec": {"storageClassName": "gold", "resources": {"requests": {"storage": "11Gi"}}}}
    with pytest.raises(m.StatusError, match="gold.storageclass"):
        _quota_validate(ctx, pvc, resource="persistentvolumeclaims")
    pvc["spec"]["storageClassName"] = "silver"
    _quota_validate(ctx, pvc, resource="persistentvolumeclaims")


def test_gpu_quota_counts_device_granular_extended_resources():
    """The fork extension: amd.com/gpu is charged from spec.extendedResources (ResourceV2's
    rewrite), under the bare name and requests.amd.com/gpu."""
    ctx = Ctx(_quota("gpu", {"amd.com/gpu": "4", "requests.amd.com/gpu": "4"}, {"amd.com/gpu": "3", "requests.amd.com/gpu": "3"}))
    pod = _pod("g", 1)
    pod["spec"]["extendedResources"] = [{"name": "x", "resources": {"limits": {"amd.com/gpu": "2"}, "requests": {"amd.com/gpu": "2"}}}]
    with pytest.raises(m.StatusError, match="amd.com/gpu=2"):
        _quota_validate(ctx, pod)
    pod["spec"]["extendedResources"][0]["resources"] = {"limits": {"amd.com/gpu": "1"}, "requests": {"amd.com/gpu": "1"}}
    _quota_validate(ctx, pod)
    assert ctx.objs[("resourcequotas", "test", "gpu")]["status"]["used"] == {"amd.com/gpu": "4", "requests.amd.com/gpu": "4"}


# --------------------------------------------------------------------- live apiserver
def test_round4_probes_refused_by_a_live_apiserver():
    """The probes of the round-4 review: a 10m-CPU pod under `min: 100m`, a 10x limit/request
    under `maxLimitRequestRatio: 2`, a 2-CPU pod under `hard: {cpu: "1"}`, a 2Gi-limit pod under
    `limits.memory: 1Gi` — all refused; BestEffort pods are not charged to a NotBestEffort quota."""
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "lr"}})
            await c.create({"apiVersion": "v1", "kind": "LimitRange", "metadata": {"name": "l", "namespace": "lr"},
                            "spec": {"limits": [{"type": "Container", "min": {"cpu": "100m"},
                                                 "maxLimitRequestRatio": {"cpu": "2"}}]}}, "lr")

            async def pod(ns, name, req=None, lim=None):
                res = {}
                if req:
                    res["requests"] = req
                if lim:
                    res["limits"] = lim
                try:
                    return await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": ns},
                                           "spec": {"containers": [{"name": "c", "image": "busybox", "resources": res}]}}, ns)
                except m.StatusError as e:
                    return e
            e = await pod("lr", "small", {"cpu": "10m"}, {"cpu": "10m"})
            assert isinstance(e, m.StatusError) and e.code == 403 and "minimum cpu usage per Container is 100m" in str(e)
            e = await pod("lr", "ratio", {"cpu": "100m"}, {"cpu": "1"})
            assert isinstance(e, m.StatusError) and "max limit to request ratio per Container is 2" in str(e)
            ok = await pod("lr", "fine", {"cpu": "200m"}, {"cpu": "300m"})
            assert isinstance(ok, dict)
            # quota: without the controller the status is filled in here, as the controller would
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "rq"}})
            for name, hard, scopes in (("cpu", {"cpu": "1", "limits.memory": "1Gi"}, None),
                                       ("nbe", {"pods": "1"}, ["NotBestEffort"])):
                q = await c.create({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": name, "namespace": "rq"},
                                    "spec": {"hard": hard, **({"scopes": scopes} if scopes else {})}}, "rq")
                q["status"] = {"hard": hard, "used": {k: "0" for k in hard}}
                await c.update(q, sub="status")
            e = await pod("rq", "big", {"cpu": "2", "memory": "100Mi"}, {"memory": "100Mi"})
            assert isinstance(e, m.StatusError) and "exceeded quota: cpu, requested: cpu=2, used: cpu=0, limited: cpu=1" in str(e)
            e = await pod("rq", "mem", {"cpu": "100m", "memory": "2Gi"}, {"memory": "2Gi"})
            assert isinstance(e, m.StatusError) and "limits.memory=2Gi" in str(e)
            e = await pod("rq", "nolimit", {"cpu": "100m"})
            assert isinstance(e, m.StatusError) and "must specify limits.memory" in str(e)
            assert isinstance(await pod("rq", "be1"), m.StatusError)       # cpu quota needs requests
            okp = await pod("rq", "ok", {"cpu": "500m", "memory": "100Mi"}, {"memory": "100Mi"})
            assert isinstance(okp, dict)
            used = (await c.get("resourcequotas", "cpu", "rq"))["status"]["used"]
            assert used == {"cpu": "500m", "limits.memory": "100Mi"}
            assert (await c.get("resourcequotas", "nbe", "rq"))["status"]["used"] == {"pods": "1"}
    run(go(), 90)


@pytest.mark.timeout(180)
async def test_concurrent_creates_over_etcd_admit_exactly_the_quota():
    """40 concurrent pod creates against `pods: 5` through an apiserver on --etcd-servers (amdkube
    etcd, bridged writes group-committed): exactly 5 are admitted, the other 35 are refused by
    the quota, and status.used ends at 5."""
    from amdkube.apiserver import APIServer
    from amdkube.client import Client
    from amdkube.store.etcd3 import Etcd3Store
    from tests.test_etcd import ServerThread
    with ServerThread(wire=True) as st:
        s = await asyncio.to_thread(Etcd3Store, st.address)
        srv = await APIServer(s).start()
        cs = [Client(srv.url, token=srv.loopback_token) for _ in range(8)]
        try:
            assert srv._bridged
            q = await cs[0].create({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "five", "namespace": "default"},
                                    "spec": {"hard": {"pods": "5"}}}, "default")
            q["status"] = {"hard": {"pods": "5"}, "used": {"pods": "0"}}
            await cs[0].update(q, sub="status")

            async def create(i):
                try:
                    return await cs[i % 8].create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": "default"},
                                                   "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
                except m.StatusError as e:
                    return e
            res = await asyncio.gather(*(create(i) for i in range(40)))
            made = [r for r in res if isinstance(r, dict)]
            refused = [r for r in res if isinstance(r, m.StatusError)]
            assert len(made) == 5, [str(r)[:120] for r in refused[:3]]
            assert len(refused) == 35 and all(r.code == 403 and "exceeded quota: five" in str(r) for r in refused)
            assert (await cs[0].get("resourcequotas", "five", "default"))["status"]["used"] == {"pods": "5"}
            items, _ = await cs[0].list("pods", "default")
            assert len(items) == 5
        finally:
            for c in cs:
                await c.close()
            await srv.stop()
            s.close()


@pytest.mark.timeout(180)
async def test_concurrent_bridged_binds_and_service_allocations_never_collide():
    """with bridged writes over Etcd3Store other requests run while a write is
    in flight. Eight concurrent binds of eight pods to the SAME device: exactly one wins, the
    rest get 409. Eight concurrent Services asking for one clusterIP / one nodePort: one each.
    24 Services auto-allocated concurrently get 24 distinct clusterIPs and nodePorts."""
    from amdkube.apiserver import APIServer
    from amdkube.benchmark.schedperf import fake_node
    from amdkube.client import Client
    from amdkube.smi import FakeBackend
    from amdkube.store.etcd3 import Etcd3Store
    from tests.test_etcd import ServerThread
    with ServerThread(wire=True) as st:
        s = await asyncio.to_thread(Etcd3Store, st.address)
        srv = await APIServer(s).start()
        cs = [Client(srv.url, token=srv.loopback_token) for _ in range(8)]
        try:
            assert srv._bridged
            node = fake_node(0, 8, FakeBackend())
            await cs[0].create(node)
            dev = sorted(node["status"]["extendedResources"]["amd.com/gpu"]["resources"])[0]
            for i in range(8):
                await cs[0].create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"g{i}", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": "1"}}}]}},
                                   "default")
            pods = [await cs[0].get("pods", f"g{i}", "default") for i in range(8)]

            async def bind(i):
                pres = pods[i]["spec"]["extendedResources"][0]["name"]
                try:
                    await cs[i].bind("default", f"g{i}", node["metadata"]["name"], {pres: {"resources": [dev]}})
                    return 201
                except m.StatusError as e:
                    return e.code
            codes = await asyncio.gather(*(bind(i) for i in range(8)))
            assert sorted(codes) == [201] + [409] * 7, codes
            owners = [p for p in (await cs[0].list("pods", "default"))[0]
                      if dev in sum((r.get("assigned") or [] for r in p["spec"].get("extendedResources") or []), [])]
            assert len(owners) == 1

            async def svc(i, **spec):
                try:
                    return await cs[i % 8].create({"apiVersion": "v1", "kind": "Service",
                                                   "metadata": {"name": f"s{i}-{len(spec)}", "namespace": "default"},
                                                   "spec": {"ports": [{"port": 80}], **spec}}, "default")
                except m.StatusError as e:
                    return e
            ips = await asyncio.gather(*(svc(i, clusterIP="10.0.0.77") for i in range(8)))
            assert sum(isinstance(r, dict) for r in ips) == 1
            nps = await asyncio.gather(*(svc(i, type="NodePort", ports=[{"port": 80, "nodePort": 30777}]) for i in range(8, 16)))
            assert sum(isinstance(r, dict) for r in nps) == 1
            autos = await asyncio.gather(*(svc(i, type="NodePort", selector={"a": str(i)}) for i in range(16, 40)))
            assert all(isinstance(r, dict) for r in autos)
            assert len({r["spec"]["clusterIP"] for r in autos}) == 24
            assert len({r["spec"]["ports"][0]["nodePort"] for r in autos}) == 24
            assert not srv.registry.services._pending and not srv.registry._device_claims
        finally:
            for c in cs:
                await c.close()
            await srv.stop()
            s.close()


def test_quota_controller_status_write_conflicts_with_a_reservation_made_after_its_read():
    """The controller writes status with the resourceVersion it read (resource_quota_controller.go
    :350-371): when the admission plugin reserved usage between that read and the write, the
    write is a 409 and the reservation stays, instead of being overwritten by stale usage."""
    import types
    from amdkube.controllers.policy import ResourceQuotaController
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            q = await c.create({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "rq"},
                                "spec": {"hard": {"pods": "3"}}}, "default")
            q["status"] = {"hard": {"pods": "3"}, "used": {"pods": "0"}}
            stale = await c.update_status(q)
            ctrl = ResourceQuotaController(types.SimpleNamespace(client=c))
            ctrl.q_inf = types.SimpleNamespace(get=lambda key: m.deepcopy(stale), list=lambda: [stale])
            # the controller's pod informer still lags with two pods it counts
            cached = [{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"old{i}", "namespace": "default"},
                       "spec": {"containers": [{"name": "c", "image": "busybox"}]}, "status": {"phase": "Running"}}
                      for i in range(2)]
            ctrl.pod_inf = types.SimpleNamespace(list=lambda: cached)
            ctrl.count_infs = {}
            # a reservation lands after the controller's read
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "new"},
                            "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
            assert (await c.get("resourcequotas", "rq", "default"))["status"]["used"] == {"pods": "1"}
            with pytest.raises(m.StatusError) as e:
                await ctrl.sync("default/rq")
            assert e.value.code == 409
            assert (await c.get("resourcequotas", "rq", "default"))["status"]["used"] == {"pods": "1"}
            # once the informer has the newer quota the retried sync writes
            fresh = await c.get("resourcequotas", "rq", "default")
            ctrl.q_inf = types.SimpleNamespace(get=lambda key: m.deepcopy(fresh), list=lambda: [fresh])
            await ctrl.sync("default/rq")
            assert (await c.get("resourcequotas", "rq", "default"))["status"]["used"] == {"pods": "2"}
    run(go(), 60)
