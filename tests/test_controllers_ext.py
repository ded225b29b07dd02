"""The rest of kube-controller-manager (controllermanager.go:332-363): statefulset,
replicationcontroller, cronjob, disruption (+ eviction), HPA (CPU and MI355X GPU
utilization), resourcequota, serviceaccount(+token), csr approve/sign/clean, bootstrap
signer / token cleaner, ttl, clusterrole aggregation, PV binder / provisioner / protection /
expansion / attach-detach, cloud service load balancers and routes.

Reference tests mirrored: pkg/controller/statefulset/stateful_set_control_test.go,
pkg/controller/cronjob/utils_test.go, pkg/controller/disruption/disruption_test.go +
pkg/registry/core/pod/storage/eviction_test.go, pkg/controller/podautoscaler/horizontal_test.go,
pkg/controller/resourcequota, pkg/controller/serviceaccount/tokens_controller_test.go,
pkg/controller/certificates/approver/sarapprove_test.go, pkg/controller/bootstrap,
pkg/controller/ttl/ttl_controller_test.go, pkg/controller/volume/persistentvolume/binder_test.go,
pkg/controller/service/service_controller_test.go, pkg/controller/route/route_controller_test.go."""
from __future__ import annotations

import asyncio
import base64
import calendar
import os
import subprocess
import time

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.cloudprovider import Fake, get_cloud_provider
from amdkube.controllers import ControllerManager, Options, resolve_controllers
from amdkube.controllers.accounts import detached_jws, verify_detached_jws
from amdkube.controllers.apps import CronSchedule, unmet_schedule_times
from amdkube.controllers.policy import ttl_for
from amdkube.controllers.volumes import find_best_match
from amdkube.localcluster import LocalCluster


async def until(fn, timeout=20.0, every=0.05):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    last = None
    while loop.time() < end:
        last = await fn()
        if last:
            return last
        await asyncio.sleep(every)
    raise TimeoutError(f"condition not met (last={last!r})")


def pod_tpl(labels, image="amdkube/pause:3.1", **spec):
    return {"metadata": {"labels": labels}, "spec": {"containers": [{"name": "c", "image": image}], **spec}}


# ------------------------------------------------------------------------ pure units
def test_cron_schedule_semantics():
    s = CronSchedule("*/15 9-17 * * mon-fri")
    t = calendar.timegm((2026, 10, 16, 17, 50, 0))         # Friday 17:50
    assert time.gmtime(s.next_after(t))[:5] == (2026, 10, 19, 9, 0)   # → Monday 09:00
    assert time.gmtime(CronSchedule("@monthly").next_after(calendar.timegm((2026, 12, 15, 0, 0, 0))))[:3] == (2027, 1, 1)
    # dom and dow both restricted: either may match (vixie cron)
    s = CronSchedule("0 0 13 * 5")
    hits = []
    t = calendar.timegm((2026, 1, 1, 0, 0, 0))
    for _ in range(6):
        t = s.next_after(t)
        hits.append(time.gmtime(t))
    assert all(h.tm_mday == 13 or h.tm_wday == 4 for h in hits)
    for bad in ("* * *", "61 * * * *", "*/0 * * * *", "a b c d e"):
        with pytest.raises(ValueError):
            CronSchedule(bad)
    assert len(unmet_schedule_times(CronSchedule("* * * * *"), 0, 60 * 100)) == 100
    with pytest.raises(RuntimeError):
        unmet_schedule_times(CronSchedule("* * * * *"), 0, 60 * 102)


def test_ttl_boundaries_and_jws():
    assert [ttl_for(n) for n in (1, 100, 101, 500, 1000, 2000, 5000, 10001)] == [0, 0, 15, 15, 30, 60, 300, 600]
    jws = detached_jws("kubeconfig-bytes", "abcdef", "0123456789abcdef")
    head, empty, sig = jws.split(".")
    assert empty == "" and verify_detached_jws(jws, "kubeconfig-bytes", "abcdef", "0123456789abcdef")
    assert not verify_detached_jws(jws, "tampered", "abcdef", "0123456789abcdef")


def test_pv_best_match():
    def pv(name, size, modes=("ReadWriteOnce",), cls="", labels=None, ref=None):
        return {"metadata": {"name": name, "labels": labels or {}},
                "spec": {"capacity": {"storage": size}, "accessModes": list(modes), "storageClassName": cls,
                         **({"claimRef": ref} if ref else {})}, "status": {"phase": "Available"}}
    claim = {"metadata": {"name": "c", "namespace": "ns", "uid": "u1"},
             "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "5Gi"}}}}
    vols = [pv("small", "1Gi"), pv("big", "100Gi"), pv("fit", "10Gi"), pv("rom", "6Gi", modes=("ReadOnlyMany",)),
            pv("other-class", "5Gi", cls="fast")]
    assert m.name_of(find_best_match(claim, vols)) == "fit"
    vols.append(pv("prebound", "50Gi", ref={"namespace": "ns", "name": "c"}))
    assert m.name_of(find_best_match(claim, vols)) == "prebound"
    sel = dict(claim, spec=dict(claim["spec"], selector={"matchLabels": {"tier": "gold"}}))
    assert find_best_match(sel, vols[:3]) is None
    assert m.name_of(find_best_match(sel, vols + [pv("gold", "20Gi", labels={"tier": "gold"})])) == "gold"


def test_controller_set_matches_reference_names():
    names = set(resolve_controllers("*", Options(allocate_node_cidrs=True, cloud=Fake()))) | {"bootstrapsigner", "tokencleaner"}
    ref = {"endpoint", "replicationcontroller", "podgc", "resourcequota", "namespace", "serviceaccount", "garbagecollector",
           "daemonset", "job", "deployment", "replicaset", "horizontalpodautoscaling", "disruption", "statefulset", "cronjob",
           "csrsigning", "csrapproving", "csrcleaner", "ttl", "bootstrapsigner", "tokencleaner", "service", "route",
           "persistentvolume-binder", "attachdetach", "persistentvolume-expander", "clusterrole-aggregation", "pvc-protection",
           "pv-protection"}
    assert ref <= names and "nodelifecycle" in names and "nodeipam" in names
    assert "ttl" not in resolve_controllers("*,-ttl", Options())
    with pytest.raises(ValueError):
        resolve_controllers("bogus", Options())


# ------------------------------------------------------------------ integration
async def test_statefulset_ordered_with_provisioned_claims(tmp_path):
    kw = {"hostpath_pv_root": str(tmp_path / "pv")}
    async with LocalCluster(gpus="none", controllers_kw=kw, relist_period=0.2) as lc:
        c = lc.client
        await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass",
                        "metadata": {"name": "local", "annotations": {"storageclass.kubernetes.io/is-default-class": "true"}},
                        "provisioner": "amdkube.io/host-path", "reclaimPolicy": "Delete", "allowVolumeExpansion": True})
        await c.create({"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "db"},
                        "spec": {"replicas": 2, "serviceName": "db", "selector": {"matchLabels": {"app": "db"}},
                                 "template": pod_tpl({"app": "db"}),
                                 "volumeClaimTemplates": [{"metadata": {"name": "data"}, "spec": {
                                     "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}}]}},
                       "default")
        seen = []

        async def both_running():
            pods = {m.name_of(p): p for p in (await c.list("pods", "default"))[0]}
            for n in ("db-0", "db-1"):
                if n in pods and n not in seen:
                    seen.append(n)
            return all(pods.get(n, {}).get("status", {}).get("phase") == "Running" for n in ("db-0", "db-1"))
        await until(both_running, 30)
        assert seen == ["db-0", "db-1"]   # OrderedReady
        p0 = await c.get("pods", "db-0", "default")
        assert p0["spec"]["hostname"] == "db-0" and p0["spec"]["subdomain"] == "db"
        pvc = await c.get("persistentvolumeclaims", "data-db-0", "default")
        assert pvc["status"]["phase"] == "Bound"
        pv = await c.get("persistentvolumes", pvc["spec"]["volumeName"])
        assert os.path.isdir(pv["spec"]["hostPath"]["path"]) and pv["spec"]["claimRef"]["name"] == "data-db-0"
        assert "kubernetes.io/pvc-protection" in pvc["metadata"]["finalizers"]
        st = await until(lambda: _status_ready(c, "statefulsets", "db", 2))
        assert st["updateRevision"].startswith("db-")
        # expansion of a bound claim on an expandable class
        await c.patch("persistentvolumeclaims", "data-db-0", {"spec": {"resources": {"requests": {"storage": "2Gi"}}}}, "default")
        await until(lambda: _cap(c, "data-db-0", "2Gi"))
        # scale down removes the highest ordinal
        await c.patch("statefulsets", "db", {"spec": {"replicas": 1}}, "default")
        await until(lambda: _gone(c, "pods", "db-1"), 30)
        assert await c.get_or_none("pods", "db-0", "default") is not None
        # host-path volumes are not attachable: the attach/detach controller leaves them alone
        # (CSI / FlexVolume / block attachments are covered in test_volumes.py)
        node = await c.get("nodes", lc.node_name)
        assert not node["status"].get("volumesAttached") and not node["status"].get("volumesInUse")
        # deleting a claim of a stopped ordinal releases and (Delete policy) removes its volume
        pv1 = (await c.get("persistentvolumeclaims", "data-db-1", "default"))["spec"]["volumeName"]
        await c.delete("persistentvolumeclaims", "data-db-1", "default")
        await until(lambda: _gone(c, "persistentvolumes", pv1, ns=""), 20)


async def _status_ready(c, res, name, n):
    o = await c.get(res, name, "default")
    st = o.get("status") or {}
    return st if st.get("readyReplicas") == n else None


async def _cap(c, name, want):
    p = await c.get("persistentvolumeclaims", name, "default")
    return ((p.get("status") or {}).get("capacity") or {}).get("storage") == want


async def _gone(c, res, name, ns="default"):
    return await c.get_or_none(res, name, ns) is None


async def test_replication_controller_and_pdb_eviction():
    async with LocalCluster(gpus="none", relist_period=0.2) as lc:
        c = lc.client
        await c.create({"apiVersion": "v1", "kind": "ReplicationController", "metadata": {"name": "rc"},
                        "spec": {"replicas": 2, "selector": {"app": "rc"}, "template": pod_tpl({"app": "rc"})}}, "default")
        await until(lambda: _status_ready(c, "replicationcontrollers", "rc", 2), 30)
        await c.create({"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget", "metadata": {"name": "pdb"},
                        "spec": {"minAvailable": 1, "selector": {"matchLabels": {"app": "rc"}}}}, "default")

        async def allowed(n):
            p = await c.get("poddisruptionbudgets", "pdb", "default")
            return (p.get("status") or {}).get("disruptionsAllowed") == n and p["status"].get("currentHealthy") == 2
        await until(lambda: allowed(1))
        pods = [m.name_of(p) for p in (await c.list("pods", "default", label_selector="app=rc"))[0]]
        ev = {"apiVersion": "policy/v1beta1", "kind": "Eviction", "metadata": {"name": pods[0], "namespace": "default"}}
        await c.request("POST", f"/api/v1/namespaces/default/pods/{pods[0]}/eviction", body=ev)
        ev["metadata"]["name"] = pods[1]
        with pytest.raises(m.StatusError) as ei:
            await c.request("POST", f"/api/v1/namespaces/default/pods/{pods[1]}/eviction", body=ev)
        assert ei.value.code == 429
        # the RC replaces the evicted pod; once healthy again the budget reopens
        await until(lambda: allowed(1), 30)


class FakeMetrics:
    def __init__(self):
        self.values = {}

    async def pod_metrics(self, ns):
        return dict(self.values)


async def test_hpa_scales_on_gpu_and_cpu_utilization():
    fm = FakeMetrics()
    kw = {"hpa_metrics": fm, "hpa_sync_period": 0.2, "hpa_upscale_delay": 0.0, "hpa_downscale_delay": 0.0}
    async with LocalCluster(gpus="none", controllers_kw=kw, relist_period=0.2) as lc:
        c = lc.client
        tpl = pod_tpl({"app": "infer"})
        tpl["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "500m"}}
        await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "infer"},
                        "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "infer"}}, "template": tpl}}, "default")
        await until(lambda: _status_ready(c, "deployments", "infer", 1), 30)
        await c.create({"apiVersion": "autoscaling/v1", "kind": "HorizontalPodAutoscaler",
                        "metadata": {"name": "infer", "annotations": {"autoscaling.amd.com/target-gpu-utilization": "50"}},
                        "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "infer"},
                                 "minReplicas": 1, "maxReplicas": 3}}, "default")
        pod = (await c.list("pods", "default", label_selector="app=infer"))[0][0]
        fm.values = {m.name_of(pod): {"gpu_util": 95.0}}          # ratio 1.9 → ceil(1.9 × 1) = 2
        await until(lambda: _replicas(c, "infer", 2))
        h = await c.get("horizontalpodautoscalers", "infer", "default")
        assert h["status"]["desiredReplicas"] == 2 and h["metadata"]["annotations"]["autoscaling.amd.com/current-gpu-utilization"] == "95.0"
        await until(lambda: _status_ready(c, "deployments", "infer", 2), 30)
        # CPU target: 2 pods at 900m of 500m requested → 180 % vs 60 % → ceil(3 × 2) = 6, capped at max 3
        pods = (await c.list("pods", "default", label_selector="app=infer"))[0]
        fm.values = {m.name_of(p): {"cpu_milli": 900.0, "gpu_util": 50.0} for p in pods}
        await c.patch("horizontalpodautoscalers", "infer", {"spec": {"targetCPUUtilizationPercentage": 60}}, "default")
        await until(lambda: _replicas(c, "infer", 3))
        await until(lambda: _status_ready(c, "deployments", "infer", 3), 30)
        # idle → down to minReplicas; every pod reports (a pod without a metric counts as at target
        # on a scale-down, replica_calculator.go)
        pods = (await c.list("pods", "default", label_selector="app=infer"))[0]
        fm.values = {m.name_of(p): {"cpu_milli": 1.0, "gpu_util": 1.0} for p in pods}
        await until(lambda: _replicas(c, "infer", 1))


async def _replicas(c, name, n):
    d = await c.get("deployments", name, "default")
    return d["spec"]["replicas"] == n


async def test_cronjob_creates_jobs_and_forbids_overlap():
    async with LocalCluster(gpus="none", relist_period=0.2) as lc:
        c = lc.client
        lc.controllers.get("cronjob").period = 0.2
        await c.create({"apiVersion": "batch/v1beta1", "kind": "CronJob", "metadata": {"name": "tick"},
                        "spec": {"schedule": "@every 1s", "concurrencyPolicy": "Forbid",
                                 "jobTemplate": {"spec": {"template": {"spec": {
                                     "restartPolicy": "Never",
                                     "containers": [{"name": "c", "image": "busybox", "args": ["-c", "sleep 30"]}]}}}}}},
                       "default")

        async def jobs():
            return (await c.list("jobs", "default"))[0]
        js = await until(jobs, 15)
        await asyncio.sleep(2.5)
        assert len(await jobs()) == 1     # Forbid: the first job is still active
        cj = await c.get("cronjobs", "tick", "default")
        assert cj["status"]["active"][0]["name"] == m.name_of(js[0]) and cj["status"]["lastScheduleTime"]
        # getJobFromTemplate: the name carries the scheduled time (getTimeHash: Unix seconds)
        assert m.name_of(js[0]) == f"tick-{int(m.parse_time(cj['status']['lastScheduleTime']))}"
        await c.patch("cronjobs", "tick", {"spec": {"concurrencyPolicy": "Replace"}}, "default")
        first = m.uid_of(js[0])

        async def replaced():
            return all(m.uid_of(j) != first for j in await jobs())
        await until(replaced, 15)


async def test_quota_serviceaccounts_tokens_rbac(tmp_path):
    key = b"test-service-account-signing-key"
    async with LocalCluster(gpus="none", api_kw={"authorization_mode": "RBAC", "service_account_key": key,
                                                 "token_auth": {"admin-token": {"name": "admin", "groups": ["system:masters"]}}},
                            controllers_kw={"service_account_key": key}, with_kubelet=False) as lc:
        admin = Client(lc.api.url, token="admin-token")
        try:
            await admin.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            sa = await until(lambda: admin.get_or_none("serviceaccounts", "default", "team"))
            sa = await until(lambda: _with_secret(admin, "team"))
            sec = await admin.get("secrets", sa["secrets"][0]["name"], "team")
            assert sec["type"] == "kubernetes.io/service-account-token"
            token = base64.b64decode(sec["data"]["token"]).decode()
            tr = await admin.create({"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview", "spec": {"token": token}})
            assert tr["status"]["authenticated"] and tr["status"]["user"]["username"] == "system:serviceaccount:team:default"
            sac = Client(lc.api.url, token=token)
            try:
                with pytest.raises(m.StatusError) as ei:
                    await sac.list("pods", "team")
                assert ei.value.code == 403
                await admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                                    "metadata": {"name": "sa-view", "namespace": "team"},
                                    "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "view"},
                                    "subjects": [{"kind": "ServiceAccount", "name": "default", "namespace": "team"}]}, "team")
                assert (await sac.list("pods", "team"))[0] == []
                with pytest.raises(m.StatusError):
                    await sac.list("pods", "default")          # the RoleBinding is namespaced
                with pytest.raises(m.StatusError):
                    await sac.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}}, "team")
                # deleting the token's secret revokes it
                await admin.delete("secrets", sec["metadata"]["name"], "team")
                with pytest.raises(m.StatusError) as ei:
                    await sac.list("pods", "team")
                assert ei.value.code == 401
            finally:
                await sac.close()
            # resource quota usage
            await admin.create({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"},
                                "spec": {"hard": {"pods": "10", "configmaps": "5", "requests.cpu": "4", "amd.com/gpu": "8"}}}, "team")

            async def populated():     # e2e waitForResourceQuota: admission needs status.used first
                q = await admin.get("resourcequotas", "q", "team")
                return q if (q.get("status") or {}).get("used") else None
            await until(populated)
            await admin.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm"}, "data": {}}, "team")
            await admin.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"},
                                "spec": {"containers": [{"name": "c", "image": "x", "resources": {
                                    "requests": {"cpu": "1500m"}, "limits": {"amd.com/gpu": "2"}}}]}}, "team")

            async def used():
                q = await admin.get("resourcequotas", "q", "team")
                u = (q.get("status") or {}).get("used") or {}
                return u if u.get("pods") == "1" and u.get("amd.com/gpu") == "2" else None
            u = await until(used)
            assert u["configmaps"] == "1" and u["requests.cpu"] == "1500m"
        finally:
            await admin.close()


async def _with_secret(c, ns):
    sa = await c.get_or_none("serviceaccounts", "default", ns)
    return sa if sa and sa.get("secrets") else None


def _openssl(*args, **kw):
    subprocess.run(["openssl", *args], check=True, capture_output=True, **kw)


async def test_node_csr_auto_approved_and_signed(tmp_path):
    d = str(tmp_path)
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/ca.key", "-out", f"{d}/ca.crt", "-days", "1",
             "-subj", "/CN=amdkube-ca")
    _openssl("req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/n.key", "-out", f"{d}/n.csr",
             "-subj", "/O=system:nodes/CN=system:node:mi355x-1")
    _openssl("req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/u.key", "-out", f"{d}/u.csr", "-subj", "/CN=alice")
    kw = {"cluster_signing_cert_file": f"{d}/ca.crt", "cluster_signing_key_file": f"{d}/ca.key"}
    users = {"mallory-token": {"name": "mallory", "groups": []}, "alice-token": {"name": "alice", "groups": []}}
    async with LocalCluster(gpus="none", api_kw={"authorization_mode": "RBAC", "token_auth": users}, controllers_kw=kw,
                            with_kubelet=False) as lc:
        c = lc.client
        b = lambda s: base64.b64encode(s.encode()).decode()  # noqa: E731
        await c.create({"apiVersion": "v1", "kind": "Secret", "type": "bootstrap.kubernetes.io/token",
                        "metadata": {"name": "bootstrap-token-abcdef"},
                        "data": {"token-id": b("abcdef"), "token-secret": b("0123456789abcdef"),
                                 "usage-bootstrap-authentication": b("true")}}, "kube-system")
        # anyone may request certificates (RBAC here: bootstrappers via policy, others via this binding)
        await c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                        "metadata": {"name": "csr-create"},
                        "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "system:node-bootstrapper"},
                        "subjects": [{"kind": "Group", "name": "system:authenticated"}]})

        def csr(name, path):
            return {"apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest", "metadata": {"name": name},
                    "spec": {"request": base64.b64encode(open(path, "rb").read()).decode(), "username": "spoofed",
                             "groups": ["system:masters"], "usages": ["digital signature", "key encipherment", "client auth"]}}
        for token, name, path in (("abcdef.0123456789abcdef", "node-csr", f"{d}/n.csr"), ("alice-token", "alice-csr", f"{d}/u.csr"),
                                  ("mallory-token", "rogue-csr", f"{d}/n.csr")):
            uc = Client(lc.api.url, token=token)
            try:
                o = await uc.create(csr(name, path))
            finally:
                await uc.close()
            assert o["spec"]["username"] != "spoofed" and "system:masters" not in o["spec"]["groups"]

        async def issued():
            o = await c.get("certificatesigningrequests", "node-csr")
            return (o.get("status") or {}).get("certificate")
        cert = base64.b64decode(await until(issued, 20))
        open(f"{d}/n.crt", "wb").write(cert)
        _openssl("verify", "-CAfile", f"{d}/ca.crt", f"{d}/n.crt")
        o = await c.get("certificatesigningrequests", "node-csr")
        assert o["status"]["conditions"][0]["reason"] == "AutoApproved"
        for other in ("alice-csr", "rogue-csr"):   # not a node cert / requester not allowed
            o = await c.get("certificatesigningrequests", other)
            assert not (o.get("status") or {}).get("conditions")
        cleaner = lc.controllers.get("csrcleaner")
        o = await c.get("certificatesigningrequests", "node-csr")
        assert not cleaner.expired(o) and cleaner.expired(o, now=time.time() + 7200)


async def test_bootstrap_signer_token_cleaner_ttl_and_aggregation():
    names = ["bootstrapsigner", "tokencleaner", "ttl", "clusterrole-aggregation"]
    async with LocalCluster(gpus="none", relist_period=0.2, controllers_kw={}) as lc:
        cm = ControllerManager(Client(lc.api.url), names)
        await cm.start()
        c = lc.client
        try:
            kubeconfig = "apiVersion: v1\nkind: Config\nclusters: []\n"
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cluster-info"},
                            "data": {"kubeconfig": kubeconfig}}, "kube-public")
            b = lambda s: base64.b64encode(s.encode()).decode()  # noqa: E731
            await c.create({"apiVersion": "v1", "kind": "Secret", "type": "bootstrap.kubernetes.io/token",
                            "metadata": {"name": "bootstrap-token-abcdef"},
                            "data": {"token-id": b("abcdef"), "token-secret": b("0123456789abcdef"),
                                     "usage-bootstrap-signing": b("true"), "usage-bootstrap-authentication": b("true"),
                                     "expiration": b(m.format_time(time.time() + 2))}}, "kube-system")

            async def signed():
                o = await c.get("configmaps", "cluster-info", "kube-public")
                return (o.get("data") or {}).get("jws-kubeconfig-abcdef")
            jws = await until(signed)
            assert verify_detached_jws(jws, kubeconfig, "abcdef", "0123456789abcdef")
            # the bootstrap token authenticates until it expires, then the cleaner removes it
            tr = await c.create({"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview",
                                 "spec": {"token": "abcdef.0123456789abcdef"}})
            assert tr["status"]["user"]["username"] == "system:bootstrap:abcdef"
            assert "system:bootstrappers" in tr["status"]["user"]["groups"]
            await until(lambda: _gone(c, "secrets", "bootstrap-token-abcdef", "kube-system"), 10)
            await until(lambda: _unsigned(c), 10)
            # ttl annotation
            node = await until(lambda: _ttl(c, lc.node_name))
            assert node == "0"
            # aggregation
            await c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                            "metadata": {"name": "gpu-ops", "labels": {"amd.com/aggregate-to-gpu": "true"}},
                            "rules": [{"apiGroups": [""], "resources": ["nodes"], "verbs": ["get"]}]})
            await c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": "gpu-admin"},
                            "aggregationRule": {"clusterRoleSelectors": [{"matchLabels": {"amd.com/aggregate-to-gpu": "true"}}]}})

            async def aggregated():
                return (await c.get("clusterroles", "gpu-admin")).get("rules")
            assert (await until(aggregated))[0]["resources"] == ["nodes"]
        finally:
            await cm.stop()
            await cm.client.close()


async def _unsigned(c):
    o = await c.get("configmaps", "cluster-info", "kube-public")
    return "jws-kubeconfig-abcdef" not in (o.get("data") or {})


async def _ttl(c, node):
    n = await c.get("nodes", node)
    return m.annotations_of(n).get("node.alpha.kubernetes.io/ttl")


async def test_cloud_load_balancer_and_routes():
    fake = Fake()
    bm = get_cloud_provider("baremetal", {"loadBalancerIPRange": "192.168.50.0/29", "programRoutes": False})
    async with LocalCluster(gpus="none", relist_period=0.2, node_status_update_frequency=0.3,
                            controllers_kw={"cloud": bm, "allocate_node_cidrs": True}) as lc:
        c = lc.client
        svc = await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "lb"},
                              "spec": {"type": "LoadBalancer", "selector": {"app": "x"}, "ports": [{"port": 80}]}}, "default")
        assert svc["spec"]["ports"][0]["nodePort"]

        async def ingress():
            s = await c.get("services", "lb", "default")
            return (((s.get("status") or {}).get("loadBalancer") or {}).get("ingress") or [None])[0]
        ing = await until(ingress)
        assert ing["ip"].startswith("192.168.50.")
        # routes: the node's pod CIDR becomes a route; NetworkUnavailable=False
        routes = bm.routes()
        await until(lambda: _true(any(r.target_node == lc.node_name for r in routes.list("kubernetes"))))
        # the service stops being a LoadBalancer → balancer released, status cleared
        # (as in the reference, the NodePort/LoadBalancer-only externalTrafficPolicy goes with the type)
        await c.patch("services", "lb", {"spec": {"type": "ClusterIP", "externalTrafficPolicy": None,
                                                  "ports": [{"port": 80, "nodePort": None}]}}, "default")
        await until(lambda: _true(not bm.load_balancer().assigned))
    # the fake provider records the same calls
    async with LocalCluster(gpus="none", with_kubelet=False, controllers_kw={"cloud": fake}) as lc:
        await lc.client.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "lb"},
                                "spec": {"type": "LoadBalancer", "ports": [{"port": 80}]}}, "default")
        await until(lambda: _true("create" in fake.calls))
        await lc.client.delete("services", "lb", "default")
        await until(lambda: _true("delete" in fake.calls))


async def _true(v):
    return v


async def test_route_controller_deletes_only_routes_inside_the_cluster_cidr():
    """route_controller.go:264-275 isResponsibleForRoute: a NAT-instance default route named like
    an instance route (AWS lists every instance route as `{cluster}-{cidr}`) and a tenant route
    outside --cluster-cidr survive; a stale in-cluster route is deleted."""
    from amdkube.cloudprovider import Route
    from amdkube.controllers.cloud import RouteController

    class Routes:
        named = False

        def __init__(self):
            self.rs = [Route("kubernetes-0.0.0.0/0", "nat-instance", "0.0.0.0/0"),
                       Route("tenant", "db-server", "172.16.5.0/24"),
                       Route("kubernetes-stale", "gone-node", "10.244.7.0/24"),
                       Route("kubernetes-n1", "n1", "10.244.1.0/24")]
            self.deleted = []

        def list(self, cluster):
            return list(self.rs)

        def create(self, cluster, name, r):
            self.rs.append(r)

        def delete(self, cluster, r):
            self.deleted.append(r.destination_cidr)
            self.rs.remove(r)

    class Cloud:
        def __init__(self):
            self.r = Routes()

        def routes(self):
            return self.r

    class Nodes:
        def list(self):
            return [{"metadata": {"name": "n1", "uid": "u1"}, "spec": {"podCIDR": "10.244.1.0/24"}, "status": {
                "conditions": [{"type": "NetworkUnavailable", "status": "False"}]}}]

    class Mgr:
        client = None
        nodes = Nodes()
    cloud = Cloud()
    rc = RouteController(Mgr(), cloud, "kubernetes", "10.244.0.0/16")
    rc.node_inf = Mgr.nodes
    await rc.sync("@all")
    assert cloud.r.deleted == ["10.244.7.0/24"]
    assert {r.destination_cidr for r in cloud.r.rs} == {"0.0.0.0/0", "172.16.5.0/24", "10.244.1.0/24"}
    assert not rc.responsible_for(Route("x", "n", "10.0.0.0/8"))          # wider than the cluster CIDR
    assert rc.responsible_for(Route("x", "n", "10.244.255.0/24"))
