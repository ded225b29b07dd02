"""The reference's remaining admission plugins (plugin/pkg/admission/*/admission_test.go
tables, condensed): AlwaysPullImages, LimitPodHardAntiAffinityTopology, EventRateLimit,
DenyEscalatingExec/DenyExecOnPrivileged, OwnerReferencesPermissionEnforcement,
ImagePolicyWebhook, InitialResources, PersistentVolumeLabel, PersistentVolumeClaimResize,
PodPreset, PodTolerationRestriction, PodSecurityPolicy, SecurityContextDeny, Initializers."""
import asyncio
import json

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import admission_ext as X
from amdkube.apiserver.admission import CONNECT, CREATE, UPDATE, Attributes, Chain
from amdkube.localcluster import LocalCluster
from tests.conftest import run


class Ctx:
    def __init__(self, objects=None, allow=lambda *a: True, namespaces=None):
        self.objects = objects or {}
        self.allow = allow
        self.namespaces = namespaces or {}
        self.cloud = None

    def get_namespace(self, n):
        return self.namespaces.get(n, {"metadata": {"name": n}})

    def list_objects(self, plural, ns, group=""):
        return [o for o in self.objects.get(plural, []) if not ns or m.namespace_of(o) in ("", ns)]

    def get_object(self, plural, ns, name):
        return next((o for o in self.objects.get(plural, []) if m.name_of(o) == name), None)

    def authorize(self, user, verb, group, resource, sub="", ns="", name=""):
        return self.allow(user, verb, group, resource, sub, ns, name)

    def plural_for_kind(self, av, kind):
        return kind.lower() + "s"


def pod(name="p", **spec):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "ns", "labels": {"app": "x"}},
            "spec": {"containers": [{"name": "c", "image": "busybox"}], **spec}}


def attrs(obj, op=CREATE, resource="pods", sub="", old=None, user=None):
    return Attributes(op, resource, sub, "ns", m.name_of(obj or old or {}), obj, old, user or {"name": "alice", "groups": []})


def test_always_pull_and_antiaffinity_and_scdeny():
    p = pod(initContainers=[{"name": "i", "image": "x", "imagePullPolicy": "Never"}])
    a = attrs(p)
    X.AlwaysPullImages().admit(a, Ctx())
    assert all(c["imagePullPolicy"] == "Always" for c in p["spec"]["containers"] + p["spec"]["initContainers"])
    p["spec"]["containers"][0]["imagePullPolicy"] = "IfNotPresent"
    with pytest.raises(m.StatusError):
        X.AlwaysPullImages().validate(a, Ctx())
    bad = pod(affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {}, "topologyKey": "failure-domain.beta.kubernetes.io/zone"}]}})
    with pytest.raises(m.StatusError):
        X.LimitPodHardAntiAffinityTopology().validate(attrs(bad), Ctx())
    X.LimitPodHardAntiAffinityTopology().validate(attrs(pod()), Ctx())
    for spec in ({"securityContext": {"runAsUser": 0}}, {"securityContext": {"fsGroup": 1}},
                 {"securityContext": {"supplementalGroups": [1]}}):
        with pytest.raises(m.StatusError):
            X.SecurityContextDeny().validate(attrs(pod(**spec)), Ctx())
    p = pod()
    p["spec"]["containers"][0]["securityContext"] = {"seLinuxOptions": {"level": "s0"}}
    with pytest.raises(m.StatusError):
        X.SecurityContextDeny().validate(attrs(p), Ctx())
    X.SecurityContextDeny().validate(attrs(pod()), Ctx())


def test_event_rate_limit_buckets():
    plug = X.EventRateLimit([{"type": "Namespace", "qps": 0.001, "burst": 3, "cacheSize": 2},
                             {"type": "Server", "qps": 0.001, "burst": 100}])
    ev = {"kind": "Event", "metadata": {"name": "e", "namespace": "ns"}, "involvedObject": {"kind": "Pod"}}
    for _ in range(3):
        plug.validate(attrs(ev, resource="events"), Ctx())
    with pytest.raises(m.StatusError) as ei:
        plug.validate(attrs(ev, resource="events"), Ctx())
    assert ei.value.code == 429
    other = Attributes(CREATE, "events", "", "other", "e", ev, None, {})
    plug.validate(other, Ctx())                     # its own namespace bucket
    plug.validate(attrs(pod()), Ctx())              # not an event: ignored


def test_deny_exec_plugins():
    priv = pod()
    priv["spec"]["containers"][0]["securityContext"] = {"privileged": True}
    hostpid = pod(hostPID=True)
    for plug, target, denied in ((X.DenyEscalatingExec(), priv, True), (X.DenyEscalatingExec(), hostpid, True),
                                 (X.DenyExecOnPrivileged(), hostpid, False), (X.DenyExecOnPrivileged(), priv, True),
                                 (X.DenyEscalatingExec(), pod(), False)):
        a = Attributes(CONNECT, "pods", "exec", "ns", "p", None, target, {})
        if denied:
            with pytest.raises(m.StatusError):
                plug.validate(a, Ctx())
        else:
            plug.validate(a, Ctx())


def test_owner_references_permission_enforcement():
    ref = {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs", "uid": "u1"}
    p = pod()
    p["metadata"]["ownerReferences"] = [dict(ref)]
    no_delete = Ctx(allow=lambda u, verb, *r: verb != "delete")
    with pytest.raises(m.StatusError):
        X.OwnerReferencesPermissionEnforcement().validate(attrs(p), no_delete)
    X.OwnerReferencesPermissionEnforcement().validate(attrs(p), Ctx())
    p["metadata"]["ownerReferences"][0]["blockOwnerDeletion"] = True
    no_finalizers = Ctx(allow=lambda u, verb, g, res, sub, *r: not (sub == "finalizers"))
    with pytest.raises(m.StatusError):
        X.OwnerReferencesPermissionEnforcement().validate(attrs(p), no_finalizers)
    # unchanged references need nothing
    X.OwnerReferencesPermissionEnforcement().validate(attrs(p, UPDATE, old=json.loads(json.dumps(p))), Ctx(allow=lambda *a: False))


def test_image_policy_webhook_review_cache_and_default():
    from aiohttp import web

    async def go():
        calls = []

        async def review(request):
            body = await request.json()
            calls.append(body)
            allowed = all(not c["image"].startswith("evil/") for c in body["spec"]["containers"])
            return web.json_response({**body, "status": {"allowed": allowed, "reason": "" if allowed else "evil image"}})
        app = web.Application()
        app.router.add_post("/review", review)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        plug = X.ImagePolicyWebhook(url=f"http://127.0.0.1:{port}/review")
        ok = pod()
        ok["metadata"]["annotations"] = {"mycluster.image-policy.k8s.io/ticket": "1234", "other": "x"}
        await plug.admit_async(attrs(ok), Ctx())
        again = pod("p2")
        again["metadata"]["annotations"] = dict(ok["metadata"]["annotations"])
        await plug.admit_async(attrs(again), Ctx())    # identical review spec → cached
        assert len(calls) == 1 and calls[0]["spec"]["annotations"] == {"mycluster.image-policy.k8s.io/ticket": "1234"}
        bad = pod()
        bad["spec"]["containers"][0]["image"] = "evil/miner"
        with pytest.raises(m.StatusError) as ei:
            await plug.admit_async(attrs(bad), Ctx())
        assert "evil image" in ei.value.message
        await runner.cleanup()
        down = X.ImagePolicyWebhook(url=f"http://127.0.0.1:{port}/review", default_allow=True, timeout=0.5)
        p = pod("q")
        p["spec"]["containers"][0]["image"] = "other"
        await down.admit_async(attrs(p), Ctx())
        assert p["metadata"]["annotations"]["alpha.image-policy.k8s.io/failed-open"] == "true"
        with pytest.raises(m.StatusError):
            await X.ImagePolicyWebhook(url=f"http://127.0.0.1:{port}/review", timeout=0.5).admit_async(attrs(p), Ctx())
    run(go(), 30)


def test_initial_resources_percentile_estimate():
    class Src:
        def usage(self, res, image, ns, exact):
            if exact:
                return list(range(10))                  # too few samples for the exact tag
            return [float(i) for i in range(100)] if res == "cpu" else [float(1 << 20)] * 60
    p = pod()
    p["spec"]["containers"].append({"name": "set", "image": "busybox", "resources": {"requests": {"cpu": "1"}}})
    X.InitialResources(Src(), percentile=90).admit(attrs(p), Ctx())
    c0, c1 = p["spec"]["containers"]
    assert c0["resources"]["requests"] == {"cpu": "90m", "memory": str(1 << 20)}
    assert c1["resources"]["requests"]["cpu"] == "1" and c1["resources"]["requests"]["memory"] == str(1 << 20)
    assert "Initial Resources plugin set" in p["metadata"]["annotations"]["kubernetes.io/initial-resources"]


def test_pv_label_and_pvc_resize():
    class Cloud:
        def volume_labels(self, pv):
            return {"failure-domain.beta.kubernetes.io/zone": "z1", "failure-domain.beta.kubernetes.io/region": "r1"}
    pv = {"metadata": {"name": "pv"}, "spec": {"gcePersistentDisk": {"pdName": "d"}}}
    X.PersistentVolumeLabel(Cloud()).admit(attrs(pv, resource="persistentvolumes"), Ctx())
    assert pv["metadata"]["labels"]["failure-domain.beta.kubernetes.io/zone"] == "z1"
    with pytest.raises(m.StatusError):
        X.PersistentVolumeLabel().admit(attrs({"metadata": {"name": "x"}, "spec": {"awsElasticBlockStore": {}}},
                                              resource="persistentvolumes"), Ctx())
    X.PersistentVolumeLabel().admit(attrs({"metadata": {"name": "x"}, "spec": {"hostPath": {}}}, resource="persistentvolumes"), Ctx())

    def pvc(size, phase="Bound"):
        return {"metadata": {"name": "c", "namespace": "ns"}, "spec": {"storageClassName": "fast", "volumeName": "pv1",
                                                                        "resources": {"requests": {"storage": size}}},
                "status": {"phase": phase}}
    ctx = Ctx({"storageclasses": [{"metadata": {"name": "fast"}, "allowVolumeExpansion": True}],
               "persistentvolumes": [{"metadata": {"name": "pv1"}, "spec": {"gcePersistentDisk": {"pdName": "d"}}}]})
    plug = X.PersistentVolumeClaimResize()
    plug.validate(attrs(pvc("2Gi"), UPDATE, "persistentvolumeclaims", old=pvc("1Gi")), ctx)
    with pytest.raises(m.StatusError):
        plug.validate(attrs(pvc("2Gi"), UPDATE, "persistentvolumeclaims", old=pvc("1Gi", "Pending")), ctx)
    no_exp = Ctx({"storageclasses": [{"metadata": {"name": "fast"}}], "persistentvolumes": ctx.objects["persistentvolumes"]})
    with pytest.raises(m.StatusError):
        plug.validate(attrs(pvc("2Gi"), UPDATE, "persistentvolumeclaims", old=pvc("1Gi")), no_exp)


def test_pod_preset_merge_and_conflict():
    preset = {"metadata": {"name": "db", "namespace": "ns", "resourceVersion": "7"},
              "spec": {"selector": {"matchLabels": {"app": "x"}}, "env": [{"name": "DB_PORT", "value": "6379"}],
                       "volumeMounts": [{"mountPath": "/cache", "name": "cache"}], "volumes": [{"name": "cache", "emptyDir": {}}]}}
    p = pod()
    X.PodPreset().admit(attrs(p), Ctx({"podpresets": [preset]}))
    c = p["spec"]["containers"][0]
    assert c["env"] == [{"name": "DB_PORT", "value": "6379"}] and c["volumeMounts"][0]["mountPath"] == "/cache"
    assert p["spec"]["volumes"] == [{"name": "cache", "emptyDir": {}}]
    assert p["metadata"]["annotations"]["podpreset.admission.kubernetes.io/podpreset-db"] == "7"
    q = pod()
    q["spec"]["containers"][0]["env"] = [{"name": "DB_PORT", "value": "1"}]
    X.PodPreset().admit(attrs(q), Ctx({"podpresets": [preset]}))
    assert q["spec"]["containers"][0]["env"] == [{"name": "DB_PORT", "value": "1"}] and "annotations" not in q["metadata"]
    r = pod()
    r["metadata"]["labels"] = {"app": "other"}
    X.PodPreset().admit(attrs(r), Ctx({"podpresets": [preset]}))
    assert "env" not in r["spec"]["containers"][0]


def test_pod_toleration_restriction():
    ns = {"ns": {"metadata": {"name": "ns", "annotations": {
        X.NS_DEFAULT_TOLERATIONS: json.dumps([{"key": "gpu", "operator": "Exists", "effect": "NoSchedule"}]),
        X.NS_WHITELIST_TOLERATIONS: json.dumps([{"key": "gpu", "operator": "Exists", "effect": "NoSchedule"},
                                                {"key": "node.kubernetes.io/memory-pressure", "operator": "Exists",
                                                 "effect": "NoSchedule"}])}}}}
    plug = X.PodTolerationRestriction()
    p = pod()
    plug.admit(attrs(p), Ctx(namespaces=ns))
    assert p["spec"]["tolerations"] == [{"key": "gpu", "operator": "Exists", "effect": "NoSchedule"}]
    plug.validate(attrs(p), Ctx(namespaces=ns))
    g = pod()
    g["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "1"}}
    plug.admit(attrs(g), Ctx(namespaces=ns))
    assert {t["key"] for t in g["spec"]["tolerations"]} == {"gpu", "node.kubernetes.io/memory-pressure"}
    bad = pod(tolerations=[{"key": "gpu", "operator": "Equal", "value": "x", "effect": "NoSchedule"}])
    with pytest.raises(m.StatusError):
        plug.admit(attrs(bad), Ctx(namespaces=ns))
    other = pod(tolerations=[{"key": "dedicated", "operator": "Exists"}])
    with pytest.raises(m.StatusError):      # Admit ends with Validate, as the reference's does
        plug.admit(attrs(other), Ctx(namespaces=ns))
    with pytest.raises(m.StatusError):
        plug.validate(attrs(other), Ctx(namespaces=ns))


def _psp(name, **spec):
    base = {"runAsUser": {"rule": "RunAsAny"}, "seLinux": {"rule": "RunAsAny"}, "supplementalGroups": {"rule": "RunAsAny"},
            "fsGroup": {"rule": "RunAsAny"}, "volumes": ["*"]}
    base.update(spec)
    return {"apiVersion": "extensions/v1beta1", "kind": "PodSecurityPolicy", "metadata": {"name": name}, "spec": base}


def test_pod_security_policy_selection_defaulting_and_denial():
    restricted = _psp("a-restricted", runAsUser={"rule": "MustRunAs", "ranges": [{"min": 1000, "max": 2000}]},
                      fsGroup={"rule": "MustRunAs", "ranges": [{"min": 5, "max": 5}]}, requiredDropCapabilities=["NET_RAW"],
                      volumes=["emptyDir", "secret"])
    privileged = _psp("z-privileged", privileged=True, hostNetwork=True)
    ctx = Ctx({"podsecuritypolicies": [restricted, privileged]})
    plug = X.PodSecurityPolicy()
    p = pod()
    plug.admit(attrs(p), ctx)        # a policy that admits the pod unmodified wins over a mutating one
    assert p["metadata"]["annotations"][X.PSP_ANNOTATION] == "z-privileged" and "securityContext" not in p["spec"]
    only_restricted = Ctx({"podsecuritypolicies": [restricted, privileged]},
                          allow=lambda u, verb, g, res, sub, ns, name: name != "z-privileged")
    p = pod()
    plug.admit(attrs(p), only_restricted)      # defaulted into the restricted policy
    assert p["metadata"]["annotations"][X.PSP_ANNOTATION] == "a-restricted"
    sc = p["spec"]["containers"][0]["securityContext"]
    assert sc["runAsUser"] == 1000 and sc["capabilities"]["drop"] == ["NET_RAW"] and p["spec"]["securityContext"]["fsGroup"] == 5
    plug.validate(attrs(p), only_restricted)
    hp = pod(hostNetwork=True)
    plug.admit(attrs(hp), ctx)       # only the privileged policy allows host networking
    assert hp["metadata"]["annotations"][X.PSP_ANNOTATION] == "z-privileged"
    with pytest.raises(m.StatusError) as ei:
        plug.admit(attrs(pod(hostNetwork=True)), only_restricted)
    assert "unable to validate against any pod security policy" in ei.value.message
    # the pod's service account may grant the policy even when the user cannot
    sa_only = Ctx({"podsecuritypolicies": [privileged]},
                  allow=lambda u, *r: u.get("name", "").startswith("system:serviceaccount:ns:builder"))
    hp2 = pod(hostNetwork=True, serviceAccountName="builder")
    plug.admit(attrs(hp2), sa_only)
    assert hp2["metadata"]["annotations"][X.PSP_ANNOTATION] == "z-privileged"
    with pytest.raises(m.StatusError):
        plug.admit(attrs(pod(hostNetwork=True)), Ctx({"podsecuritypolicies": []}))
    X.PodSecurityPolicy(fail_on_no_policies=False).admit(attrs(pod()), Ctx({"podsecuritypolicies": []}))


def test_initializers_hide_objects_until_initialized():
    async def go():
        chain = ("NamespaceLifecycle", "Initializers")
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False,
                                api_kw={"admission_plugins": chain}) as lc:
            c = lc.client
            await c.create({"apiVersion": "admissionregistration.k8s.io/v1alpha1", "kind": "InitializerConfiguration",
                            "metadata": {"name": "cfg"}, "initializers": [{"name": "sidecar.initializer.example.com", "rules": [
                                {"apiGroups": [""], "apiVersions": ["v1"], "resources": ["configmaps"]}]}]})
            cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm", "namespace": "default"}, "data": {"a": "1"}}
            created = await c.request("POST", "/api/v1/namespaces/default/configmaps", params={"includeUninitialized": "true"},
                                      body=cm)
            assert created["metadata"]["initializers"]["pending"] == [{"name": "sidecar.initializer.example.com"}]
            assert (await c.request("GET", "/api/v1/namespaces/default/configmaps"))["items"] == []
            full = await c.request("GET", "/api/v1/namespaces/default/configmaps", params={"includeUninitialized": "true"})
            assert [m.name_of(x) for x in full["items"]] == ["cm"]
            # a blocking create returns once the initializer removed itself
            cm2 = dict(cm, metadata={"name": "cm2", "namespace": "default"})
            waiter = asyncio.create_task(c.create(cm2))
            await asyncio.sleep(0.2)
            assert not waiter.done()
            cur = await c.get("configmaps", "cm2", "default")
            cur["data"]["injected"] = "yes"
            cur["metadata"]["initializers"]["pending"] = []
            await c.update(cur)
            done = await asyncio.wait_for(waiter, 5)
            assert done["data"]["injected"] == "yes" and "initializers" not in done["metadata"]
            assert [m.name_of(x) for x in (await c.request("GET", "/api/v1/namespaces/default/configmaps"))["items"]] == ["cm2"]
    run(go(), 60)


def test_deny_escalating_exec_through_apiserver():
    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False,
                                api_kw={"admission_plugins": ("NamespaceLifecycle", "DenyEscalatingExec")}) as lc:
            p = pod("priv")
            p["metadata"]["namespace"] = "default"
            p["spec"]["containers"][0]["securityContext"] = {"privileged": True}
            await lc.client.create(p)
            with pytest.raises(m.StatusError) as ei:
                await lc.client.request("GET", "/api/v1/namespaces/default/pods/priv/exec", params={"command": "ls"})
            assert ei.value.code == 403 and "privileged" in ei.value.message
    run(go(), 30)
