"""Admission plugins against the reference's tables.

Transcribed from plugin/pkg/admission/*/admission_test.go:
  defaulttolerationseconds (TestForgivenessAdmission, TestHandles), extendedresourcetoleration
  (TestAdmit), podnodeselector (TestPodAdmission, TestHandles, TestIgnoreUpdatingInitializedPod),
  podtolerationrestriction (TestPodAdmission, with its namespace annotations carried from case to
  case as the Go test does), priority (TestPriorityClassAdmission, TestDefaultPriority,
  TestPodAdmission), storageclass/setdefault (TestAdmission), alwayspullimages, antiaffinity and
  exec (TestAdmission / TestInterPodAffinityAdmission / TestAdmission), and the namespace
  lifecycle plugin (apiserver/pkg/admission/plugin/namespace/lifecycle/admission_test.go);
  noderestriction (TestAdmit: the pod rows as a grid over pod kind, subresource and operation,
  then the unknown/unnamed pod, reference, node, unrelated-object and unrelated-user rows).
"""
from __future__ import annotations

import copy
import json

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import admission as A
from amdkube.apiserver import admission_ext as X
from amdkube.apiserver.admission import CONNECT, CREATE, DELETE, UPDATE, Attributes

NR, UR = "node.kubernetes.io/not-ready", "node.kubernetes.io/unreachable"
DNR, DUR = "node.alpha.kubernetes.io/notReady", "node.alpha.kubernetes.io/unreachable"


class Ctx:
    def __init__(self, namespaces=None, **objects):
        self.namespaces = namespaces if namespaces is not None else {}
        self.objects = objects

    def get_namespace(self, n):
        return self.namespaces.get(n)

    def list_objects(self, plural, ns, group=""):
        return list(self.objects.get(plural, []))

    def get_object(self, plural, ns, name):
        return next((o for o in self.objects.get(plural, []) if m.name_of(o) == name), None)


def _ns(name="testNamespace", **ann):
    return {name: {"metadata": {"name": name, "annotations": ann} if ann else {"name": name}}}


def _pod(name="testPod", ns="testNamespace", **spec):
    return {"metadata": {"name": name, "namespace": ns}, "spec": spec}


def _attrs(obj, op=CREATE, ns="testNamespace", name=None, old=None, resource="pods", sub="", group=""):
    return Attributes(op, resource, sub, ns, m.name_of(obj or {}) if name is None else name, obj, old, {}, group=group)


def _t(key="", op="", effect="", value="", seconds=None):
    t = {}
    for k, v in (("key", key), ("operator", op), ("value", value), ("effect", effect)):
        if v:
            t[k] = v
    if seconds is not None:
        t["tolerationSeconds"] = seconds
    return t


# ------------------------------------------------------------ DefaultTolerationSeconds
DEF_NR, DEF_UR = _t(NR, "Exists", "NoExecute", seconds=300), _t(UR, "Exists", "NoExecute", seconds=300)


@pytest.mark.parametrize("desc,given,expected", [
    ("pod has no tolerations", [], [DEF_NR, DEF_UR]),
    ("pod has alpha tolerations, untouched", [_t(DNR, "Exists", "NoExecute", seconds=300), _t(DUR, "Exists", "NoExecute", seconds=300)],
     [_t(DNR, "Exists", "NoExecute", seconds=300), _t(DUR, "Exists", "NoExecute", seconds=300), DEF_NR, DEF_UR]),
    ("pod has alpha not-ready toleration", [_t(DNR, "Exists", "NoExecute", seconds=300)],
     [_t(DNR, "Exists", "NoExecute", seconds=300), DEF_NR, DEF_UR]),
    ("pod has alpha unreachable toleration", [_t(DUR, "Exists", "NoExecute", seconds=300)],
     [_t(DUR, "Exists", "NoExecute", seconds=300), DEF_NR, DEF_UR]),
    ("pod has tolerations, none for the node taints", [_t("foo", "Equal", "NoSchedule", "bar", 700)],
     [_t("foo", "Equal", "NoSchedule", "bar", 700), DEF_NR, DEF_UR]),
    ("pod tolerates not-ready", [_t(NR, "Exists", "NoExecute", seconds=700)], [_t(NR, "Exists", "NoExecute", seconds=700), DEF_UR]),
    ("pod tolerates unreachable", [_t(UR, "Exists", "NoExecute", seconds=700)], [_t(UR, "Exists", "NoExecute", seconds=700), DEF_NR]),
    ("pod tolerates both", [_t(NR, "Exists", "NoExecute", seconds=700), _t(UR, "Exists", "NoExecute", seconds=700)],
     [_t(NR, "Exists", "NoExecute", seconds=700), _t(UR, "Exists", "NoExecute", seconds=700)]),
    ("pod tolerates unreachable with any effect", [_t(UR, "Exists", seconds=700)],
     [_t(UR, "Exists", seconds=700), DEF_NR]),
    ("pod has a wildcard toleration", [_t(op="Exists", seconds=700)], [_t(op="Exists", seconds=700)]),
])
def test_default_toleration_seconds(desc, given, expected):
    p = _pod(tolerations=copy.deepcopy(given))
    A.DefaultTolerationSeconds().admit(_attrs(p, ns="foo", name="name"), Ctx())
    assert p["spec"]["tolerations"] == expected, desc


def test_default_toleration_seconds_handles():
    h = A.DefaultTolerationSeconds()
    assert [h.handles(op) for op in (UPDATE, CREATE, DELETE, CONNECT)] == [True, True, False, False]


# --------------------------------------------------------- ExtendedResourceToleration
ER1, ER2 = "example.com/device-ek", "example.com/device-do"


def _c(*resources):
    return {"name": "c", "resources": {"requests": {r: "1" for r in resources}}} if resources else {"name": "c"}


@pytest.mark.parametrize("desc,spec,expected", [
    ("empty pod", {}, None),
    ("container without extended resources", {"containers": [{"name": "c", "resources": {"requests": {"cpu": "1"}}}]}, None),
    ("init container without extended resources", {"initContainers": [{"name": "c", "resources": {"requests": {"cpu": "1"}}}]}, None),
    ("container with an extended resource", {"containers": [_c(ER1)]}, [_t(ER1, "Exists", "NoSchedule")]),
    ("init container with an extended resource", {"initContainers": [_c(ER2)]}, [_t(ER2, "Exists", "NoSchedule")]),
    ("existing tolerations preserved", {"containers": [_c(ER1)], "tolerations": [_t("foo", "Equal", "NoSchedule", "bar")]},
     [_t("foo", "Equal", "NoSchedule", "bar"), _t(ER1, "Exists", "NoSchedule")]),
    ("multiple extended resources, sorted", {"containers": [_c(ER1)], "initContainers": [_c(ER2)]},
     [_t(ER2, "Exists", "NoSchedule"), _t(ER1, "Exists", "NoSchedule")]),
    ("existing correct toleration", {"containers": [_c(ER1)], "tolerations": [_t(ER1, "Exists", "NoSchedule")]},
     [_t(ER1, "Exists", "NoSchedule")]),
    ("same key, other effect and value", {"containers": [_c(ER1)], "tolerations": [_t(ER1, "Equal", "NoExecute", "foo")]},
     [_t(ER1, "Equal", "NoExecute", "foo"), _t(ER1, "Exists", "NoSchedule")]),
    ("wildcard toleration", {"containers": [_c(ER1)], "tolerations": [_t(op="Exists")]},
     [_t(op="Exists"), _t(ER1, "Exists", "NoSchedule")]),
])
def test_extended_resource_toleration(desc, spec, expected):
    p = _pod(**copy.deepcopy(spec))
    A.ExtendedResourceToleration().admit(_attrs(p, ns="foo", name="name"), Ctx())
    assert p["spec"].get("tolerations") == expected, desc


# -------------------------------------------------------------------- PodNodeSelector
@pytest.mark.parametrize("default,ns_sel,whitelist,pod_sel,merged,ignore_ns,admit,name", [
    ("", None, "", {}, {}, True, True, "No node selectors"),
    ("infra = false", None, "", {}, {"infra": "false"}, True, True, "Default node selector and no conflicts"),
    ("", " infra = false ", "", {}, {"infra": "false"}, False, True, "TestNamespace node selector with whitespaces and no conflicts"),
    ("infra = false", "infra=true", "", {}, {"infra": "true"}, False, True, "Default and namespace node selector, no conflicts"),
    ("infra = false", "", "", {}, {}, False, True, "Empty namespace node selector and no conflicts"),
    ("infra = false", "infra=true", "", {"env": "test"}, {"infra": "true", "env": "test"}, False, True,
     "TestNamespace and pod node selector, no conflicts"),
    ("env = test", "infra=true", "", {"infra": "false"}, None, False, False, "Conflicting pod and namespace node selector, one label"),
    ("env=dev", "infra=false, env = test", "", {"env": "dev", "color": "blue"}, None, False, False,
     "Conflicting pod and namespace node selector, multiple labels"),
    ("env=dev", "infra=false, env = dev", "env=dev, infra=false, color=blue", {"env": "dev", "color": "blue"},
     {"infra": "false", "env": "dev", "color": "blue"}, False, True, "Merged pod node selectors satisfy the whitelist"),
    ("env=dev", "infra=false, env = dev", "env=dev, infra=true, color=blue", {"env": "dev", "color": "blue"}, None, False, False,
     "Merged pod node selectors conflict with the whitelist"),
    ("env=dev", None, "env=prd", {}, None, True, False, "Default node selector conflict with the whitelist"),
])
def test_pod_node_selector(default, ns_sel, whitelist, pod_sel, merged, ignore_ns, admit, name):
    # the Go test leaves the previous case's annotation in place when a case ignores the namespace
    # selector; each of those cases decides the same without it, so a bare namespace stands in
    ctx = Ctx(_ns() if ignore_ns else _ns(**{A.PodNodeSelector.ANNOTATION: ns_sel}))
    h = A.PodNodeSelector({"clusterDefaultNodeSelector": default, "testNamespace": whitelist})
    p = _pod(nodeSelector=dict(pod_sel))
    old = _pod(nodeSelector={"old": "true"})
    old["metadata"]["initializers"] = {"pending": [{"name": "init"}]}
    for op, o in ((CREATE, None), (UPDATE, old)):      # an update of an uninitialized pod acts as a create
        for step in (h.admit, h.validate):
            if admit:
                step(_attrs(p, op, old=o), ctx)
                assert p["spec"]["nodeSelector"] == merged, name
            else:
                with pytest.raises(m.StatusError) as e:
                    step(_attrs(p, op, old=o), ctx)
                assert e.value.code == 403 and e.value.message.startswith('pods "testPod" is forbidden: pod node label selector'), name


def test_pod_node_selector_handles_and_initialized_updates():
    h = A.PodNodeSelector(None)
    assert [h.handles(op) for op in (CREATE, UPDATE, CONNECT, DELETE)] == [True, True, False, False]
    ctx = Ctx(_ns(**{A.PodNodeSelector.ANNOTATION: "infra=true"}))
    p = _pod(nodeSelector={"infra": "false"})
    h.admit(_attrs(p, UPDATE, old=copy.deepcopy(p)), ctx)      # initialized: its node selector is immutable
    assert p["spec"]["nodeSelector"] == {"infra": "false"}


# --------------------------------------------------------- PodTolerationRestriction
TK = _t("testKey", "Equal", "NoSchedule", "testValue")
TK1 = _t("testKey", "Equal", "NoSchedule", "testValue1")
TK2 = _t("testKey", "Equal", "NoSchedule", "testValue2")
MP = _t("node.kubernetes.io/memory-pressure", "Exists", "NoSchedule")
BEST_EFFORT = [{"name": "test"}]
BURSTABLE = [{"name": "test", "resources": {"limits": {"cpu": "1000m"}, "requests": {"cpu": "500m"}}}]
GUARANTEED = [{"name": "test", "resources": {"limits": {"cpu": "1000m"}, "requests": {"cpu": "1000m"}}}]

PTR_CASES = [
    (BEST_EFFORT, [TK], None, None, None, [], [TK], True, "default cluster tolerations with empty pod tolerations and nil namespace tolerations"),
    (BEST_EFFORT, [TK], [], None, None, [TK], [TK], True, "default cluster tolerations with pod tolerations specified"),
    (BEST_EFFORT, [], [TK], None, None, [TK], [TK], True, "namespace tolerations"),
    (BEST_EFFORT, [], [TK], None, None, [], [TK], True, "no pod tolerations"),
    (BEST_EFFORT, [], [TK], None, None, [TK1], None, False, "conflicting pod and namespace tolerations"),
    (BEST_EFFORT, [TK2], [], None, None, [TK1], [TK1], True,
     "conflicting pod and default cluster tolerations but overridden by empty namespace tolerations"),
    (BEST_EFFORT, [], [TK], [TK], None, [], [TK], True, "merged pod tolerations satisfy whitelist"),
    (BEST_EFFORT, [TK], [], None, None, [], [], True, "Override default cluster toleration by empty namespace level toleration"),
    (BEST_EFFORT, None, None, [], [TK1], [TK], [TK], True,
     "pod toleration conflicts with default cluster white list which is overridden by empty namespace whitelist"),
    (BEST_EFFORT, [], [TK], [TK1], None, [], None, False, "merged pod tolerations conflict with the whitelist"),
    (BURSTABLE, [], [TK], [], None, [], [MP, TK], True, "added memoryPressure/DiskPressure for Burstable pod"),
    (GUARANTEED, [], [TK], [], None, [], [MP, TK], True, "added memoryPressure/DiskPressure for Guaranteed pod"),
]


def test_pod_toleration_restriction_table():
    ns = {"metadata": {"name": "testNamespace"}}
    for containers, default, ns_tols, whitelist, cluster_wl, pod_tols, merged, admit, name in PTR_CASES:
        if ns_tols is not None:           # the Go test replaces the annotations only when a case sets them
            ns["metadata"]["annotations"] = {X.NS_DEFAULT_TOLERATIONS: json.dumps(ns_tols)}
        if whitelist is not None:
            ns["metadata"]["annotations"][X.NS_WHITELIST_TOLERATIONS] = json.dumps(whitelist)
        ctx = Ctx({"testNamespace": ns})
        h = X.PodTolerationRestriction(default or [], cluster_wl or [])
        p = _pod(containers=copy.deepcopy(containers), tolerations=copy.deepcopy(pod_tols))
        old = copy.deepcopy(p)
        old["metadata"]["initializers"] = {"pending": [{"name": "init"}]}
        old["spec"]["tolerations"] = [TK1]
        for op, o in ((CREATE, None), (UPDATE, old)):
            q = copy.deepcopy(p)
            if admit:
                h.admit(_attrs(q, op, old=o), ctx)
                assert q["spec"]["tolerations"] == merged, name
            else:
                with pytest.raises(m.StatusError) as e:
                    h.admit(_attrs(q, op, old=o), ctx)
                assert e.value.code == 500, name


def test_pod_toleration_restriction_leaves_initialized_updates_to_the_whitelist():
    ctx = Ctx(_ns(**{X.NS_DEFAULT_TOLERATIONS: json.dumps([TK])}))
    p = _pod(containers=copy.deepcopy(BEST_EFFORT))
    X.PodTolerationRestriction().admit(_attrs(p, UPDATE, old=copy.deepcopy(p)), ctx)
    assert not p["spec"].get("tolerations")


def test_pod_toleration_restriction_bad_annotation():
    ctx = Ctx(_ns(**{X.NS_DEFAULT_TOLERATIONS: "{not json"}))
    with pytest.raises(m.StatusError):
        X.PodTolerationRestriction().admit(_attrs(_pod(containers=copy.deepcopy(BEST_EFFORT))), ctx)


# ------------------------------------------------------------------------- Priority
def _pc(name, value, default=False):
    return {"apiVersion": "scheduling.k8s.io/v1alpha1", "kind": "PriorityClass", "metadata": {"name": name}, "value": value,
            "globalDefault": default}


DEFAULT1, DEFAULT2, NONDEFAULT1 = _pc("default1", 1000, True), _pc("default2", 2000, True), _pc("nondefault1", 2000)


@pytest.mark.parametrize("name,existing,new,err", [
    ("one default class", [], DEFAULT1, None),
    ("more than one default classes", [DEFAULT1], DEFAULT2,
     'priorityclasses.scheduling.k8s.io "default2" is forbidden: PriorityClass default1 is already marked as default. Only one default can exist'),
    ("too high PriorityClass value", [], _pc("toohighclass", 1000000001),
     'priorityclasses.scheduling.k8s.io "toohighclass" is forbidden: maximum allowed value of a user defined priority is 1000000000'),
    ("system name conflict", [], _pc("system-cluster-critical", 1000000001),
     'maximum allowed value of a user defined priority is 1000000000'),
    ("system name with an allowed value", [], _pc("system-node-critical", 5),
     'the name of the priority class is a reserved name for system use only: system-node-critical'),
])
def test_priority_class_admission(name, existing, new, err):
    a = _attrs(new, ns="", resource="priorityclasses", group="scheduling.k8s.io")
    if err is None:
        A.Priority().validate(a, Ctx(priorityclasses=existing))
    else:
        with pytest.raises(m.StatusError) as e:
            A.Priority().validate(a, Ctx(priorityclasses=existing))
        assert err in e.value.message and e.value.code == 403, name


def test_priority_default_class_update():
    """TestDefaultPriority's "update default class and remove its global default" and the
    update-to-the-same-default case: updating the default class itself is allowed."""
    a = _attrs(_pc("default1", 5, True), UPDATE, ns="", resource="priorityclasses", group="scheduling.k8s.io",
               old=DEFAULT1)
    A.Priority().validate(a, Ctx(priorityclasses=[DEFAULT1]))
    a = _attrs(_pc("other", 5, True), UPDATE, ns="", resource="priorityclasses", group="scheduling.k8s.io")
    with pytest.raises(m.StatusError):
        A.Priority().validate(a, Ctx(priorityclasses=[DEFAULT1]))


MIRROR = {"kubernetes.io/config.mirror": "x"}


@pytest.mark.parametrize("name,existing,spec,ann,expected,err", [
    ("Pod with priority class", [DEFAULT1, NONDEFAULT1], {"priorityClassName": "default1"}, None, 1000, None),
    ("Pod without priority class", [DEFAULT1], {}, None, 1000, None),
    ("pod without priority class and no existing priority class", [], {}, None, 0, None),
    ("pod without priority class and no default class", [NONDEFAULT1], {}, None, 0, None),
    ("pod with a system priority class", [], {"priorityClassName": "system-cluster-critical"}, None, 2000000000, None),
    ("Pod with non-existing priority class", [DEFAULT1, NONDEFAULT1], {"priorityClassName": "non-existing"}, None, None,
     (500, 'failed to get default priority class non-existing: priorityclass.scheduling.k8s.io "non-existing" not found')),
    ("pod with integer priority", [], {"priorityClassName": "default1", "priority": 1000}, None, None,
     (403, 'pods "pod-w-integer-priority" is forbidden: the integer value of priority must not be provided in pod spec.')),
    ("mirror pod with system priority class", [], {"priorityClassName": "system-cluster-critical"}, MIRROR, 2000000000, None),
    ("mirror pod with integer priority", [], {"priorityClassName": "default1", "priority": 1000}, MIRROR, None,
     (403, 'pods "pod-w-integer-priority" is forbidden: the integer value of priority must not be provided')),
])
def test_priority_pod_admission(name, existing, spec, ann, expected, err):
    p = _pod("pod-w-integer-priority", **copy.deepcopy(spec))
    if ann:
        p["metadata"]["annotations"] = dict(ann)
    if err is None:
        A.Priority().admit(_attrs(p), Ctx(priorityclasses=existing))
        assert p["spec"]["priority"] == expected, name
    else:
        with pytest.raises(m.StatusError) as e:
            A.Priority().admit(_attrs(p), Ctx(priorityclasses=existing))
        assert (e.value.code, e.value.message[:len(err[1])]) == err, name


# -------------------------------------------------------------- DefaultStorageClass
def _sc(name, ann=None):
    return {"metadata": {"name": name, "annotations": ann or {}}, "provisioner": "x"}


DEF_SC = _sc("default", {"storageclass.kubernetes.io/is-default-class": "true"})
DEF_SC2 = _sc("default2", {"storageclass.kubernetes.io/is-default-class": "true"})
BETA_SC = _sc("beta", {"storageclass.beta.kubernetes.io/is-default-class": "true"})
NOT_DEF = _sc("nondefault", {"storageclass.kubernetes.io/is-default-class": "false"})
NO_ANN = _sc("nondefault2")


@pytest.mark.parametrize("name,classes,claim_class,claim_ann,expected,err", [
    ("no default, no modification of PVCs", [NOT_DEF, NO_ANN], None, None, None, False),
    ("one default, modify PVC with class=nil", [DEF_SC, NOT_DEF, NO_ANN], None, None, "default", False),
    ("one default, no modification of PVC with class=''", [DEF_SC, NOT_DEF], "", None, "", False),
    ("one default, no modification of PVC with class='foo'", [DEF_SC, NOT_DEF], "foo", None, "foo", False),
    ("one default, no modification of PVC with the beta annotation", [DEF_SC],
     None, {"volume.beta.kubernetes.io/storage-class": ""}, None, False),
    ("two defaults, error with PVC with class=nil", [DEF_SC, DEF_SC2, NOT_DEF], None, None, None, True),
    ("two defaults, no modification with PVC with class=''", [DEF_SC, DEF_SC2], "", None, "", False),
    ("one beta default", [BETA_SC, NOT_DEF], None, None, "beta", False),
])
def test_default_storage_class(name, classes, claim_class, claim_ann, expected, err):
    pvc = {"metadata": {"name": "claimWithNoClass", "namespace": "ns"}, "spec": {}}
    if claim_class is not None:
        pvc["spec"]["storageClassName"] = claim_class
    if claim_ann:
        pvc["metadata"]["annotations"] = dict(claim_ann)
    a = _attrs(pvc, ns="ns", resource="persistentvolumeclaims")
    if err:
        with pytest.raises(m.StatusError) as e:
            A.DefaultStorageClass().admit(a, Ctx(storageclasses=classes))
        assert e.value.message == ('persistentvolumeclaims "claimWithNoClass" is forbidden: Internal error occurred: '
                                   '2 default StorageClasses were found')
    else:
        A.DefaultStorageClass().admit(a, Ctx(storageclasses=classes))
        assert pvc["spec"].get("storageClassName") == expected, name


# ------------------------------------------------ AlwaysPullImages / anti-affinity / exec
def test_always_pull_images_messages():
    p = _pod("123", containers=[{"name": "ctr1", "image": "image"}, {"name": "ctr2", "image": "image", "imagePullPolicy": "Never"}],
             initContainers=[{"name": "init1", "image": "image", "imagePullPolicy": "IfNotPresent"}])
    a = _attrs(p, name="123")
    with pytest.raises(m.StatusError) as e:
        X.AlwaysPullImages().validate(a, Ctx())
    assert e.value.message == ('pods "123" is forbidden: spec.initContainers[0].imagePullPolicy: Unsupported value: '
                               '"IfNotPresent": supported values: "Always"')
    X.AlwaysPullImages().admit(a, Ctx())
    X.AlwaysPullImages().validate(a, Ctx())
    assert {c["imagePullPolicy"] for c in p["spec"]["containers"] + p["spec"]["initContainers"]} == {"Always"}
    # other resources and subresources are ignored
    X.AlwaysPullImages().validate(_attrs(_pod(containers=[{"name": "c"}]), sub="exec"), Ctx())
    X.AlwaysPullImages().validate(_attrs({"metadata": {"name": "x"}}, resource="services"), Ctx())


def _anti(*keys):
    return {"affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchExpressions": [{"key": "security", "operator": "In", "values": ["S2"]}]}, "topologyKey": k}
        for k in keys]}}}


@pytest.mark.parametrize("spec,ok", [
    (_anti("kubernetes.io/hostname"), True),
    (_anti("failure-domain.beta.kubernetes.io/zone"), False),
    (_anti("kubernetes.io/hostname", "failure-domain.beta.kubernetes.io/zone"), False),
    ({"affinity": {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 10, "podAffinityTerm": {"topologyKey": "failure-domain.beta.kubernetes.io/zone"}}]}}}, True),
    ({"affinity": {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"topologyKey": "failure-domain.beta.kubernetes.io/zone"}]}}}, True),
    ({}, True),
])
def test_inter_pod_affinity_admission(spec, ok):
    p = _pod(**copy.deepcopy(spec))
    if ok:
        X.LimitPodHardAntiAffinityTopology().validate(_attrs(p), Ctx())
    else:
        with pytest.raises(m.StatusError) as e:
            X.LimitPodHardAntiAffinityTopology().validate(_attrs(p), Ctx())
        assert e.value.message == ('pods "testPod" is forbidden: affinity.PodAntiAffinity.RequiredDuringScheduling has '
                                   'TopologyKey failure-domain.beta.kubernetes.io/zone but only key kubernetes.io/hostname is allowed')


@pytest.mark.parametrize("spec,escalating,on_privileged", [
    ({"hostPID": True}, "cannot exec into or attach to a container using host pid", None),
    ({"hostIPC": True}, "cannot exec into or attach to a container using host ipc", None),
    ({"containers": [{"name": "c", "securityContext": {"privileged": True}}]}, "cannot exec into or attach to a privileged container",
     "cannot exec into or attach to a privileged container"),
    ({"initContainers": [{"name": "i", "securityContext": {"privileged": True}}]},
     "cannot exec into or attach to a privileged container", "cannot exec into or attach to a privileged container"),
    ({"containers": [{"name": "c", "securityContext": {"privileged": False}}]}, None, None),
    ({}, None, None),
])
def test_deny_exec(spec, escalating, on_privileged):
    ctx = Ctx(pods=[_pod("pod", **spec)])
    for plug, msg in ((X.DenyEscalatingExec(), escalating), (X.DenyExecOnPrivileged(), on_privileged)):
        for sub in ("exec", "attach"):
            a = Attributes(CONNECT, "pods", sub, "testNamespace", "pod", None, None, {})
            if msg is None:
                plug.validate(a, ctx)
            else:
                with pytest.raises(m.StatusError) as e:
                    plug.validate(a, ctx)
                assert e.value.message == f'pods "pod" is forbidden: {msg}'
    # portforward is not exec or attach
    X.DenyEscalatingExec().validate(Attributes(CONNECT, "pods", "portforward", "testNamespace", "pod", None, None, {}), ctx)


# ------------------------------------------------------------------ NamespaceLifecycle
def test_namespace_lifecycle():
    h = A.NamespaceLifecycle()
    active = {"metadata": {"name": "test"}, "status": {"phase": "Active"}}
    terminating = {"metadata": {"name": "test"}, "status": {"phase": "Terminating"}}
    pod = _pod("123", ns="test", containers=[{"name": "ctr", "image": "image"}])
    h.validate(_attrs(pod, ns="test"), Ctx({"test": active}))
    with pytest.raises(m.StatusError) as e:
        h.validate(_attrs(pod, ns="test"), Ctx({"test": terminating}))
    assert e.value.message == ('pods "123" is forbidden: unable to create new content in namespace test because it is '
                               'being terminated.')
    # updates and deletes in a terminating namespace are allowed (finalization needs them)
    h.validate(_attrs(pod, UPDATE, ns="test", old=pod), Ctx({"test": terminating}))
    h.validate(_attrs(pod, DELETE, ns="test"), Ctx({"test": terminating}))
    # subresources are not exempt: a binding in a terminating namespace is refused
    with pytest.raises(m.StatusError):
        h.validate(_attrs({"metadata": {"name": "123"}}, ns="test", sub="binding"), Ctx({"test": terminating}))
    # a missing namespace
    with pytest.raises(m.StatusError) as e:
        h.validate(_attrs(pod, ns="missing"), Ctx({}))
    assert e.value.code == 404 and e.value.message == 'namespaces "missing" not found'
    # access reviews skip the lookup; cluster-scoped objects too
    h.validate(_attrs({"metadata": {}}, ns="missing", resource="localsubjectaccessreviews", group="authorization.k8s.io"), Ctx({}))
    h.validate(_attrs({"metadata": {"name": "n"}}, ns="", resource="nodes"), Ctx({}))


@pytest.mark.parametrize("ns,ok", [("default", False), ("kube-system", False), ("kube-public", False), ("other", True)])
def test_namespace_lifecycle_immortal(ns, ok):
    a = _attrs(None, DELETE, ns="", name=ns, resource="namespaces")
    if ok:
        A.NamespaceLifecycle().validate(a, Ctx())
    else:
        with pytest.raises(m.StatusError) as e:
            A.NamespaceLifecycle().validate(a, Ctx())
        assert e.value.message == f'namespaces "{ns}" is forbidden: this namespace may not be deleted'


# -------------------------------------------------------------------- NodeRestriction
MYNODE = {"name": "system:node:mynode", "groups": ["system:nodes"]}
BOB = {"name": "bob", "groups": []}


def _nr_pod(name, node, mirror):
    p = {"metadata": {"name": name, "namespace": "ns"}, "spec": {"nodeName": node} if node else {}}
    if mirror:
        p["metadata"]["annotations"] = {"kubernetes.io/config.mirror": ""}
    return p


NR_PODS = {"mirrorpod-self": _nr_pod("mymirrorpod", "mynode", True), "mirrorpod-other": _nr_pod("othermirrorpod", "othernode", True),
           "mirrorpod-unbound": _nr_pod("unboundmirrorpod", "", True), "pod-self": _nr_pod("mypod", "mynode", False),
           "pod-other": _nr_pod("otherpod", "othernode", False), "pod-unbound": _nr_pod("unboundpod", "", False)}


def _nr_expect(kind, sub, op):
    """The TestAdmit rows for one pod kind, subresource and operation (admission_test.go:113-477)."""
    bound_self = kind.endswith("-self")
    if sub == "":
        if op == CREATE:
            if not kind.startswith("mirror"):
                return "can only create mirror pods"
            return "" if bound_self else "spec.nodeName set to itself"
        if op == UPDATE:
            return "forbidden: unexpected operation"
        return "" if bound_self else "spec.nodeName set to itself"
    if sub == "status":
        if op == UPDATE:
            return "" if bound_self else "spec.nodeName set to itself"
        return "forbidden: unexpected operation"
    if op == CREATE:
        return "" if bound_self else "spec.nodeName set to itself"
    return "forbidden: unexpected operation"


NR_GRID = [(k, sub, op, unnamed) for k in NR_PODS for sub in ("", "status", "eviction")
           for op in ((CREATE, UPDATE, DELETE)) for unnamed in ((False, True) if sub == "eviction" and op == CREATE else (False,))]


@pytest.mark.parametrize("kind,sub,op,unnamed", NR_GRID)
def test_node_restriction_pods(kind, sub, op, unnamed):
    pod = NR_PODS[kind]
    ctx = Ctx(pods=list(NR_PODS.values()))
    if sub == "eviction":
        obj = {"metadata": {} if unnamed else {"name": m.name_of(pod), "namespace": "ns"}}
    else:
        obj = None if op == DELETE else copy.deepcopy(pod)
    old = copy.deepcopy(pod) if op == UPDATE else None
    a = Attributes(op, "pods", sub, "ns", m.name_of(pod), obj, old, MYNODE)
    want = _nr_expect(kind, sub, op)
    if not want:
        A.NodeRestriction().admit(a, ctx)
    else:
        with pytest.raises(m.StatusError) as e:
            A.NodeRestriction().admit(a, ctx)
        assert want in f"{e.value.reason.lower()}: {e.value.message}" or want in e.value.message


CONFIG_A = {"configMapRef": {"name": "foo", "namespace": "bar", "uid": "fooUID"}}
CONFIG_B = {"configMapRef": {"name": "qux", "namespace": "bar", "uid": "quxUID"}}


def _node(name, cs=None):
    return {"metadata": {"name": name}, "spec": {"configSource": cs} if cs else {}}


@pytest.mark.parametrize("name,resource,sub,op,obj,old,aname,user,err", [
    ("forbid delete of unknown pod", "pods", "", DELETE, None, None, "unknown", MYNODE, "not found"),
    ("forbid create of eviction for unknown pod", "pods", "eviction", CREATE, {"metadata": {"name": "unknown"}}, None, "unknown",
     MYNODE, "not found"),
    ("forbid create of unnamed eviction for unknown pod", "pods", "eviction", CREATE, {"metadata": {}}, None, "unknown", MYNODE,
     "not found"),
    ("allow create of eviction for unnamed pod", "pods", "eviction", CREATE, {"metadata": {"name": "mypod"}}, None, "", MYNODE, ""),
    ("forbid create of unnamed eviction for unnamed pod", "pods", "eviction", CREATE, {"metadata": {}}, None, "", MYNODE,
     "could not determine pod from request data"),
    ("forbid create of pod referencing service account", "pods", "", CREATE,
     {**_nr_pod("sapod", "mynode", True), "spec": {"nodeName": "mynode", "serviceAccountName": "foo"}}, None, "sapod", MYNODE,
     "reference a service account"),
    ("forbid create of pod referencing secret", "pods", "", CREATE,
     {**_nr_pod("secretpod", "mynode", True), "spec": {"nodeName": "mynode", "volumes": [{"name": "v", "secret": {"secretName": "foo"}}]}},
     None, "secretpod", MYNODE, "reference secrets"),
    ("forbid create of pod referencing an env secret", "pods", "", CREATE,
     {**_nr_pod("secretpod", "mynode", True), "spec": {"nodeName": "mynode", "containers": [
         {"name": "c", "env": [{"name": "X", "valueFrom": {"secretKeyRef": {"name": "s", "key": "k"}}}]}]}},
     None, "secretpod", MYNODE, "reference secrets"),
    ("forbid create of pod referencing configmap", "pods", "", CREATE,
     {**_nr_pod("cmpod", "mynode", True), "spec": {"nodeName": "mynode", "volumes": [{"name": "v", "configMap": {"name": "foo"}}]}},
     None, "cmpod", MYNODE, "reference configmaps"),
    ("forbid create of pod referencing persistentvolumeclaim", "pods", "", CREATE,
     {**_nr_pod("pvcpod", "mynode", True), "spec": {"nodeName": "mynode", "volumes": [
         {"name": "v", "persistentVolumeClaim": {"claimName": "foo"}}]}}, None, "pvcpod", MYNODE, "reference persistentvolumeclaims"),
    ("allow create of my node", "nodes", "", CREATE, _node("mynode"), None, "mynode", MYNODE, ""),
    ("allow create of my node pulling name from object", "nodes", "", CREATE, _node("mynode"), None, "", MYNODE, ""),
    ("allow update of my node", "nodes", "", UPDATE, _node("mynode"), _node("mynode"), "mynode", MYNODE, ""),
    ("allow delete of my node", "nodes", "", DELETE, None, None, "mynode", MYNODE, ""),
    ("allow update of my node status", "nodes", "status", UPDATE, _node("mynode"), _node("mynode"), "mynode", MYNODE, ""),
    ("forbid create of my node with non-nil configSource", "nodes", "", CREATE, _node("mynode", CONFIG_A), None, "mynode", MYNODE,
     "create with non-nil configSource"),
    ("forbid update of my node: nil configSource to new non-nil configSource", "nodes", "", UPDATE, _node("mynode", CONFIG_A),
     _node("mynode"), "mynode", MYNODE, "update configSource to a new non-nil configSource"),
    ("forbid update of my node: non-nil configSource to new non-nil configSource", "nodes", "", UPDATE, _node("mynode", CONFIG_B),
     _node("mynode", CONFIG_A), "mynode", MYNODE, "update configSource to a new non-nil configSource"),
    ("allow update of my node: non-nil configSource unchanged", "nodes", "", UPDATE, _node("mynode", CONFIG_A),
     _node("mynode", CONFIG_A), "mynode", MYNODE, ""),
    ("allow update of my node: non-nil configSource to nil configSource", "nodes", "", UPDATE, _node("mynode"),
     _node("mynode", CONFIG_A), "mynode", MYNODE, ""),
    ("forbid create of other node", "nodes", "", CREATE, _node("othernode"), None, "othernode", MYNODE, "cannot modify node"),
    ("forbid create of other node pulling name from object", "nodes", "", CREATE, _node("othernode"), None, "", MYNODE,
     "cannot modify node"),
    ("forbid update of other node", "nodes", "", UPDATE, _node("othernode"), _node("othernode"), "othernode", MYNODE, "cannot modify node"),
    ("forbid delete of other node", "nodes", "", DELETE, None, None, "othernode", MYNODE, "cannot modify node"),
    ("forbid update of other node status", "nodes", "status", UPDATE, _node("othernode"), _node("othernode"), "othernode", MYNODE,
     "cannot modify node"),
    ("allow create of unrelated object", "configmaps", "", CREATE, {"metadata": {}}, None, "mycm", MYNODE, ""),
    ("allow update of unrelated object", "configmaps", "", UPDATE, {"metadata": {}}, {"metadata": {}}, "mycm", MYNODE, ""),
    ("allow delete of unrelated object", "configmaps", "", DELETE, None, None, "mycm", MYNODE, ""),
    ("allow unrelated user creating a normal pod unbound", "pods", "", CREATE, _nr_pod("unboundpod", "", False), None, "unboundpod",
     BOB, ""),
    ("allow unrelated user update of normal pod unbound", "pods", "", UPDATE, _nr_pod("unboundpod", "", False),
     _nr_pod("unboundpod", "", False), "unboundpod", BOB, ""),
    ("allow unrelated user delete of normal pod status unbound", "pods", "status", DELETE, None, None, "unboundpod", BOB, ""),
    ("forbid a node user without a node name", "pods", "", CREATE, _nr_pod("x", "", True), None, "x",
     {"name": "system:node:", "groups": ["system:nodes"]}, 'could not determine node from user "system:node:"'),
    ("a node name without the nodes group is not a node", "nodes", "", UPDATE, _node("othernode"), _node("othernode"), "othernode",
     {"name": "system:node:mynode", "groups": []}, ""),
    ("forbid a claim spec update by a node", "persistentvolumeclaims", "", UPDATE, {"metadata": {"name": "c"}},
     {"metadata": {"name": "c"}}, "c", MYNODE, "may only update PVC status"),
])
def test_node_restriction_table(name, resource, sub, op, obj, old, aname, user, err):
    ctx = Ctx(pods=list(NR_PODS.values()))
    a = Attributes(op, resource, sub, "ns", aname, copy.deepcopy(obj), copy.deepcopy(old), user)
    if not err:
        A.NodeRestriction().admit(a, ctx)
    else:
        with pytest.raises(m.StatusError) as e:
            A.NodeRestriction().admit(a, ctx)
        assert err in e.value.message, name


@pytest.mark.parametrize("expand,new_status,err", [
    (False, {"capacity": {"storage": "2Gi"}}, 'node "mynode" may not update persistentvolumeclaim metadata'),
    (True, {"capacity": {"storage": "2Gi"}, "conditions": [{"type": "Resizing", "status": "True"}]}, ""),
    (True, {"phase": "Lost"}, 'node "mynode" may not update fields other than status.capacity and status.conditions'),
])
def test_node_restriction_claim_status(expand, new_status, err):
    old = {"metadata": {"name": "c", "resourceVersion": "1"}, "spec": {"volumeName": "v"}, "status": {"phase": "Bound"}}
    new = copy.deepcopy(old)
    new["metadata"]["resourceVersion"] = "2"
    new["status"].update(new_status)
    a = Attributes(UPDATE, "persistentvolumeclaims", "status", "ns", "c", new, old, MYNODE)
    if err:
        with pytest.raises(m.StatusError) as e:
            A.NodeRestriction(expand_persistent_volumes=expand).admit(a, Ctx())
        assert err in e.value.message
    else:
        A.NodeRestriction(expand_persistent_volumes=expand).admit(a, Ctx())


# --------------------------------------------------------------------- ServiceAccount
TOKEN_PATH = "/var/run/secrets/kubernetes.io/serviceaccount"


def _sa(name="default", uid="12345", secrets=(), pulls=(), ann=None, ns="myns"):
    md = {"name": name, "namespace": ns, "uid": uid}
    if ann:
        md["annotations"] = ann
    return {"metadata": md, "secrets": [{"name": s} for s in secrets], "imagePullSecrets": [{"name": s} for s in pulls]}


def _token(name, sa="default", uid="12345", type_="kubernetes.io/service-account-token", ns="myns"):
    return {"metadata": {"name": name, "namespace": ns, "annotations": {
        "kubernetes.io/service-account.name": sa, "kubernetes.io/service-account.uid": uid}}, "type": type_}


def _sa_attrs(pod, op=CREATE, old=None, resource="pods"):
    return Attributes(op, resource, "", "myns", "myname", pod, old, {})


def test_service_account_ignores():
    h = A.ServiceAccount()
    assert not h.handles(DELETE) and not h.handles(CONNECT) and h.handles(CREATE) and h.handles(UPDATE)
    pod, old = {"spec": {}}, {"spec": {}}
    h.admit(_sa_attrs(pod, UPDATE, old), Ctx())                      # update of an initialized pod
    assert "serviceAccountName" not in pod["spec"]
    h.admit(_sa_attrs({"spec": {}}, resource="configmaps"), Ctx())   # not a pod resource
    h.admit(_sa_attrs(None), Ctx())                                  # nil object
    h.admit(_sa_attrs({"kind": "Binding", "target": {}}), Ctx())     # not a pod object
    mirror = {"metadata": {"annotations": {"kubernetes.io/config.mirror": "true"}}, "spec": {"containers": [{}]}}
    h.admit(_sa_attrs(mirror), Ctx())
    assert "serviceAccountName" not in mirror["spec"]


@pytest.mark.parametrize("spec,msg", [
    ({"serviceAccountName": "default"}, "a mirror pod may not reference service accounts"),
    ({"volumes": [{"name": "v", "secret": {"secretName": "mysecret"}}]}, "a mirror pod may not reference secrets"),
    ({"imagePullSecrets": [{"name": "pull"}]}, "a mirror pod may not reference secrets"),
])
def test_service_account_rejects_mirror_pods(spec, msg):
    pod = {"metadata": {"annotations": {"kubernetes.io/config.mirror": "true"}}, "spec": spec}
    with pytest.raises(m.StatusError) as e:
        A.ServiceAccount().admit(_sa_attrs(pod), Ctx())
    assert e.value.message == f'pods "myname" is forbidden: {msg}'


def test_service_account_missing_token():
    ctx = Ctx(serviceaccounts=[_sa()])
    pod = {"spec": {"containers": [{}]}}
    A.ServiceAccount().admit(_sa_attrs(pod), ctx)                    # tolerates a missing API token
    assert pod["spec"]["serviceAccountName"] == "default" and not pod["spec"].get("volumes")
    with pytest.raises(m.StatusError) as e:
        A.ServiceAccount(require_api_token=True).admit(_sa_attrs({"spec": {"containers": [{}]}}), ctx)
    assert e.value.code == 504 and e.value.reason == "ServerTimeout"
    assert e.value.message == ('No API token found for service account "default", retry after the token is automatically '
                               'created and added to the service account')


def test_service_account_denies_invalid_service_account():
    with pytest.raises(m.StatusError) as e:
        A.ServiceAccount().admit(_sa_attrs({"spec": {"serviceAccountName": "other", "containers": [{}]}}), Ctx())
    assert e.value.message == ('pods "myname" is forbidden: error looking up service account myns/other: serviceaccount '
                               '"other" not found')


def test_service_account_automounts_api_token():
    ctx = Ctx(serviceaccounts=[_sa(secrets=["token-name"])], secrets=[_token("token-name")])
    want_vol = {"name": "token-name", "secret": {"secretName": "token-name"}}
    want_mount = {"name": "token-name", "readOnly": True, "mountPath": TOKEN_PATH}
    h = A.ServiceAccount(require_api_token=True)
    pod = {"spec": {"containers": [{}]}}
    h.admit(_sa_attrs(pod), ctx)
    assert pod["spec"]["volumes"] == [want_vol] and pod["spec"]["containers"][0]["volumeMounts"] == [want_mount]
    # an update of an uninitialized pod is admitted like a create; the old pod's mounts do not count
    old = {"metadata": {"initializers": {"pending": [{"name": "init"}]}},
           "spec": {"containers": [{"volumeMounts": [{"name": "wrong-token-name", "readOnly": True, "mountPath": TOKEN_PATH}]}]}}
    pod = {"spec": {"containers": [{}]}}
    h.admit(_sa_attrs(pod, UPDATE, old), ctx)
    assert pod["spec"]["volumes"] == [want_vol] and pod["spec"]["containers"][0]["volumeMounts"] == [want_mount]
    # init containers get the mount too
    pod = {"spec": {"initContainers": [{}], "containers": [{}]}}
    h.admit(_sa_attrs(pod), ctx)
    assert pod["spec"]["initContainers"][0]["volumeMounts"] == [want_mount] and len(pod["spec"]["volumes"]) == 1


def test_service_account_respects_existing_mount():
    ctx = Ctx(serviceaccounts=[_sa(secrets=["token-name"])], secrets=[_token("token-name")])
    mine = {"name": "my-custom-mount", "readOnly": False, "mountPath": TOKEN_PATH}
    pod = {"spec": {"containers": [{"volumeMounts": [dict(mine)]}]}}
    A.ServiceAccount(require_api_token=True).admit(_sa_attrs(pod), ctx)
    assert pod["spec"]["containers"][0]["volumeMounts"] == [mine] and not pod["spec"].get("volumes")


def test_service_account_token_volume_name_collision():
    ctx = Ctx(serviceaccounts=[_sa(secrets=["token-name"])], secrets=[_token("token-name")])
    pod = {"spec": {"containers": [{}], "volumes": [{"name": "token-name", "emptyDir": {}}]}}
    A.ServiceAccount().admit(_sa_attrs(pod), ctx)
    vol = pod["spec"]["volumes"][1]
    assert vol["name"].startswith("token-name-") and vol["secret"] == {"secretName": "token-name"}
    assert pod["spec"]["containers"][0]["volumeMounts"][0]["name"] == vol["name"]


ENFORCE = {"kubernetes.io/enforce-mountable-secrets": "true"}


@pytest.mark.parametrize("spec", [
    {"volumes": [{"name": "foo", "secret": {"secretName": "foo"}}], "containers": [{}]},
    {"initContainers": [{"name": "container-1", "env": [{"name": "env-1", "valueFrom": {"secretKeyRef": {"name": "foo"}}}]}]},
    {"containers": [{"name": "container-1", "env": [{"name": "env-1", "valueFrom": {"secretKeyRef": {"name": "foo"}}}]}]},
])
def test_service_account_allows_referenced_secret(spec):
    ctx = Ctx(serviceaccounts=[_sa(secrets=["foo"], ann=ENFORCE)])
    A.ServiceAccount().admit(_sa_attrs({"spec": copy.deepcopy(spec)}), ctx)


@pytest.mark.parametrize("spec,msg", [
    ({"volumes": [{"name": "foo", "secret": {"secretName": "foo"}}], "containers": [{}]},
     'volume with secret.secretName="foo" is not allowed because service account default does not reference that secret'),
    ({"initContainers": [{"name": "container-1", "env": [{"name": "env-1", "valueFrom": {"secretKeyRef": {"name": "foo"}}}]}]},
     'init container container-1 with envVar env-1 referencing secret.secretName="foo" is not allowed because service account '
     'default does not reference that secret'),
    ({"containers": [{"name": "container-2", "env": [{"name": "env-1", "valueFrom": {"secretKeyRef": {"name": "foo"}}}]}]},
     'container container-2 with envVar env-1 referencing secret.secretName="foo" is not allowed because service account '
     'default does not reference that secret'),
])
def test_service_account_rejects_unreferenced_secrets(spec, msg):
    ctx = Ctx(serviceaccounts=[_sa(ann=ENFORCE)])
    with pytest.raises(m.StatusError) as e:
        A.ServiceAccount().admit(_sa_attrs({"spec": copy.deepcopy(spec)}), ctx)
    assert e.value.message == f'pods "myname" is forbidden: {msg}'
    # a permissive account (annotation false or absent) allows them; LimitSecretReferences enforces for all
    A.ServiceAccount().admit(_sa_attrs({"spec": copy.deepcopy(spec)}),
                             Ctx(serviceaccounts=[_sa(ann={"kubernetes.io/enforce-mountable-secrets": "false"})]))
    with pytest.raises(m.StatusError):
        A.ServiceAccount(limit_secret_references=True).admit(_sa_attrs({"spec": copy.deepcopy(spec)}), Ctx(serviceaccounts=[_sa()]))


def test_service_account_image_pull_secrets():
    enforce = Ctx(serviceaccounts=[_sa(pulls=["foo"], ann=ENFORCE)])
    A.ServiceAccount().admit(_sa_attrs({"spec": {"imagePullSecrets": [{"name": "foo"}]}}), enforce)
    with pytest.raises(m.StatusError) as e:
        A.ServiceAccount().admit(_sa_attrs({"spec": {"imagePullSecrets": [{"name": "bar"}]}}), enforce)
    assert e.value.message == ('pods "myname" is forbidden: imagePullSecrets[0].name="bar" is not allowed because service '
                               'account default does not reference that imagePullSecret')
    ctx = Ctx(serviceaccounts=[_sa(pulls=["foo", "bar"])])
    pod = {"spec": {"imagePullSecrets": [{"name": "lalala"}]}}          # TestDoNotAddImagePullSecrets
    A.ServiceAccount().admit(_sa_attrs(pod), ctx)
    assert pod["spec"]["imagePullSecrets"] == [{"name": "lalala"}]
    pod = {"spec": {}}                                                  # TestAddImagePullSecrets
    A.ServiceAccount().admit(_sa_attrs(pod), ctx)
    assert pod["spec"]["imagePullSecrets"] == [{"name": "foo"}, {"name": "bar"}]


def test_service_account_multiple_referenced_secrets():
    ctx = Ctx(serviceaccounts=[_sa("mysa", "mysauid", secrets=["token1", "token2"])],
              secrets=[_token("token2", "mysa", "mysauid"), _token("token1", "mysa", "mysauid")])
    pod = {"spec": {"serviceAccountName": "mysa", "containers": [{"name": "container-1"}]}}
    A.ServiceAccount(require_api_token=True).admit(_sa_attrs(pod), ctx)
    assert [v["name"] for v in pod["spec"]["volumes"]] == ["token1"]


def test_get_service_account_tokens():
    sa = _sa(ns="namespace")
    secrets = [_token("nonSATokenSecret", type_="kubernetes.io/dockercfg", ns="namespace"),
               _token("differentSAToken", sa="someOtherSA", ns="namespace"),
               _token("differentUID", uid="someOtherUID", ns="namespace"),
               _token("matchingSAToken", ns="namespace")]
    got = A.ServiceAccount.service_account_tokens(sa, Ctx(secrets=secrets))
    assert [m.name_of(s) for s in got] == ["matchingSAToken"]


# -------------------------------------------------------------------------- PodPreset
def _pp(name="hello", **spec):
    return {"metadata": {"name": name, "namespace": "namespace", "resourceVersion": "1"},
            "spec": {"selector": {"matchExpressions": [{"key": "security", "operator": "In", "values": ["S2"]}]}, **spec}}


def _env(*kv):
    return [{"name": k, "value": v} for k, v in kv]


def _vm(*np):
    return [{"name": n, "mountPath": p} for n, p in np]


@pytest.mark.parametrize("field,keys,what,orig,mod,result", [
    ("env", ("name",), "env", None, _env(("abc", "value2"), ("ABC", "value3")), _env(("abc", "value2"), ("ABC", "value3"))),
    ("env", ("name",), "env", _env(("abcd", "value2"), ("hello", "value3")), _env(("abc", "value2"), ("ABC", "value3")),
     _env(("abcd", "value2"), ("hello", "value3"), ("abc", "value2"), ("ABC", "value3"))),
    ("env", ("name",), "env", _env(("abc", "value3")), _env(("abc", "value2"), ("ABC", "value3")), None),
    ("env", ("name",), "env", _env(("abc", "value2"), ("hello", "value3")), _env(("abc", "value2"), ("ABC", "value3")),
     _env(("abc", "value2"), ("hello", "value3"), ("ABC", "value3"))),
    ("volumeMounts", ("name", "mountPath"), "volume mounts", None, _vm(("simply-mounted-volume", "/opt/")),
     _vm(("simply-mounted-volume", "/opt/"))),
    ("volumeMounts", ("name", "mountPath"), "volume mounts", _vm(("etc-volume", "/etc/")), _vm(("simply-mounted-volume", "/opt/")),
     _vm(("etc-volume", "/etc/"), ("simply-mounted-volume", "/opt/"))),
    ("volumeMounts", ("name", "mountPath"), "volume mounts", _vm(("etc-volume", "/etc/")),
     _vm(("simply-mounted-volume", "/opt/"), ("etc-volume", "/things/")), None),                     # conflict on name
    ("volumeMounts", ("name", "mountPath"), "volume mounts", _vm(("etc-volume", "/etc/")),
     _vm(("simply-mounted-volume", "/opt/"), ("things-volume", "/etc/")), None),                     # conflict on mount path
    ("volumeMounts", ("name", "mountPath"), "volume mounts", _vm(("etc-volume", "/etc/")),
     _vm(("simply-mounted-volume", "/opt/"), ("etc-volume", "/etc/")), _vm(("etc-volume", "/etc/"), ("simply-mounted-volume", "/opt/"))),
    ("volumes", ("name",), "volumes", None, [{"name": "vol", "emptyDir": {}}], [{"name": "vol", "emptyDir": {}}]),
    ("volumes", ("name",), "volumes", [{"name": "etc-volume", "hostPath": {"path": "/etc"}}], [{"name": "vol", "emptyDir": {}}],
     [{"name": "etc-volume", "hostPath": {"path": "/etc"}}, {"name": "vol", "emptyDir": {}}]),
    ("volumes", ("name",), "volumes", [{"name": "vol", "hostPath": {"path": "/etc"}}], [{"name": "vol", "emptyDir": {}}], None),
    ("volumes", ("name",), "volumes", [{"name": "vol", "emptyDir": {}}], [{"name": "vol", "emptyDir": {}}],
     [{"name": "vol", "emptyDir": {}}]),
])
def test_pod_preset_merges(field, keys, what, orig, mod, result):
    merged, errs = X.PodPreset._merge_by(orig, [_pp(**{field: mod})], field, keys, what)
    if result is None:
        assert errs and errs[0].startswith(f"merging {what} for hello has a conflict on")
    else:
        assert not errs and merged == result


def test_pod_preset_env_from_is_appended():
    cm = {"configMapRef": {"name": "abc"}}
    pod = {"metadata": {"name": "mypod", "labels": {"security": "S2"}}, "spec": {"containers": [
        {"name": "c", "envFrom": [{"configMapRef": {"name": "thing"}}]}]}}
    X.PodPreset.apply(pod, [_pp(envFrom=[cm, {"prefix": "pre_", **cm}])])
    assert pod["spec"]["containers"][0]["envFrom"] == [{"configMapRef": {"name": "thing"}}, cm, {"prefix": "pre_", **cm}]


def _preset_pod(labels=None, ann=None):
    md = {"name": "mypod", "namespace": "namespace", "labels": labels if labels is not None else {"security": "S2"}}
    if ann:
        md["annotations"] = ann
    return {"metadata": md, "spec": {"containers": [{"name": "mycontainer", "image": "image",
                                                     "env": _env(("abc", "value2"), ("ABC", "value3"))}]}}


def _preset_admit(pod, presets, ns="namespace"):
    ctx = Ctx(podpresets=presets)
    ctx.list_objects = lambda plural, n, group="": [p for p in presets if m.namespace_of(p) == n]
    X.PodPreset().admit(Attributes(CREATE, "pods", "", ns, "mypod", pod, None, {}), ctx)


def test_pod_preset_admit():
    good = _pp(env=_env(("abcd", "value")), volumeMounts=_vm(("etc-volume", "/etc/")),
               volumes=[{"name": "etc-volume", "hostPath": {"path": "/etc"}}], envFrom=[{"configMapRef": {"name": "abc"}}])
    pod = _preset_pod()
    _preset_admit(pod, [good])                                                        # TestAdmit
    c = pod["spec"]["containers"][0]
    assert c["env"] == _env(("abc", "value2"), ("ABC", "value3"), ("abcd", "value"))
    assert c["volumeMounts"] == _vm(("etc-volume", "/etc/")) and c["envFrom"] == [{"configMapRef": {"name": "abc"}}]
    assert pod["spec"]["volumes"] == [{"name": "etc-volume", "hostPath": {"path": "/etc"}}]
    assert pod["metadata"]["annotations"] == {"podpreset.admission.kubernetes.io/podpreset-hello": "1"}
    conflicting = _pp(env=_env(("abc", "value")))
    for pod, presets, ns in ((_preset_pod(), [conflicting], "othernamespace"),              # DifferentNamespaceShouldDoNothing
                             (_preset_pod(labels={"security": "S1"}), [conflicting], "namespace"),   # NonMatchingLabels
                             (_preset_pod(), [conflicting], "namespace"),                   # ConflictShouldNotModifyPod
                             (_preset_pod(ann={"kubernetes.io/config.mirror": "mirror"}), [good], "namespace"),   # MirrorPod
                             (_preset_pod(ann={"podpreset.admission.kubernetes.io/exclude": "true"}), [good], "namespace")):
        before = copy.deepcopy(pod)
        _preset_admit(pod, presets, ns)
        assert pod == before


# --------------------------------------------------------------------- EventRateLimit
def _rq(kind="Event", ns="", user="", event=None, delay=0, ok=True):
    return (kind, ns, user, event, delay, ok)


def _soi(factory):
    """createSourceAndObjectKeyInclusionRequests."""
    return [_rq(event=factory("A")), _rq(event=factory("A"), ok=False), _rq(event=factory("B"))]


def _comp(c):
    return {"source": {"component": c}}


NS_A, NS_B = "A", "B"
ERL_CASES = [
    ("event not blocked when tokens available", dict(server=3), [_rq()]),
    ("non-event not blocked", dict(server=3), [_rq("NonEvent")]),
    ("event blocked after tokens exhausted", dict(server=3), [_rq(), _rq(), _rq(), _rq(ok=False)]),
    ("non-event not blocked after tokens exhausted", dict(server=3), [_rq(), _rq(), _rq(), _rq("NonEvent")]),
    ("non-events should not count against limit", dict(server=3), [_rq(), _rq(), _rq("NonEvent"), _rq()]),
    ("event accepted after token refill", dict(server=3), [_rq(), _rq(), _rq(), _rq(ok=False), _rq(delay=1)]),
    ("event blocked by namespace limits", dict(server=100, ns=(3, 10)), [_rq(ns="A")] * 3 + [_rq(ns="A", ok=False)]),
    ("event from other namespace not blocked", dict(server=100, ns=(3, 10)), [_rq(ns="A")] * 3 + [_rq(ns="B")]),
    ("events from other namespaces should not count against limit", dict(server=100, ns=(3, 10)),
     [_rq(ns="A"), _rq(ns="A"), _rq(ns="B"), _rq(ns="A")]),
    ("event accepted after namespace token refill", dict(server=100, ns=(3, 10)),
     [_rq(ns="A")] * 3 + [_rq(ns="A", ok=False), _rq(ns="A", delay=1)]),
    ("event from other namespaces should not clear namespace limits", dict(server=100, ns=(3, 10)),
     [_rq(ns="A")] * 3 + [_rq(ns="B"), _rq(ns="A", ok=False)]),
    ("namespace limits from lru namespace should clear when cache size exceeded", dict(server=100, ns=(3, 2)),
     [_rq(ns="A"), _rq(ns="A"), _rq(ns="B"), _rq(ns="B"), _rq(ns="B"), _rq(ns="A"), _rq(ns="B", ok=False),
      _rq(ns="A", ok=False), _rq(ns="C"), _rq(ns="A", ok=False), _rq(ns="B")]),
    ("event blocked by source+object limits", dict(server=100, so=(3, 10)),
     [_rq(event=_comp("A"))] * 3 + [_rq(event=_comp("A"), ok=False)]),
    ("event from other source+object not blocked", dict(server=100, so=(3, 10)),
     [_rq(event=_comp("A"))] * 3 + [_rq(event=_comp("B"))]),
    ("events from other source+object should not count against limit", dict(server=100, so=(3, 10)),
     [_rq(event=_comp("A")), _rq(event=_comp("A")), _rq(event=_comp("B")), _rq(event=_comp("A"))]),
    ("event accepted after source+object token refill", dict(server=100, so=(3, 10)),
     [_rq(event=_comp("A"))] * 3 + [_rq(event=_comp("A"), ok=False), _rq(event=_comp("A"), delay=1)]),
    ("event from other source+object should not clear source+object limits", dict(server=100, so=(3, 10)),
     [_rq(event=_comp("A"))] * 3 + [_rq(event=_comp("B")), _rq(event=_comp("A"), ok=False)]),
    ("source+object limits from lru source+object should clear when cache size exceeded", dict(server=100, so=(3, 2)),
     [_rq(event=_comp(c), ok=ok) for c, ok in (("A", True), ("A", True), ("B", True), ("B", True), ("B", True), ("A", True),
                                              ("B", False), ("A", False), ("C", True), ("A", False), ("B", True))]),
    ("source host should be included in source+object key", dict(server=100, so=(1, 10)),
     _soi(lambda lbl: {"source": {"host": lbl}})),
    ("involved object kind should be included in source+object key", dict(server=100, so=(1, 10)),
     _soi(lambda lbl: {"involvedObject": {"kind": lbl}})),
    ("involved object namespace should be included in source+object key", dict(server=100, so=(1, 10)),
     _soi(lambda lbl: {"involvedObject": {"namespace": lbl}})),
    ("involved object name should be included in source+object key", dict(server=100, so=(1, 10)),
     _soi(lambda lbl: {"involvedObject": {"name": lbl}})),
    ("involved object UID should be included in source+object key", dict(server=100, so=(1, 10)),
     _soi(lambda lbl: {"involvedObject": {"uid": lbl}})),
    ("involved object APIVersion should be included in source+object key", dict(server=100, so=(1, 10)),
     _soi(lambda lbl: {"involvedObject": {"apiVersion": lbl}})),
    ("event blocked by user limits", dict(user=(3, 10)), [_rq(user="A")] * 3 + [_rq(user="A", ok=False)]),
    ("event from other user not blocked", dict(), [_rq(user="A")] * 3 + [_rq(user="B")]),
    ("events from other user should not count against limit", dict(), [_rq(user="A"), _rq(user="A"), _rq(user="B"), _rq(user="A")]),
]


@pytest.mark.parametrize("name,cfg,requests", ERL_CASES, ids=[c[0] for c in ERL_CASES])
def test_event_rate_limiting(name, cfg, requests):
    now = [1000.0]
    limits = []
    if cfg.get("server"):
        limits.append({"type": "Server", "qps": 1, "burst": cfg["server"]})
    if cfg.get("ns"):
        limits.append({"type": "Namespace", "qps": 1, "burst": cfg["ns"][0], "cacheSize": cfg["ns"][1]})
    if cfg.get("user"):
        limits.append({"type": "User", "qps": 1, "burst": cfg["user"][0], "cacheSize": cfg["user"][1]})
    if cfg.get("so"):
        limits.append({"type": "SourceAndObject", "qps": 1, "burst": cfg["so"][0], "cacheSize": cfg["so"][1]})
    plug = X.EventRateLimit(limits or [{"type": "Server", "qps": 1, "burst": 10 ** 9}], clock=lambda: now[0])
    for i, (kind, ns, user, event, delay, ok) in enumerate(requests):
        now[0] += delay
        a = Attributes(CREATE, "resource", "", ns, "name", copy.deepcopy(event) or {}, None, {"name": user}, kind)
        if ok:
            plug.validate(a, Ctx())
        else:
            with pytest.raises(m.StatusError) as e:
                plug.validate(a, Ctx())
            assert e.value.code == 429 and e.value.message.startswith("limit reached on type"), (name, i)


def test_event_rate_limit_every_limit_takes_a_token():
    """Validate consults every enforcer even after one rejected (the reference keeps the last
    error): a Server rejection still spends the Namespace token."""
    now = [0.0]
    plug = X.EventRateLimit([{"type": "Server", "qps": 1, "burst": 1}, {"type": "Namespace", "qps": 1, "burst": 2}],
                            clock=lambda: now[0])
    a = Attributes(CREATE, "events", "", "ns", "e", {}, None, {}, "Event")
    plug.validate(a, Ctx())
    with pytest.raises(m.StatusError) as e:
        plug.validate(a, Ctx())
    assert e.value.message == "limit reached on type Server for key "
    with pytest.raises(m.StatusError) as e:
        plug.validate(a, Ctx())                       # both exhausted now; the last limit's error wins
    assert e.value.message == "limit reached on type Namespace for key ns"


# ------------------------------------------------- OwnerReferencesPermissionEnforcement
def _gc_allow(user, verb, group, resource, sub="", ns="", name=""):
    """gc_admission_test.go fakeAuthorizer."""
    u = (user or {}).get("name")
    if u == "non-deleter":
        return not (verb == "delete" or (verb == "update" and sub == "finalizers"))
    if u == "non-pod-deleter":
        return not ((verb == "delete" and resource == "pods") or (verb == "update" and resource == "pods" and sub == "finalizers"))
    if u == "non-rc-deleter":
        return not ((verb == "delete" and resource == "replicationcontrollers")
                    or (verb == "update" and resource == "replicationcontrollers" and sub == "finalizers"))
    return True


class GCCtx(Ctx):
    def authorize(self, user, verb, group, resource, sub="", ns="", name=""):
        return _gc_allow(user, verb, group, resource, sub, ns, name)

    def plural_for_kind(self, av, kind):
        return {"ReplicationController": "replicationcontrollers", "DaemonSet": "daemonsets", "Pod": "pods"}.get(kind)


def _ref(kind, name, uid, block):
    r = {"apiVersion": "v1" if kind != "DaemonSet" else "extensions/v1beta1", "kind": kind, "name": name, "uid": uid}
    if block is not None:
        r["blockOwnerDeletion"] = block
    return r


BLOCK_RC1, BLOCK_RC2 = _ref("ReplicationController", "rc1", "rc1", True), _ref("ReplicationController", "rc2", "rc2", True)
NOTBLOCK_RC1, NOTBLOCK_RC2 = _ref("ReplicationController", "rc1", "rc1", False), _ref("ReplicationController", "rc2", "rc2", False)
NILBLOCK_RC1, NILBLOCK_RC2 = _ref("ReplicationController", "rc1", "rc1", None), _ref("ReplicationController", "rc2", "rc2", None)
BLOCK_DS1 = _ref("DaemonSet", "ds1", "ds1", True)


def _owned(*refs):
    return {"metadata": {"name": "p", "namespace": "ns", "ownerReferences": [dict(r) for r in refs]}}


CANT_DELETE, CANT_BLOCK = "cannot set an ownerRef on a resource you can't delete", "cannot set blockOwnerDeletion"


@pytest.mark.parametrize("name,user,resource,sub,old,new,err", [
    ("super-user, create, no objectref change", "super", "pods", "", None, _owned(), None),
    ("super-user, create, objectref change", "super", "pods", "", None, _owned(NILBLOCK_RC1), None),
    ("non-deleter, create, no objectref change", "non-deleter", "pods", "", None, _owned(), None),
    ("non-deleter, create, objectref change", "non-deleter", "pods", "", None, _owned(NILBLOCK_RC1), CANT_DELETE),
    ("non-pod-deleter, create, objectref change", "non-pod-deleter", "pods", "", None, _owned(NILBLOCK_RC1), CANT_DELETE),
    ("non-pod-deleter, create, objectref change, but not a pod", "non-pod-deleter", "not-pods", "", None, _owned(NILBLOCK_RC1), None),
    ("non-deleter, update, no objectref change", "non-deleter", "pods", "", _owned(NILBLOCK_RC1), _owned(NILBLOCK_RC1), None),
    ("non-deleter, update, objectref change", "non-deleter", "pods", "", _owned(), _owned(NILBLOCK_RC1), CANT_DELETE),
    ("non-deleter, update, objectref change two", "non-deleter", "pods", "", _owned(NILBLOCK_RC1),
     _owned(NILBLOCK_RC1, NILBLOCK_RC2), CANT_DELETE),
    ("non-pod-deleter, update status, objectref change", "non-pod-deleter", "pods", "status", _owned(), _owned(NILBLOCK_RC1), None),
    ("non-pod-deleter, update, objectref change", "non-pod-deleter", "pods", "", _owned(), _owned(NILBLOCK_RC1), CANT_DELETE),
    ("super-user, create, some ownerReferences have blockOwnerDeletion=true", "super", "pods", "", None,
     _owned(BLOCK_RC1, BLOCK_RC2), None),
    ("non-rc-deleter, create, all ownerReferences have blockOwnerDeletion=false or nil", "non-rc-deleter", "pods", "", None,
     _owned(NOTBLOCK_RC1, NILBLOCK_RC2), None),
    ("non-rc-deleter, create, some ownerReferences have blockOwnerDeletion=true", "non-rc-deleter", "pods", "", None,
     _owned(BLOCK_RC1, NOTBLOCK_RC2), CANT_BLOCK),
    ("non-rc-deleter, create, blockOwnerDeletion=true pointing to a daemonset", "non-rc-deleter", "pods", "", None,
     _owned(BLOCK_DS1), None),
    ("non-rc-deleter, update, no ownerReferences change blockOwnerDeletion", "non-rc-deleter", "pods", "", _owned(NILBLOCK_RC1),
     _owned(NOTBLOCK_RC1), None),
    ("non-rc-deleter, update, blockOwnerDeletion false to true", "non-rc-deleter", "pods", "", _owned(NOTBLOCK_RC1),
     _owned(BLOCK_RC1), CANT_BLOCK),
    ("non-rc-deleter, update, blockOwnerDeletion nil to true", "non-rc-deleter", "pods", "", _owned(NILBLOCK_RC1),
     _owned(BLOCK_RC1), CANT_BLOCK),
    ("non-rc-deleter, update, already blocking", "non-rc-deleter", "pods", "", _owned(BLOCK_RC1),
     _owned(BLOCK_RC1, NOTBLOCK_RC2), None),
    ("non-rc-deleter, update, add a new blocking reference", "non-rc-deleter", "pods", "", _owned(BLOCK_RC1),
     _owned(BLOCK_RC1, BLOCK_RC2), CANT_BLOCK),
])
def test_gc_admission(name, user, resource, sub, old, new, err):
    a = Attributes(CREATE if old is None else UPDATE, resource, sub, "ns", "p", copy.deepcopy(new), copy.deepcopy(old),
                   {"name": user})
    if err is None:
        X.OwnerReferencesPermissionEnforcement().validate(a, GCCtx())
    else:
        with pytest.raises(m.StatusError) as e:
            X.OwnerReferencesPermissionEnforcement().validate(a, GCCtx())
        assert e.value.code == 403 and err in e.value.message, name


# ------------------------------------------------- PersistentVolumeClaimResize / scdeny
def _claim(storage, phase, volume="", cls=None):
    spec = {"resources": {"requests": {"storage": storage}}}
    if volume:
        spec["volumeName"] = volume
    if cls is not None:
        spec["storageClassName"] = cls
    return {"metadata": {"name": "claim1", "namespace": "ns"}, "spec": spec, "status": {"phase": phase}}


RESIZE_CTX = dict(storageclasses=[{"metadata": {"name": "gold"}, "allowVolumeExpansion": True}, {"metadata": {"name": "silver"}}],
                  persistentvolumes=[{"metadata": {"name": "volume1"}, "spec": {"glusterfs": {"endpoints": "http://localhost:8080/"},
                                                                               "storageClassName": "gold"}},
                                     {"metadata": {"name": "volume2"}, "spec": {"hostPath": {}, "storageClassName": "gold"}}])


@pytest.mark.parametrize("name,new,old,err", [
    ("pvc-resize, update, no error", _claim("2Gi", "Bound", "volume1", "gold"), _claim("1Gi", "Bound", "volume1", "gold"), None),
    ("pvc-resize, update, volume plugin error", _claim("2Gi", "Bound", "volume2", "gold"), _claim("1Gi", "Bound", "volume2", "gold"),
     "volume plugin does not support resize"),
    ("pvc-resize, update, dynamically provisioned error (no class)", _claim("2Gi", "Bound", "volume3"),
     _claim("1Gi", "Bound", "volume3"),
     "only dynamically provisioned pvc can be resized and the storageclass that provisions the pvc must support resize"),
    ("pvc-resize, update, dynamically provisioned error (class without expansion)", _claim("2Gi", "Bound", "volume4", "silver"),
     _claim("1Gi", "Bound", "volume4", "silver"),
     "only dynamically provisioned pvc can be resized and the storageclass that provisions the pvc must support resize"),
    ("PVC update with no change in size", _claim("1Gi", "Pending", "", "silver"), _claim("1Gi", "Bound", "volume4", "silver"), None),
    ("expand pvc in pending state", _claim("2Gi", "Pending", "", "silver"), _claim("1Gi", "Pending", "", "silver"),
     "Only bound persistent volume claims can be expanded"),
    ("bound claim whose volume is missing", _claim("2Gi", "Bound", "gone", "gold"), _claim("1Gi", "Bound", "gone", "gold"),
     "Error updating persistent volume claim because fetching associated persistent volume failed"),
])
def test_pvc_resize_admission(name, new, old, err):
    a = Attributes(UPDATE, "persistentvolumeclaims", "", "ns", "claim1", copy.deepcopy(new), copy.deepcopy(old), {})
    if err is None:
        X.PersistentVolumeClaimResize().validate(a, Ctx(**RESIZE_CTX))
    else:
        with pytest.raises(m.StatusError) as e:
            X.PersistentVolumeClaimResize().validate(a, Ctx(**RESIZE_CTX))
        assert e.value.message == f'persistentvolumeclaims "claim1" is forbidden: {err}', name


@pytest.mark.parametrize("psc,csc,err", [
    ({"supplementalGroups": [1234]}, None, "SecurityContext.SupplementalGroups is forbidden"),
    ({"seLinuxOptions": {"level": "s0"}}, None, "pod.Spec.SecurityContext.SELinuxOptions is forbidden"),
    ({"runAsUser": 1}, None, "pod.Spec.SecurityContext.RunAsUser is forbidden"),
    ({"fsGroup": 1234}, None, "SecurityContext.FSGroup is forbidden"),
    (None, {"seLinuxOptions": {"level": "s0"}}, "SecurityContext.SELinuxOptions is forbidden"),
    (None, {"runAsUser": 1}, "SecurityContext.RunAsUser is forbidden"),
    ({}, {}, None),
    (None, None, None),
])
def test_security_context_deny(psc, csc, err):
    for kind in ("containers", "initContainers"):
        spec = {kind: [{"name": "c", **({"securityContext": csc} if csc is not None else {})}]}
        if psc is not None:
            spec["securityContext"] = psc
        a = _attrs({"metadata": {"name": "pod"}, "spec": spec})
        if err is None:
            X.SecurityContextDeny().validate(a, Ctx())
        else:
            with pytest.raises(m.StatusError) as e:
                X.SecurityContextDeny().validate(a, Ctx())
            assert e.value.message == f'pods "pod" is forbidden: {err}'
