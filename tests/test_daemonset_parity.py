"""DaemonSet controller held to the reference's tests.

Transcribed, cited by line (pkg/controller/daemon/):
* daemon_controller_test.go — every sync scenario from TestSimpleDaemonSetLaunchesPods :414 to
  TestPortConflictNodeDaemonDoesNotLaunchCriticalPod :1501 (each under both update strategies
  where the reference loops over them), with the same create / delete / event counts;
  TestNodeShouldRunDaemonPod :1539, TestUpdateNode :1664, TestDeleteNoDaemonPod :1735,
  TestGetNodesToDaemonPods :1910, TestAddNode :1973, the pod-event tests :1999-2283.
  TestDeleteFinalStateUnknown :382 has no counterpart: amdkube informers deliver the last known
  object on delete, never a tombstone.
* update_test.go — TestDaemonSetUpdatesPods :28, ...WhenNewPosIsNotReady :70, ...AllOldPodsNotReady
  :100, ...NoTemplateChanged :129, TestGetUnavailableNumbers :151.
* util/daemonset_util_test.go — TestIsPodUpdated :49, TestCreatePodTemplate :140.
The fakes (FakePodControl + the daemon test's store-backed wrapper, the fake clientset, the
FakeRecorder's buffered event count) are re-expressed; controller refs name apps/v1 (the
reference's extensions/v1beta1 — both groups serve the same DaemonSets here).
"""
from __future__ import annotations

import json
import uuid

import pytest

from amdkube.api import meta as m
from amdkube.controllers import daemonset as D
from amdkube.controllers.daemonset import DaemonSetController
from amdkube.controllers.deployment import compute_hash
from tests.conftest import run
from tests.test_replicaset_parity import FakeFactory, FakeInformer

SIMPLE_DS_LABEL = {"name": "simple-daemon", "type": "production"}
SIMPLE_DS_LABEL2 = {"name": "simple-daemon", "type": "test"}
SIMPLE_NODE_LABEL = {"color": "blue", "speed": "fast"}
SIMPLE_NODE_LABEL2 = {"color": "red", "speed": "fast"}
NO_SCHEDULE_TOLERATIONS = [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}]
NO_SCHEDULE_TAINTS = [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}]
NO_EXECUTE_TAINTS = [{"key": "dedicated", "value": "user1", "effect": "NoExecute"}]
NODE_NOT_READY = [{"key": "node.kubernetes.io/not-ready", "effect": "NoExecute", "timeAdded": "2017-01-01T00:00:00Z"}]
NODE_UNREACHABLE = [{"key": "node.kubernetes.io/unreachable", "effect": "NoExecute", "timeAdded": "2017-01-01T00:00:00Z"}]


def _clone(o):
    return json.loads(json.dumps(o))


# ------------------------------------------------------------------ fixtures (daemon_controller_test.go:95-235)
def new_daemon_set(name):
    return {"apiVersion": "extensions/v1beta1", "kind": "DaemonSet",
            "metadata": {"uid": str(uuid.uuid4()), "name": name, "namespace": "default"},
            "spec": {"revisionHistoryLimit": 2, "updateStrategy": {"type": "OnDelete"}, "templateGeneration": 0,
                     "selector": {"matchLabels": dict(SIMPLE_DS_LABEL)},
                     "template": {"metadata": {"labels": dict(SIMPLE_DS_LABEL)},
                                  "spec": {"containers": [{"image": "foo/bar",
                                                           "terminationMessagePath": "/dev/termination-log",
                                                           "imagePullPolicy": "IfNotPresent"}],
                                           "dnsPolicy": "Default"}}},
            "status": {}}


def rolling_strategy():
    return {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 1}}


def on_delete_strategy():
    return {"type": "OnDelete"}


STRATEGIES = [on_delete_strategy(), rolling_strategy()]
STRATEGY_IDS = ["OnDelete", "RollingUpdate"]


def new_node(name, labels=None):
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": labels or {}},
            "status": {"conditions": [{"type": "Ready", "status": "True"}], "allocatable": {"pods": "100"}}}


def new_pod(prefix, node_name, labels, ds=None):
    labels = dict(labels or {})
    if ds is not None:
        labels[D.HASH_LABEL] = compute_hash(ds["spec"]["template"], ds["status"].get("collisionCount"))
        spec = _clone(ds["spec"]["template"]["spec"])
    else:
        spec = {"containers": [{"image": "foo/bar", "terminationMessagePath": "/dev/termination-log",
                                "imagePullPolicy": "IfNotPresent"}]}
    if node_name:
        spec["nodeName"] = node_name
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": prefix + uuid.uuid4().hex[:5], "generateName": prefix, "labels": labels,
                        "namespace": "default", "uid": str(uuid.uuid4())},
           "spec": spec, "status": {}}
    if ds is not None:
        pod["metadata"]["ownerReferences"] = [m.new_controller_ref(ds, "apps/v1", "DaemonSet")]
    return pod


def add_nodes(store, start, n, labels=None):
    for i in range(start, start + n):
        store.add(new_node(f"node-{i}", labels))


def add_pods(store, node_name, labels, ds, n):
    for _ in range(n):
        store.add(new_pod(f"{node_name}-", node_name, labels, ds))


def add_failed_pods(store, node_name, labels, ds, n):
    for _ in range(n):
        p = new_pod(f"{node_name}-", node_name, labels, ds)
        p["status"] = {"phase": "Failed"}
        store.add(p)


def bare_pod(spec, name=None, phase=None, labels=None, ns=""):
    """`&v1.Pod{Spec: ...}`: no name, no namespace unless given."""
    p = {"metadata": {"name": name or "", "namespace": ns}, "spec": _clone(spec), "status": {}}
    if labels is not None:
        p["metadata"]["labels"] = labels
    if phase:
        p["status"]["phase"] = phase
    return p


def resource_pod_spec(node_name, memory, cpu):
    spec = {"containers": [{"resources": {"requests": {"memory": memory, "cpu": cpu, "pods": "100"}}}]}
    if node_name:
        spec["nodeName"] = node_name
    return spec


def allocatable(memory, cpu):
    return {"memory": memory, "cpu": cpu, "pods": "100"}


def mark_ready(p):
    conds = [c for c in p.setdefault("status", {}).get("conditions") or [] if c.get("type") != "Ready"]
    p["status"]["conditions"] = conds + [{"type": "Ready", "status": "True"}]


def set_critical(ds):
    ds["metadata"]["namespace"] = "kube-system"
    ds["spec"]["template"]["metadata"].setdefault("annotations", {})[D.CRITICAL_ANNOTATION] = ""


# ------------------------------------------------------------------ fakes
class Recorder:
    def __init__(self):
        self.events = []

    def event(self, obj, etype, reason, msg):
        self.events.append((etype, reason, msg))


class PodControl:
    """controller.FakePodControl wrapped by the daemon test's store-backed fakePodControl."""

    def __init__(self, store):
        self.store = store
        self.pod_ids: dict[str, dict] = {}
        self.create_limit = 0
        self.clear()

    def clear(self):
        self.templates, self.controller_refs, self.delete_names, self.patches = [], [], [], []
        self.create_call_count = 0

    async def create_pods_on_node(self, node_name, ns, template, owner, ref):
        self.create_call_count += 1
        if self.create_limit and self.create_call_count > self.create_limit:
            raise RuntimeError(f'failed to create pod on node "{node_name}"')
        self.templates.append(_clone(template))
        self.controller_refs.append(dict(ref))
        spec = _clone(template.get("spec") or {})
        if node_name:
            spec["nodeName"] = node_name
        pod = {"metadata": {"labels": dict((template.get("metadata") or {}).get("labels") or {}), "namespace": ns,
                            "generateName": f"{node_name}-", "name": f"{node_name}-{uuid.uuid4().hex[:5]}",
                            "uid": str(uuid.uuid4())},
               "spec": spec, "status": {}}
        self.store.add(pod)
        self.pod_ids[m.name_of(pod)] = pod

    async def delete_pod(self, ns, name, owner):
        self.delete_names.append(name)
        pod = self.pod_ids.pop(name, None)
        if pod is None:
            raise RuntimeError(f'pod "{name}" does not exist')
        self.store.delete(pod)

    async def patch_pod(self, ns, name, patch):
        self.patches.append(patch)


class Client:
    """fake.NewSimpleClientset: tracked objects; status updates recorded."""

    def __init__(self, *objs):
        self.objs = {}
        for o in objs:
            self._put(o)
        self.status_updates = []

    @staticmethod
    def _res(o):
        return {"DaemonSet": "daemonsets", "ControllerRevision": "controllerrevisions.apps", "Pod": "pods"}[o["kind"]]

    def _put(self, o):
        self.objs[(self._res(o), m.key_of(o))] = _clone(o)

    async def get(self, resource, name, ns=""):
        o = self.objs.get((resource, f"{ns}/{name}" if ns else name))
        if o is None:
            raise m.StatusError(404, "NotFound", f"{resource} {name} not found")
        return _clone(o)

    async def create(self, obj, ns=""):
        key = (self._res(obj), m.key_of(obj))
        if key in self.objs:
            raise m.StatusError(409, "AlreadyExists", "exists")
        self._put(obj)
        return _clone(obj)

    async def update(self, obj, sub=""):
        if sub == "status":
            self.status_updates.append(_clone(obj))
        self._put(obj)
        return _clone(obj)

    async def delete(self, resource, name, ns=""):
        self.objs.pop((resource, f"{ns}/{name}"), None)

    async def patch(self, resource, name, patch, ns="", patch_type=None):
        return {}


class Mgr:
    def __init__(self, client):
        self.client = client
        self.factory = FakeFactory()
        self.pods = FakeInformer()
        self.nodes = FakeInformer()
        self.recorder = Recorder()


def new_test_controller(*objs, critical=False):
    client = Client(*objs)
    mgr = Mgr(client)
    pc = PodControl(mgr.pods)
    dsc = DaemonSetController(mgr, pod_control=pc, critical_pods=critical)
    dsc.setup()
    return dsc, pc, client


def sync_and_validate(dsc, ds, pc, creates, deletes, events):
    try:
        run(dsc.sync(m.key_of(ds)))
    except Exception:                        # the reference ignores syncHandler's error here
        pass
    assert len(pc.templates) == creates, f"creates: want {creates}, saw {len(pc.templates)}"
    assert len(pc.delete_names) == deletes, f"deletes: want {deletes}, saw {len(pc.delete_names)}"
    assert len(dsc.recorder.events) == events, f"events: want {events}, saw {dsc.recorder.events}"
    assert len(pc.controller_refs) == creates
    for ref in pc.controller_refs:
        assert (ref["apiVersion"], ref["kind"], ref["controller"]) == ("apps/v1", "DaemonSet", True)


def clear_expectations(dsc, ds, pc):
    pc.clear()
    dsc.expectations.delete_expectations(m.key_of(ds))


def _ds(strategy, name="foo"):
    ds = new_daemon_set(name)
    ds["spec"]["updateStrategy"] = _clone(strategy)
    return ds


# ------------------------------------------------------------------ sync scenarios
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_simple_daemonset_launches_pods(strategy):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 5)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 5, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_simple_daemonset_pod_create_errors(strategy):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    pc.create_limit = 10
    add_nodes(dsc.node_inf, 0, 100)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 10, 0, 0)
    expected, p = 0, 0
    while expected <= pc.create_limit:
        expected += 1 << p
        p += 1
    assert pc.create_call_count <= expected


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_simple_daemonset_updates_status_after_launching_pods(strategy):
    ds = _ds(strategy)
    dsc, pc, client = new_test_controller(ds)
    dsc.ds_inf.add(ds)
    add_nodes(dsc.node_inf, 0, 5)
    sync_and_validate(dsc, ds, pc, 5, 0, 0)
    assert client.status_updates[-1]["status"]["currentNumberScheduled"] == 5


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_no_nodes_does_nothing(strategy):
    dsc, pc, _ = new_test_controller()
    ds = _ds(strategy)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_one_node_daemon_launches_pod(strategy):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    dsc.node_inf.add(new_node("only-node"))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_not_ready_node_daemon_does_launch_pod(strategy):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("not-ready")
    node["status"]["conditions"] = [{"type": "Ready", "status": "False"}]
    dsc.node_inf.add(node)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


def _events_for(strategy, on_delete, rolling):
    return on_delete if strategy["type"] == "OnDelete" else rolling


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_insufficient_capacity_node_daemon_does_not_launch_pod(strategy):
    spec = resource_pod_spec("too-much-mem", "75M", "75m")
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("too-much-mem")
    node["status"]["allocatable"] = allocatable("100M", "200m")
    dsc.node_inf.add(node)
    dsc.pod_inf.add(bare_pod(spec))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, _events_for(strategy, 2, 3))


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_insufficient_capacity_node_daemon_does_not_unschedule_running_pod(strategy):
    spec = resource_pod_spec("too-much-mem", "75M", "75m")
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("too-much-mem")
    node["status"]["allocatable"] = allocatable("100M", "200m")
    dsc.node_inf.add(node)
    dsc.pod_inf.add(bare_pod(spec))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, _events_for(strategy, 2, 3))


def test_insufficient_capacity_node_sufficient_capacity_with_node_label_daemon_launch_pod():
    ds = new_daemon_set("foo")
    ds["spec"]["template"]["spec"] = resource_pod_spec("", "50M", "75m")
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL)
    dsc, pc, _ = new_test_controller(ds)
    n1 = new_node("not-enough-resource")
    n1["status"]["allocatable"] = allocatable("10M", "20m")
    n2 = new_node("enough-resource", SIMPLE_NODE_LABEL)
    n2["status"]["allocatable"] = allocatable("100M", "200m")
    dsc.node_inf.add(n1)
    dsc.node_inf.add(n2)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_sufficient_capacity_with_terminated_pods_daemon_launches_pod(strategy):
    spec = resource_pod_spec("too-much-mem", "75M", "75m")
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("too-much-mem")
    node["status"]["allocatable"] = allocatable("100M", "200m")
    dsc.node_inf.add(node)
    dsc.pod_inf.add(bare_pod(spec, phase="Succeeded"))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 1)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_sufficient_capacity_node_daemon_launches_pod(strategy):
    spec = resource_pod_spec("not-too-much-mem", "75M", "75m")
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("not-too-much-mem")
    node["status"]["allocatable"] = allocatable("200M", "200m")
    dsc.node_inf.add(node)
    dsc.pod_inf.add(bare_pod(spec))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 1)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_network_unavailable_node_daemon_launches_pod(strategy):
    ds = _ds(strategy, "simple")
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("network-unavailable")
    node["status"]["conditions"] = [{"type": "NetworkUnavailable", "status": "True"}]
    dsc.node_inf.add(node)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_dont_do_anything_if_being_deleted(strategy):
    spec = resource_pod_spec("not-too-much-mem", "75M", "75m")
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    ds["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("not-too-much-mem")
    node["status"]["allocatable"] = allocatable("200M", "200m")
    dsc.node_inf.add(node)
    dsc.pod_inf.add(bare_pod(spec))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_dont_do_anything_if_being_deleted_race(strategy):
    ds = _ds(strategy)
    ds["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"     # the bare client: deleted
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 5)
    ds2 = _clone(ds)
    del ds2["metadata"]["deletionTimestamp"]                         # the cache: not deleted
    dsc.ds_inf.add(ds2)
    dsc.pod_inf.add(new_pod("pod1-", "node-0", SIMPLE_DS_LABEL))     # a matching orphan triggers the recheck
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


def _port_spec(node, port):
    return {"nodeName": node, "containers": [{"ports": [{"hostPort": port}]}]}


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_port_conflict_node_daemon_does_not_launch_pod(strategy):
    spec = _port_spec("port-conflict", 666)
    dsc, pc, _ = new_test_controller()
    dsc.node_inf.add(new_node("port-conflict"))
    dsc.pod_inf.add(bare_pod(spec))
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_port_conflict_with_same_daemon_pod_does_not_delete_pod(strategy):
    spec = _port_spec("port-conflict", 666)
    dsc, pc, _ = new_test_controller()
    node = new_node("port-conflict")
    dsc.node_inf.add(node)
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = spec
    dsc.ds_inf.add(ds)
    dsc.pod_inf.add(new_pod("foo-", "port-conflict", SIMPLE_DS_LABEL, ds))
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_no_port_conflict_node_daemon_launches_pod(strategy):
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"] = _port_spec("no-port-conflict", 6662)
    dsc, pc, _ = new_test_controller(ds)
    dsc.node_inf.add(new_node("no-port-conflict"))
    dsc.pod_inf.add(bare_pod(_port_spec("no-port-conflict", 6661)))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_pod_is_not_deleted_by_daemonset_with_empty_label_selector(strategy):
    ds = _ds(strategy)
    ds["spec"]["selector"] = {}
    ds["spec"]["template"]["spec"]["nodeSelector"] = {"foo": "bar"}
    dsc, pc, _ = new_test_controller(ds)
    dsc.node_inf.add(new_node("node1"))
    dsc.pod_inf.add(bare_pod({"nodeName": "node1"}, labels={"bang": "boom"}, ns="default"))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 1)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_deals_with_existing_pods(strategy):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    dsc.ds_inf.add(ds)
    add_nodes(dsc.node_inf, 0, 5)
    add_pods(dsc.pod_inf, "node-1", SIMPLE_DS_LABEL, ds, 1)
    add_pods(dsc.pod_inf, "node-2", SIMPLE_DS_LABEL, ds, 2)
    add_pods(dsc.pod_inf, "node-3", SIMPLE_DS_LABEL, ds, 5)
    add_pods(dsc.pod_inf, "node-4", SIMPLE_DS_LABEL2, ds, 2)
    sync_and_validate(dsc, ds, pc, 2, 5, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_selector_daemon_launches_pods(strategy):
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL)
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 4)
    add_nodes(dsc.node_inf, 4, 3, SIMPLE_NODE_LABEL)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 3, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_selector_daemon_deletes_unselected_pods(strategy):
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL)
    dsc, pc, _ = new_test_controller(ds)
    dsc.ds_inf.add(ds)
    add_nodes(dsc.node_inf, 0, 5)
    add_nodes(dsc.node_inf, 5, 5, SIMPLE_NODE_LABEL)
    add_pods(dsc.pod_inf, "node-0", SIMPLE_DS_LABEL2, ds, 2)
    add_pods(dsc.pod_inf, "node-1", SIMPLE_DS_LABEL, ds, 3)
    add_pods(dsc.pod_inf, "node-1", SIMPLE_DS_LABEL2, ds, 1)
    add_pods(dsc.pod_inf, "node-4", SIMPLE_DS_LABEL, ds, 1)
    sync_and_validate(dsc, ds, pc, 5, 4, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_selector_daemon_deals_with_existing_pods(strategy):
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL)
    dsc, pc, _ = new_test_controller(ds)
    dsc.ds_inf.add(ds)
    add_nodes(dsc.node_inf, 0, 5)
    add_nodes(dsc.node_inf, 5, 5, SIMPLE_NODE_LABEL)
    add_pods(dsc.pod_inf, "node-0", SIMPLE_DS_LABEL, ds, 1)
    add_pods(dsc.pod_inf, "node-1", SIMPLE_DS_LABEL, ds, 3)
    add_pods(dsc.pod_inf, "node-1", SIMPLE_DS_LABEL2, ds, 2)
    add_pods(dsc.pod_inf, "node-2", SIMPLE_DS_LABEL, ds, 4)
    add_pods(dsc.pod_inf, "node-6", SIMPLE_DS_LABEL, ds, 13)
    add_pods(dsc.pod_inf, "node-7", SIMPLE_DS_LABEL2, ds, 4)
    add_pods(dsc.pod_inf, "node-9", SIMPLE_DS_LABEL, ds, 1)
    add_pods(dsc.pod_inf, "node-9", SIMPLE_DS_LABEL2, ds, 1)
    sync_and_validate(dsc, ds, pc, 3, 20, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_bad_selector_daemon_does_nothing(strategy):
    dsc, pc, _ = new_test_controller()
    add_nodes(dsc.node_inf, 0, 4)
    add_nodes(dsc.node_inf, 4, 3, SIMPLE_NODE_LABEL)
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL2)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("node_name,selector,creates", [
    ("node-0", None, 1), ("node-10", None, 0), ("node-6", SIMPLE_NODE_LABEL, 1), ("node-0", SIMPLE_NODE_LABEL, 0),
], ids=["NameDaemonSetLaunchesPods", "BadNameDaemonSetDoesNothing", "NameAndSelectorDaemonSetLaunchesPods",
        "InconsistentNameSelectorDaemonSetDoesNothing"])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_name_and_selector(strategy, node_name, selector, creates):
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"]["nodeName"] = node_name
    if selector:
        ds["spec"]["template"]["spec"]["nodeSelector"] = dict(selector)
    dsc, pc, _ = new_test_controller(ds)
    if selector:
        add_nodes(dsc.node_inf, 0, 4)
        add_nodes(dsc.node_inf, 4, 3, SIMPLE_NODE_LABEL)
    else:
        add_nodes(dsc.node_inf, 0, 5)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, creates, 0, 0)


def test_selector_daemonset_launches_pods():
    ds = new_daemon_set("foo")
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL)
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 4)
    add_nodes(dsc.node_inf, 4, 3, SIMPLE_NODE_LABEL)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 3, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_node_affinity_daemon_launches_pods(strategy):
    ds = _ds(strategy)
    ds["spec"]["template"]["spec"]["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [{"key": "color", "operator": "In",
                                                     "values": [SIMPLE_NODE_LABEL["color"]]}]}]}}}
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 4)
    add_nodes(dsc.node_inf, 4, 3, SIMPLE_NODE_LABEL)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 3, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_number_ready_status(strategy):
    ds = _ds(strategy)
    dsc, pc, client = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 2, SIMPLE_NODE_LABEL)
    add_pods(dsc.pod_inf, "node-0", SIMPLE_DS_LABEL, ds, 1)
    add_pods(dsc.pod_inf, "node-1", SIMPLE_DS_LABEL, ds, 1)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)
    assert client.status_updates[-1]["status"]["numberReady"] == 0
    for p in dsc.pod_inf.list():
        mark_ready(p)
    dsc.ds_inf.add(client.status_updates[-1])            # the informer sees the status it wrote
    sync_and_validate(dsc, ds, pc, 0, 0, 0)
    assert client.status_updates[-1]["status"]["numberReady"] == 2


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_observed_generation(strategy):
    ds = _ds(strategy)
    ds["metadata"]["generation"] = 1
    dsc, pc, client = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 1, SIMPLE_NODE_LABEL)
    add_pods(dsc.pod_inf, "node-0", SIMPLE_DS_LABEL, ds, 1)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)
    assert client.status_updates[-1]["status"]["observedGeneration"] == 1


@pytest.mark.parametrize("failed,normal,creates,deletes,events", [
    (0, 1, 0, 0, 0), (0, 0, 1, 0, 0), (1, 0, 0, 1, 1), (1, 3, 0, 3, 1), (2, 1, 0, 2, 2),
], ids=["normal (do nothing)", "no pods (create 1)", "1 failed pod (kill 1), 0 normal pod",
        "1 failed pod (kill 1), 3 normal pods (kill 2)", "2 failed pods (kill 2), 1 normal pod"])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_daemon_kill_failed_pods(strategy, failed, normal, creates, deletes, events):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    dsc.ds_inf.add(ds)
    add_nodes(dsc.node_inf, 0, 1)
    add_failed_pods(dsc.pod_inf, "node-0", SIMPLE_DS_LABEL, ds, failed)
    add_pods(dsc.pod_inf, "node-0", SIMPLE_DS_LABEL, ds, normal)
    sync_and_validate(dsc, ds, pc, creates, deletes, events)


@pytest.mark.parametrize("taints,pod_prefix,deletes", [
    (NO_SCHEDULE_TAINTS, "keep-running-me", 0), (NO_EXECUTE_TAINTS, "stop-running-me", 1),
], ids=["NoScheduleTaintedDoesntEvicitRunningIntolerantPod", "NoExecuteTaintedDoesEvicitRunningIntolerantPod"])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_tainted_node_running_intolerant_pod(strategy, taints, pod_prefix, deletes):
    ds = _ds(strategy, "intolerant")
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("tainted")
    node["spec"] = {"taints": _clone(taints)}
    dsc.node_inf.add(node)
    dsc.pod_inf.add(new_pod(pod_prefix, "tainted", SIMPLE_DS_LABEL, ds))
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, deletes, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_tainted_node_daemon_does_not_launch_intolerant_pod(strategy):
    ds = _ds(strategy, "intolerant")
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("tainted")
    node["spec"] = {"taints": _clone(NO_SCHEDULE_TAINTS)}
    dsc.node_inf.add(node)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_tainted_node_daemon_launches_tolerate_pod(strategy):
    ds = _ds(strategy, "tolerate")
    ds["spec"]["template"]["spec"]["tolerations"] = _clone(NO_SCHEDULE_TOLERATIONS)
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("tainted")
    node["spec"] = {"taints": _clone(NO_SCHEDULE_TAINTS)}
    dsc.node_inf.add(node)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("taints,ready", [(NODE_NOT_READY, "False"), (NODE_UNREACHABLE, "Unknown")],
                         ids=["NotReadyNodeDaemonLaunchesPod", "UnreachableNodeDaemonLaunchesPod"])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_not_ready_or_unreachable_node_daemon_launches_pod(strategy, taints, ready):
    ds = _ds(strategy, "simple")
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("tainted")
    node["spec"] = {"taints": _clone(taints)}
    node["status"]["conditions"] = [{"type": "Ready", "status": ready}]
    dsc.node_inf.add(node)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_node_daemon_launches_tolerate_pod(strategy):
    ds = _ds(strategy, "tolerate")
    ds["spec"]["template"]["spec"]["tolerations"] = _clone(NO_SCHEDULE_TOLERATIONS)
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 1)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_daemonset_respects_termination(strategy):
    ds = _ds(strategy)
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 1, SIMPLE_NODE_LABEL)
    pod = new_pod("node-0-", "node-0", SIMPLE_DS_LABEL, ds)
    pod["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    dsc.pod_inf.add(pod)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_taint_out_of_disk_node_daemon_launches_critical_pod(strategy):
    ds = _ds(strategy, "critical")
    set_critical(ds)
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("not-enough-disk")
    node["status"]["conditions"] = [{"type": "OutOfDisk", "status": "True"}]
    node["spec"] = {"taints": [{"key": D.TAINT_OUT_OF_DISK, "effect": "NoSchedule"}]}
    dsc.node_inf.add(node)
    dsc.critical_gate = False
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)
    dsc.critical_gate = True
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_taint_pressure_node_daemon_launches_pod(strategy):
    ds = _ds(strategy, "critical")
    set_critical(ds)
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("resources-pressure")
    node["status"]["conditions"] = [{"type": "DiskPressure", "status": "True"},
                                    {"type": "MemoryPressure", "status": "True"}]
    node["spec"] = {"taints": [{"key": D.TAINT_DISK_PRESSURE, "effect": "NoSchedule"},
                               {"key": D.TAINT_MEMORY_PRESSURE, "effect": "NoSchedule"}]}
    dsc.node_inf.add(node)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 1, 0, 0)


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_insufficient_capacity_node_daemon_launches_critical_pod(strategy):
    spec = resource_pod_spec("too-much-mem", "75M", "75m")
    ds = _ds(strategy, "critical")
    ds["spec"]["template"]["spec"] = spec
    set_critical(ds)
    dsc, pc, _ = new_test_controller(ds)
    node = new_node("too-much-mem")
    node["status"]["allocatable"] = allocatable("100M", "200m")
    dsc.node_inf.add(node)
    dsc.pod_inf.add(bare_pod(spec))
    dsc.critical_gate = False
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, _events_for(strategy, 2, 3))
    dsc.critical_gate = True
    sync_and_validate(dsc, ds, pc, 1, 0, _events_for(strategy, 2, 3))


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_port_conflict_node_daemon_does_not_launch_critical_pod(strategy):
    spec = _port_spec("port-conflict", 666)
    dsc, pc, _ = new_test_controller(critical=True)
    dsc.node_inf.add(new_node("port-conflict"))
    dsc.pod_inf.add(bare_pod(spec))
    ds = _ds(strategy, "critical")
    ds["spec"]["template"]["spec"] = spec
    set_critical(ds)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


# ------------------------------------------------------------------ nodeShouldRunDaemonPod and handlers
def _ds_with_spec(spec):
    return {"metadata": {"name": "", "namespace": ""},
            "spec": {"selector": {"matchLabels": dict(SIMPLE_DS_LABEL)},
                     "template": {"metadata": {"labels": dict(SIMPLE_DS_LABEL)}, "spec": spec}}}


@pytest.mark.parametrize("pods_on_node,ds,want", [
    ([], _ds_with_spec(resource_pod_spec("", "50M", "0.5")), (True, True, True)),
    ([], _ds_with_spec(resource_pod_spec("", "200M", "0.5")), (True, False, True)),
    ([], _ds_with_spec(resource_pod_spec("other-node", "50M", "0.5")), (False, False, False)),
    ([bare_pod({"containers": [{"ports": [{"hostPort": 666}]}]})],
     _ds_with_spec({"containers": [{"ports": [{"hostPort": 666}]}]}), (False, False, False)),
])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_node_should_run_daemon_pod(strategy, pods_on_node, ds, want):
    node = new_node("test-node")
    node["status"]["allocatable"] = allocatable("100M", "1")
    dsc, _, _ = new_test_controller()
    dsc.node_inf.add(node)
    for p in pods_on_node:
        p = _clone(p)
        p["spec"]["nodeName"] = "test-node"
        dsc.pod_inf.add(p)
    ds = _clone(ds)
    ds["spec"]["updateStrategy"] = _clone(strategy)
    assert dsc.node_should_run(node, ds) == want


@pytest.mark.parametrize("old,new,ds_selector,should", [
    (new_node("node1"), new_node("node1"), SIMPLE_NODE_LABEL, False),
    (new_node("node1"), new_node("node1", SIMPLE_NODE_LABEL), SIMPLE_NODE_LABEL, True),
    (dict(new_node("node1"), spec={"taints": NO_SCHEDULE_TAINTS}), new_node("node1"), None, True),
], ids=["Nothing changed, should not enqueue", "Node labels changed", "Node taints changed"])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_update_node(strategy, old, new, ds_selector, should):
    dsc, pc, _ = new_test_controller()
    dsc.node_inf.add(_clone(old))
    ds = _ds(strategy, "ds")
    if ds_selector:
        ds["spec"]["template"]["spec"]["nodeSelector"] = dict(ds_selector)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)
    enqueued = []
    dsc.enqueue = lambda d: enqueued.append(m.name_of(d))
    dsc.update_node(_clone(old), _clone(new))
    assert ("ds" in enqueued) == should


def _full_node():
    node = new_node("node1")
    node["status"]["allocatable"] = allocatable("200M", "200m")
    return node


def _exist_pods(with_controller):
    out = []
    for i in range(4):
        p = bare_pod(resource_pod_spec("node1", "50M", "50m"), name=f"pod_{i}")
        if with_controller:
            p["metadata"]["ownerReferences"] = [{"controller": True}]
        out.append(p)
    return out


@pytest.mark.parametrize("exist,deleted,should", [
    (_exist_pods(False), bare_pod(resource_pod_spec("node1", "50M", "50m"), name="pod_0"), True),
    (_exist_pods(True), dict(bare_pod(resource_pod_spec("node1", "50M", "50m"), name="pod_0"),
                             metadata={"name": "pod_0", "namespace": "", "ownerReferences": [{"controller": True}]}), True),
    (_exist_pods(True), bare_pod(resource_pod_spec("", "50M", "50m"), name="pod_5"), False),
], ids=["Deleted non-daemon pods to release resources", "Deleted non-daemon pods (with controller) to release resources",
        "Deleted no scheduled pods"])
@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_delete_no_daemon_pod(strategy, exist, deleted, should):
    dsc, pc, _ = new_test_controller()
    dsc.node_inf.add(_full_node())
    ds = _ds(strategy, "ds")
    ds["spec"]["template"]["spec"] = resource_pod_spec("", "50M", "50m")
    dsc.ds_inf.add(ds)
    for p in exist:
        dsc.pod_inf.add(_clone(p))
    sync_and_validate(dsc, ds, pc, 0, 0, _events_for(strategy, 2, 3))
    enqueued = []
    dsc.enqueue_rate_limited = lambda d: enqueued.append(m.name_of(d))
    dsc.delete_pod(_clone(deleted))
    assert ("ds" in enqueued) == should


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_get_nodes_to_daemon_pods(strategy):
    ds, ds2 = _ds(strategy), _ds(strategy, "foo2")
    dsc, _, _ = new_test_controller(ds, ds2)
    dsc.ds_inf.add(ds)
    dsc.ds_inf.add(ds2)
    add_nodes(dsc.node_inf, 0, 2)
    failed = new_pod("matching-owned-failed-pod-1-", "node-1", SIMPLE_DS_LABEL, ds)
    failed["status"] = {"phase": "Failed"}
    wanted = [new_pod("matching-owned-0-", "node-0", SIMPLE_DS_LABEL, ds),
              new_pod("matching-orphan-0-", "node-0", SIMPLE_DS_LABEL),
              new_pod("matching-owned-1-", "node-1", SIMPLE_DS_LABEL, ds),
              new_pod("matching-orphan-1-", "node-1", SIMPLE_DS_LABEL), failed]
    ignored = [new_pod("non-matching-owned-0-", "node-0", SIMPLE_DS_LABEL2, ds),
               new_pod("non-matching-orphan-1-", "node-1", SIMPLE_DS_LABEL2),
               new_pod("matching-owned-by-other-0-", "node-0", SIMPLE_DS_LABEL, ds2)]
    for p in wanted + ignored:
        dsc.pod_inf.add(p)
    got = run(dsc.nodes_to_daemon_pods(ds))
    names = set()
    for node, pods in got.items():
        for p in pods:
            assert p["spec"]["nodeName"] == node
            names.add(m.name_of(p))
    assert names == {m.name_of(p) for p in wanted}


def _queued(dsc):
    out = []
    while len(dsc.queue):
        k = dsc.queue.get_nowait()
        dsc.queue.done(k)
        out.append(k)
    return sorted(out)


def test_add_node():
    dsc, _, _ = new_test_controller()
    ds = new_daemon_set("ds")
    ds["spec"]["template"]["spec"]["nodeSelector"] = dict(SIMPLE_NODE_LABEL)
    dsc.ds_inf.add(ds)
    dsc.add_node(new_node("node1"))
    assert len(dsc.queue) == 0
    dsc.add_node(new_node("node2", SIMPLE_NODE_LABEL))
    assert _queued(dsc) == ["default/ds"]


def _two(strategy, third_selector=None):
    dsc, _, _ = new_test_controller()
    ds1, ds2 = _ds(strategy, "foo1"), _ds(strategy, "foo2")
    dsc.ds_inf.add(ds1)
    dsc.ds_inf.add(ds2)
    if third_selector is not None:
        ds3 = _ds(strategy, "foo3")
        ds3["spec"]["selector"]["matchLabels"] = dict(third_selector)
        dsc.ds_inf.add(ds3)
    return dsc, ds1, ds2


def _bumped(p):
    p = _clone(p)
    p["metadata"]["resourceVersion"] = str(int(p["metadata"].get("resourceVersion") or 0) + 1)
    return p


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_add_pod(strategy):
    dsc, ds1, ds2 = _two(strategy)
    dsc.add_pod(new_pod("pod1-", "node-0", SIMPLE_DS_LABEL, ds1))
    assert _queued(dsc) == ["default/foo1"]
    dsc.add_pod(new_pod("pod2-", "node-0", SIMPLE_DS_LABEL, ds2))
    assert _queued(dsc) == ["default/foo2"]


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_add_pod_orphan(strategy):
    dsc, _, _ = _two(strategy, SIMPLE_DS_LABEL2)
    dsc.add_pod(new_pod("pod1-", "node-0", SIMPLE_DS_LABEL))
    assert _queued(dsc) == ["default/foo1", "default/foo2"]


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_update_pod(strategy):
    dsc, ds1, ds2 = _two(strategy)
    for ds in (ds1, ds2):
        pod = new_pod("pod-", "node-0", SIMPLE_DS_LABEL, ds)
        dsc.update_pod(pod, _bumped(pod))
        assert _queued(dsc) == [m.key_of(ds)]


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_update_pod_orphan_same_labels(strategy):
    dsc, _, _ = _two(strategy)
    pod = new_pod("pod1-", "node-0", SIMPLE_DS_LABEL)
    dsc.update_pod(pod, _bumped(pod))
    assert len(dsc.queue) == 0


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_update_pod_orphan_with_new_labels(strategy):
    dsc, _, _ = _two(strategy)
    pod = new_pod("pod1-", "node-0", SIMPLE_DS_LABEL)
    prev = _clone(pod)
    prev["metadata"]["labels"] = {"foo2": "bar2"}
    dsc.update_pod(prev, _bumped(pod))
    assert _queued(dsc) == ["default/foo1", "default/foo2"]


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_update_pod_change_controller_ref(strategy):
    dsc, ds1, ds2 = _two(strategy)
    pod = new_pod("pod1-", "node-0", SIMPLE_DS_LABEL, ds1)
    prev = _clone(pod)
    prev["metadata"]["ownerReferences"] = [m.new_controller_ref(ds2, "apps/v1", "DaemonSet")]
    dsc.update_pod(prev, _bumped(pod))
    assert len(dsc.queue) == 2


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_update_pod_controller_ref_removed(strategy):
    dsc, ds1, _ = _two(strategy)
    pod = new_pod("pod1-", "node-0", SIMPLE_DS_LABEL, ds1)
    cur = _bumped(pod)
    cur["metadata"]["ownerReferences"] = []
    dsc.update_pod(pod, cur)
    assert len(dsc.queue) == 2


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_delete_pod(strategy):
    dsc, ds1, ds2 = _two(strategy)
    dsc.delete_pod(new_pod("pod1-", "node-0", SIMPLE_DS_LABEL, ds1))
    assert _queued(dsc) == ["default/foo1"]
    dsc.delete_pod(new_pod("pod2-", "node-0", SIMPLE_DS_LABEL, ds2))
    assert _queued(dsc) == ["default/foo2"]


@pytest.mark.parametrize("strategy", STRATEGIES, ids=STRATEGY_IDS)
def test_delete_pod_orphan(strategy):
    dsc, _, _ = _two(strategy, SIMPLE_DS_LABEL2)
    dsc.delete_pod(new_pod("pod1-", "node-0", SIMPLE_DS_LABEL))
    assert len(dsc.queue) == 0


# ------------------------------------------------------------------ update_test.go
def _start_rolling(dsc, pc, ds, max_unavailable, change_template=True):
    if change_template:
        ds["spec"]["template"]["spec"]["containers"][0]["image"] = "foo2/bar2"
        ds["spec"]["templateGeneration"] += 1
    ds["spec"]["updateStrategy"] = {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": max_unavailable}}
    dsc.ds_inf.add(ds)
    clear_expectations(dsc, ds, pc)


def _mark_all_ready(dsc):
    for p in dsc.pod_inf.list():
        mark_ready(p)


def test_daemonset_updates_pods():
    ds = new_daemon_set("foo")
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 5)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 5, 0, 0)
    _mark_all_ready(dsc)
    _start_rolling(dsc, pc, ds, 2)
    for creates, deletes, ready_after in [(0, 2, False), (2, 0, True), (0, 2, False), (2, 0, True),
                                          (0, 1, False), (1, 0, True), (0, 0, False)]:
        sync_and_validate(dsc, ds, pc, creates, deletes, 0)
        if ready_after:
            _mark_all_ready(dsc)
        clear_expectations(dsc, ds, pc)


def test_daemonset_updates_when_new_pod_is_not_ready():
    ds = new_daemon_set("foo")
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 5)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 5, 0, 0)
    _mark_all_ready(dsc)
    _start_rolling(dsc, pc, ds, 3)
    for creates, deletes in [(0, 3), (3, 0), (0, 0)]:     # the new pods never become ready
        sync_and_validate(dsc, ds, pc, creates, deletes, 0)
        clear_expectations(dsc, ds, pc)


def test_daemonset_updates_all_old_pods_not_ready():
    ds = new_daemon_set("foo")
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 5)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 5, 0, 0)
    _start_rolling(dsc, pc, ds, 3)
    for creates, deletes in [(0, 5), (5, 0), (0, 0)]:     # unavailable old pods all go at once
        sync_and_validate(dsc, ds, pc, creates, deletes, 0)
        clear_expectations(dsc, ds, pc)


def test_daemonset_updates_no_template_changed():
    ds = new_daemon_set("foo")
    dsc, pc, _ = new_test_controller(ds)
    add_nodes(dsc.node_inf, 0, 5)
    dsc.ds_inf.add(ds)
    sync_and_validate(dsc, ds, pc, 5, 0, 0)
    _start_rolling(dsc, pc, ds, 3, change_template=False)
    sync_and_validate(dsc, ds, pc, 0, 0, 0)


def _ready_pod(name, node, terminating=False):
    p = new_pod(name, node, SIMPLE_DS_LABEL)
    mark_ready(p)
    if terminating:
        p["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    return p


@pytest.mark.parametrize("nodes,max_unavailable,node_pods,want", [
    (0, 0, {}, (0, 0)),
    (2, 1, {"node-0": [_ready_pod("pod-0", "node-0")], "node-1": [_ready_pod("pod-1", "node-1")]}, (1, 0)),
    (2, 0, {"node-0": [_ready_pod("pod-0", "node-0")]}, (0, 1)),
    (2, "50%", {"node-0": [_ready_pod("pod-0", "node-0")], "node-1": [_ready_pod("pod-1", "node-1")]}, (1, 0)),
    (2, "50%", {"node-0": [_ready_pod("pod-0", "node-0")],
                "node-1": [_ready_pod("pod-1", "node-1", terminating=True)]}, (1, 1)),
], ids=["No nodes", "Two nodes with ready pods", "Two nodes, one node without pods",
        "Two nodes with pods, MaxUnavailable in percents",
        "Two nodes with pods, MaxUnavailable in percents, pod terminating"])
def test_get_unavailable_numbers(nodes, max_unavailable, node_pods, want):
    dsc, _, _ = new_test_controller()
    add_nodes(dsc.node_inf, 0, nodes)
    ds = new_daemon_set("x")
    ds["spec"]["updateStrategy"]["rollingUpdate"] = {"maxUnavailable": max_unavailable}
    dsc.ds_inf.add(ds)
    assert dsc.unavailable_numbers(ds, node_pods) == want


# ------------------------------------------------------------------ util/daemonset_util_test.go
def _util_pod(labels):
    return {"metadata": {"name": "pod1", "namespace": "default", "labels": labels},
            "spec": {"nodeName": "node1", "containers": [{"image": "foo/bar"}]}}


GEN, HASH = 12345, "55555"
LABELS = {D.TEMPLATE_GEN_LABEL: str(GEN), D.HASH_LABEL: HASH}
LABELS_NO_HASH = {D.TEMPLATE_GEN_LABEL: str(GEN)}


@pytest.mark.parametrize("gen,labels,hash_,updated", [
    (GEN, LABELS, HASH, True), (GEN, LABELS, HASH + "123", True), (GEN, LABELS_NO_HASH, HASH, True),
    (GEN, LABELS_NO_HASH, "", True), (GEN, LABELS, "", True), (GEN + 1, LABELS, HASH, True),
    (GEN + 1, LABELS, HASH + "123", False), (GEN, {}, "", False), (GEN, {}, HASH, False), (GEN, None, HASH, False),
])
def test_is_pod_updated(gen, labels, hash_, updated):
    assert D.is_pod_updated(gen, _util_pod(labels), hash_) == updated


@pytest.mark.parametrize("gen,hash_,expect_unique", [(1, "", False), (2, "3242341807", True)])
def test_create_pod_template(gen, hash_, expect_unique):
    tpl = D.create_pod_template({}, gen, hash_)
    assert tpl["metadata"]["labels"][D.TEMPLATE_GEN_LABEL] == str(gen)
    if expect_unique:
        assert tpl["metadata"]["labels"][D.HASH_LABEL] == hash_
    else:
        assert D.HASH_LABEL not in tpl["metadata"]["labels"]
    keys = {(t["key"], t["effect"]) for t in tpl["spec"]["tolerations"]}
    assert keys == {(D.TAINT_NOT_READY, "NoExecute"), (D.TAINT_UNREACHABLE, "NoExecute"),
                    (D.TAINT_DISK_PRESSURE, "NoSchedule"), (D.TAINT_MEMORY_PRESSURE, "NoSchedule")}


def test_apps_v1_daemonset_without_template_generation_counts_hash_only():
    """apps/v1 objects have no templateGeneration: only the hash decides (docs/PARITY.md)."""
    assert D.is_pod_updated(None, _util_pod({D.TEMPLATE_GEN_LABEL: "None", D.HASH_LABEL: "1"}), "2") is False
    assert D.TEMPLATE_GEN_LABEL not in D.create_pod_template({}, None, "7")["metadata"]["labels"]
