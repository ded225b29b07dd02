"""Endpoints controller and RepackSubsets held to the reference's tests.

* pkg/api/v1/endpoints/util_test.go TestPackSubsets :33 — the table, extracted by
  hack/extract_endpoints_cases.py into fixtures/endpoints_cases.json and replayed against
  controllers.networking.repack_subsets. The reference orders subsets and ports by an md5 of Go's
  struct dump; amdkube orders them canonically, so both sides are compared after the same sort.
* pkg/controller/endpoint/endpoints_controller_test.go — every test, transcribed:
  syncService scenarios :156-869 (request counts and the written Endpoints),
  TestCheckLeftoverEndpoints :244, TestShouldPodBeInEndpoints :873, TestPodToEndpointAddress
  :962, TestPodChanged :996, TestDetermineNeededServiceUpdates :1051.
  TestWaitsForAllInformersToBeSynced2 :668 has no counterpart: amdkube controllers start after
  the manager's informers have synced. The reference's tests that give a Service an empty, non-nil
  selector (`map[string]string{}`, "selects all") run here with the pods' own `foo: bar` selector:
  an empty selector does not survive the API (omitempty and protobuf storage make it nil), and
  amdkube treats it as no selector (docs/PARITY.md). The reference PUTs the whole object on
  update; amdkube writes it with update too, and the tests compare the written object.
"""
from __future__ import annotations

import json
import os

import pytest

from amdkube.api import meta as m
from amdkube.controllers import networking as N
from tests.conftest import run
from tests.test_replicaset_parity import FakeFactory, FakeInformer

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "endpoints_cases.json")))


# ------------------------------------------------------------------ RepackSubsets
@pytest.mark.parametrize("case", FIX["PackSubsets"]["cases"], ids=[c["name"] for c in FIX["PackSubsets"]["cases"]])
def test_pack_subsets(case):
    got = N.repack_subsets(json.loads(json.dumps(case["given"])))
    assert got == N.sort_subsets(json.loads(json.dumps(case["expect"])))


# ------------------------------------------------------------------ harness
def add_pods(store: FakeInformer, ns: str, n_pods: int, n_ports: int, n_not_ready: int):
    """addPods: pods pod0.. labelled foo=bar at 1.2.3.(4+i), the last n_not_ready not ready."""
    for i in range(n_pods + n_not_ready):
        store.add({"metadata": {"namespace": ns, "name": f"pod{i}", "labels": {"foo": "bar"}},
                   "spec": {"containers": [{"ports": [{"name": f"port{i}", "containerPort": 8080 + j} for j in range(n_ports)]}]},
                   "status": {"podIP": f"1.2.3.{4 + i}",
                              "conditions": [{"type": "Ready", "status": "True" if i < n_pods else "False"}]}})


def add_not_ready_pods(store, ns, n_pods, n_ports, restart_policy, phase):
    for i in range(n_pods):
        store.add({"metadata": {"namespace": ns, "name": f"pod{i}", "labels": {"foo": "bar"}},
                   "spec": {"restartPolicy": restart_policy,
                            "containers": [{"ports": [{"name": f"port{i}", "containerPort": 8080 + j} for j in range(n_ports)]}]},
                   "status": {"podIP": f"1.2.3.{4 + i}", "phase": phase, "conditions": [{"type": "Ready", "status": "False"}]}})


class Client:
    """The fake endpoints handler: counts requests, keeps what was written."""

    def __init__(self):
        self.requests: list[tuple[str, dict | str]] = []

    async def create(self, obj, ns=None):
        self.requests.append(("POST", obj))
        return obj

    async def update(self, obj, sub=""):
        self.requests.append(("PUT", obj))
        return obj

    async def delete(self, resource, name, ns=""):
        self.requests.append(("DELETE", f"{resource}/{ns}/{name}"))

    async def get(self, resource, name, ns=""):
        raise AssertionError("unexpected GET")


class Mgr:
    def __init__(self):
        self.client = Client()
        self.factory = FakeFactory()
        self.pods = FakeInformer()


def controller():
    mgr = Mgr()
    c = N.EndpointsController(mgr)
    c.setup()
    return c


def ep(ns, subsets, labels=None, rv="1"):
    md = {"name": "foo", "namespace": ns, "resourceVersion": rv}
    if labels:
        md["labels"] = labels
    return {"metadata": md, "subsets": subsets}


def svc(ns, ports, selector=None, labels=None, **spec):
    md = {"name": "foo", "namespace": ns}
    if labels:
        md["labels"] = labels
    return {"metadata": md, "spec": {"selector": selector if selector is not None else {"foo": "bar"}, "ports": ports, **spec}}


def addr(ip, name, ns):
    return {"ip": ip, "nodeName": "", "targetRef": {"kind": "Pod", "name": name, "namespace": ns}}


def sync(c, key):
    run(c.sync(key))
    return c.mgr.client.requests


def written(req):
    verb, obj = req
    return verb, N.sort_subsets(json.loads(json.dumps(obj.get("subsets") or []))), m.labels_of(obj)


OLD_SUBSETS = [{"addresses": [{"ip": "6.7.8.9", "nodeName": ""}], "ports": [{"port": 1000}]}]


# ------------------------------------------------------------------ syncService
def test_sync_endpoints_items_preserve_no_selector():
    c = controller()
    c.ep_inf.add(ep("default", OLD_SUBSETS))
    c.svc_inf.add({"metadata": {"name": "foo", "namespace": "default"}, "spec": {"ports": [{"port": 80}]}})
    assert sync(c, "default/foo") == []


@pytest.mark.parametrize("subsets", [None, []], ids=["nil subsets", "empty subsets"])
def test_sync_endpoints_existing_nil_or_empty_subsets(subsets):
    c = controller()
    c.ep_inf.add(ep("default", subsets))
    c.svc_inf.add(svc("default", [{"port": 80}]))
    assert sync(c, "default/foo") == []


def test_sync_endpoints_new_no_subsets():
    c = controller()
    c.svc_inf.add(svc("default", [{"port": 80}]))
    reqs = sync(c, "default/foo")
    assert len(reqs) == 1 and written(reqs[0]) == ("POST", [], {})


def test_check_leftover_endpoints():
    c = controller()
    c.ep_inf.add(ep("default", OLD_SUBSETS))
    leader = ep("kube-system", [])
    leader["metadata"]["name"] = "kube-scheduler"
    leader["metadata"]["annotations"] = {N.LEADER_ANNOTATION: "{}"}
    c.ep_inf.add(leader)
    c.check_leftover_endpoints()
    assert len(c.queue) == 1 and run(c.queue.get()) == "default/foo"


@pytest.mark.parametrize("proto", ["TCP", "UDP"])
def test_sync_endpoints_protocol(proto):
    c = controller()
    c.ep_inf.add(ep("other", [{"addresses": [{"ip": "6.7.8.9", "nodeName": ""}], "ports": [{"port": 1000, "protocol": proto}]}]))
    add_pods(c.pod_inf, "other", 1, 1, 0)
    c.svc_inf.add(svc("other", [{"port": 80, "targetPort": 8080, "protocol": proto}]))
    reqs = sync(c, "other/foo")
    assert len(reqs) == 1
    assert written(reqs[0]) == ("PUT", [{"addresses": [addr("1.2.3.4", "pod0", "other")],
                                         "ports": [{"port": 8080, "protocol": proto}]}], {})
    assert reqs[0][1]["metadata"]["resourceVersion"] == "1"        # an update of the existing object


@pytest.mark.parametrize("ready,not_ready,expect", [
    (1, 0, [{"addresses": [addr("1.2.3.4", "pod0", "other")], "ports": [{"port": 8080, "protocol": "TCP"}]}]),
    (0, 1, [{"notReadyAddresses": [addr("1.2.3.4", "pod0", "other")], "ports": [{"port": 8080, "protocol": "TCP"}]}]),
    (1, 1, [{"addresses": [addr("1.2.3.4", "pod0", "other")], "notReadyAddresses": [addr("1.2.3.5", "pod1", "other")],
             "ports": [{"port": 8080, "protocol": "TCP"}]}]),
], ids=["selects all", "selects all not ready", "selects all mixed"])
def test_sync_endpoints_items_selects_all(ready, not_ready, expect):
    c = controller()
    c.ep_inf.add(ep("other", []))
    add_pods(c.pod_inf, "other", ready, 1, not_ready)
    c.svc_inf.add(svc("other", [{"port": 80, "protocol": "TCP", "targetPort": 8080}]))
    reqs = sync(c, "other/foo")
    assert len(reqs) == 1 and written(reqs[0]) == ("PUT", expect, {})


def test_sync_endpoints_items_preexisting():
    c = controller()
    c.ep_inf.add(ep("bar", OLD_SUBSETS))
    add_pods(c.pod_inf, "bar", 1, 1, 0)
    c.svc_inf.add(svc("bar", [{"port": 80, "protocol": "TCP", "targetPort": 8080}]))
    reqs = sync(c, "bar/foo")
    assert written(reqs[0]) == ("PUT", [{"addresses": [addr("1.2.3.4", "pod0", "bar")],
                                         "ports": [{"port": 8080, "protocol": "TCP"}]}], {})


def test_sync_endpoints_items_preexisting_identical():
    c = controller()
    c.ep_inf.add(ep("default", [{"addresses": [addr("1.2.3.4", "pod0", "default")], "ports": [{"port": 8080, "protocol": "TCP"}]}]))
    add_pods(c.pod_inf, "default", 1, 1, 0)
    c.svc_inf.add(svc("default", [{"port": 80, "protocol": "TCP", "targetPort": 8080}]))
    assert sync(c, "default/foo") == []


@pytest.mark.parametrize("labels", [None, {"foo": "bar"}], ids=["items", "items with labels"])
def test_sync_endpoints_items(labels):
    c = controller()
    add_pods(c.pod_inf, "other", 3, 2, 0)
    add_pods(c.pod_inf, "blah", 5, 2, 0)                     # make sure these aren't found!
    c.svc_inf.add(svc("other", [{"name": "port0", "port": 80, "protocol": "TCP", "targetPort": 8080},
                                {"name": "port1", "port": 88, "protocol": "TCP", "targetPort": 8088}], labels=labels))
    reqs = sync(c, "other/foo")
    assert len(reqs) == 1
    assert written(reqs[0]) == ("POST", N.sort_subsets([{
        "addresses": [addr("1.2.3.4", "pod0", "other"), addr("1.2.3.5", "pod1", "other"), addr("1.2.3.6", "pod2", "other")],
        "ports": [{"name": "port0", "port": 8080, "protocol": "TCP"}, {"name": "port1", "port": 8088, "protocol": "TCP"}]}]),
        labels or {})


def test_sync_endpoints_items_preexisting_labels_change():
    c = controller()
    c.ep_inf.add(ep("bar", OLD_SUBSETS, labels={"foo": "bar"}))
    add_pods(c.pod_inf, "bar", 1, 1, 0)
    c.svc_inf.add(svc("bar", [{"port": 80, "protocol": "TCP", "targetPort": 8080}], labels={"baz": "blah"}))
    reqs = sync(c, "bar/foo")
    assert written(reqs[0]) == ("PUT", [{"addresses": [addr("1.2.3.4", "pod0", "bar")],
                                         "ports": [{"port": 8080, "protocol": "TCP"}]}], {"baz": "blah"})


def test_sync_endpoints_headless_service():
    c = controller()
    c.ep_inf.add(ep("headless", [{"addresses": [{"ip": "6.7.8.9", "nodeName": ""}], "ports": [{"port": 1000, "protocol": "TCP"}]}]))
    add_pods(c.pod_inf, "headless", 1, 1, 0)
    c.svc_inf.add(svc("headless", [], clusterIP="None"))
    reqs = sync(c, "headless/foo")
    assert len(reqs) == 1
    assert written(reqs[0]) == ("PUT", [{"addresses": [addr("1.2.3.4", "pod0", "headless")],
                                         "ports": [{"port": 0, "protocol": "TCP"}]}], {})


@pytest.mark.parametrize("policy,phase", [("Never", "Failed"), ("Never", "Succeeded"), ("OnFailure", "Succeeded")])
def test_sync_endpoints_items_exclude_not_ready_pods(policy, phase):
    c = controller()
    c.ep_inf.add(ep("other", [], labels={"foo": "bar"}))
    add_not_ready_pods(c.pod_inf, "other", 1, 1, policy, phase)
    c.svc_inf.add(svc("other", [{"port": 80, "protocol": "TCP", "targetPort": 8080}]))
    reqs = sync(c, "other/foo")
    assert written(reqs[0]) == ("PUT", [], {})           # only the service's (no) labels change


def test_deleted_service_deletes_its_endpoints_and_deleting_pods_leave():
    c = controller()
    c.ep_inf.add(ep("ns", OLD_SUBSETS))
    assert sync(c, "ns/foo") == [("DELETE", "endpoints/ns/foo")]
    c = controller()
    add_pods(c.pod_inf, "ns", 2, 1, 0)
    c.pod_inf.items["ns/pod1"]["metadata"]["deletionTimestamp"] = "2026-10-17T00:00:00Z"
    c.svc_inf.add(svc("ns", [{"port": 80, "targetPort": 8080}]))
    assert [a["ip"] for a in written(sync(c, "ns/foo")[0])[1][0]["addresses"]] == ["1.2.3.4"]
    c = controller()                                       # tolerating unready endpoints keeps it
    add_pods(c.pod_inf, "ns", 2, 1, 0)
    c.pod_inf.items["ns/pod1"]["metadata"]["deletionTimestamp"] = "2026-10-17T00:00:00Z"
    s = svc("ns", [{"port": 80, "targetPort": 8080}])
    s["metadata"]["annotations"] = {N.TOLERATE_UNREADY: "True"}
    c.svc_inf.add(s)
    assert [a["ip"] for a in written(sync(c, "ns/foo")[0])[1][0]["addresses"]] == ["1.2.3.4", "1.2.3.5"]


# ------------------------------------------------------------------ helpers
@pytest.mark.parametrize("policy,phase,expected", [
    ("Never", "Failed", False), ("Never", "Succeeded", False), ("OnFailure", "Succeeded", False),
    ("Always", "Failed", True), ("Never", "Pending", True), ("OnFailure", "Unknown", True),
])
def test_should_pod_be_in_endpoints(policy, phase, expected):
    assert N.should_pod_be_in_endpoints({"spec": {"restartPolicy": policy}, "status": {"phase": phase}}) is expected


def test_pod_to_endpoint_address():
    store = FakeInformer()
    add_pods(store, "test", 1, 1, 0)
    [pod] = store.list()
    pod["metadata"].update(uid="u-1", resourceVersion="7")
    pod["spec"]["nodeName"] = "n1"
    epa = N.pod_to_endpoint_address(pod)
    assert epa == {"ip": "1.2.3.4", "nodeName": "n1",
                   "targetRef": {"kind": "Pod", "namespace": "test", "name": "pod0", "uid": "u-1", "resourceVersion": "7"}}


def test_pod_changed():
    store = FakeInformer()
    add_pods(store, "test", 1, 1, 0)
    [old] = store.list()
    new = json.loads(json.dumps(old))
    assert not N.pod_changed(old, new)
    new["spec"]["nodeName"] = "changed"
    assert N.pod_changed(old, new)
    new["spec"].pop("nodeName")
    new["metadata"]["resourceVersion"] = "changed"
    assert not N.pod_changed(old, new)
    new["metadata"].pop("resourceVersion")
    new["status"]["podIP"] = "1.2.3.1"
    assert N.pod_changed(old, new)
    new["status"]["podIP"] = old["status"]["podIP"]
    new["metadata"]["name"] = "wrong-name"
    assert N.pod_changed(old, new)
    new["metadata"]["name"] = old["metadata"]["name"]
    saved = old["status"]["conditions"]
    old["status"]["conditions"] = None
    assert N.pod_changed(old, new)
    old["status"]["conditions"] = saved
    new["metadata"]["deletionTimestamp"] = "2026-10-17T00:00:00Z"
    assert N.pod_changed(old, new)


@pytest.mark.parametrize("a,b,xor,union", [
    ("abc", "abc", "", "abc"), ("abc", "def", "abcdef", "abcdef"), ("abc", "", "abc", "abc"), ("", "abc", "abc", "abc"),
    ("abc", "bcd", "ad", "abcd"), ("", "", "", ""),
], ids=["no services changed", "all old services removed, new services added", "all old services removed, no new services added",
        "no old services, but new services added", "one service removed, one service added, two unchanged", "no services"])
def test_determine_needed_service_updates(a, b, xor, union):
    assert N.determine_needed_service_updates(set(a), set(b), False) == set(xor)
    assert N.determine_needed_service_updates(set(a), set(b), True) == set(union)


def test_update_pod_enqueues_by_membership_and_change():
    c = controller()
    for name, sel in (("s1", {"app": "a"}), ("s2", {"app": "b"})):
        c.svc_inf.add({"metadata": {"name": name, "namespace": "ns"}, "spec": {"selector": sel}})
    old = {"metadata": {"name": "p", "namespace": "ns", "labels": {"app": "a"}, "resourceVersion": "1"},
           "status": {"podIP": "1.1.1.1"}}
    new = json.loads(json.dumps(old))
    c._pod_update(old, new)                                   # a resync: same resourceVersion
    assert len(c.queue) == 0
    new["metadata"]["resourceVersion"] = "2"
    c._pod_update(old, new)                                   # nothing the endpoints show changed
    assert len(c.queue) == 0
    new["metadata"]["labels"] = {"app": "b"}
    c._pod_update(old, new)                                   # moved from s1 to s2: both
    assert {run(c.queue.get()) for _ in range(2)} == {"ns/s1", "ns/s2"}


def test_pack_subsets_not_ready_trumps_ready_in_either_order():
    """mapAddressByPort keeps not-ready once seen, whichever subset came first."""
    nr_first = [{"notReadyAddresses": [{"ip": "1.2.3.4"}], "ports": [{"port": 111}]},
                {"addresses": [{"ip": "1.2.3.4"}], "ports": [{"port": 111}]}]
    assert N.repack_subsets(nr_first) == [{"notReadyAddresses": [{"ip": "1.2.3.4"}], "ports": [{"port": 111}]}]
