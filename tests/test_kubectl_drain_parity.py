"""kubectl cordon / uncordon / drain at reference parity.

pkg/kubectl/cmd/drain_test.go transcribed over an in-memory fake client (the reference drives a
fake REST client the same way): TestCordon (7 cases), TestDrain (12 cases, each run once with
the eviction subresource and once with plain DELETE), TestDeletePods (waitForDelete: done,
timeout, client error). Then a live cluster: a PodDisruptionBudget holds an eviction (429,
retried every 5 s in the reference, shortened here) until a second replica is ready, DaemonSet
and mirror pods stay, and the node ends cordoned.
"""
from __future__ import annotations

import asyncio
import io

import pytest

from amdkube.api import meta as m
from amdkube.kubectl import drain as D
from tests.conftest import run

NODE = {"metadata": {"name": "node"}, "spec": {"externalID": "node"}}
CORDONED = {"metadata": {"name": "node"}, "spec": {"externalID": "node", "unschedulable": True}}
LABELS = {"my_key": "my_value"}


def _ref(kind, name, api="v1"):
    return [{"apiVersion": api, "kind": kind, "name": name, "uid": "123", "blockOwnerDeletion": True, "controller": True}]


def _pod(owner=None, volumes=None, annotations=None, phase=None):
    md = {"name": "bar", "namespace": "default", "uid": "bar-uid", "labels": LABELS}
    if owner:
        md["ownerReferences"] = owner
    if annotations:
        md["annotations"] = annotations
    p = {"metadata": md, "spec": {"nodeName": "node", "volumes": volumes or []}}
    if phase:
        p["status"] = {"phase": phase}
    return p


RC_POD = _pod(_ref("ReplicationController", "rc"))
DS_POD = _pod(_ref("DaemonSet", "ds", "extensions/v1beta1"))
ORPHANED_DS_POD = _pod()
JOB_POD = _pod(_ref("Job", "job"))
RS_POD = _pod(_ref("ReplicaSet", "rs"))
NAKED_POD = _pod()
EMPTYDIR_POD = _pod(volumes=[{"name": "scratch", "emptyDir": {"medium": ""}}])


class FakeClient:
    """The requests drain makes, answered from fixed objects; pods vanish once evicted/deleted."""

    def __init__(self, node, pods, controllers, eviction=True):
        self.node, self.pods, self.controllers, self.eviction = m.deepcopy(node), [m.deepcopy(p) for p in pods], controllers, eviction
        self.patched, self.deleted, self.evicted = None, False, False

    async def get(self, res, name, ns=""):
        if res == "nodes":
            if name != "node":
                raise m.not_found("nodes", name)
            return m.deepcopy(self.node)
        if (res, name) in self.controllers:
            return {"metadata": {"name": name}}
        raise m.not_found(res, name)

    async def get_or_none(self, res, name, ns=""):
        return next((p for p in self.pods if m.name_of(p) == name), None)

    async def list(self, res, ns="", label_selector=None, field_selector=None):
        assert res == "pods" and field_selector == "spec.nodeName=node"
        return [m.deepcopy(p) for p in self.pods], "1"

    async def patch(self, res, name, body, ns="", patch_type=None, **kw):
        assert res == "nodes" and name == "node"
        spec = dict(self.node.get("spec") or {})
        for k, v in body["spec"].items():
            if v is None:
                spec.pop(k, None)
            else:
                spec[k] = v
        self.node["spec"] = spec
        self.patched = spec
        return m.deepcopy(self.node)

    async def delete(self, res, name, ns="", grace=None, **kw):
        self.deleted = True
        self.pods = [p for p in self.pods if m.name_of(p) != name]

    async def request(self, method, path, params=None, body=None, **kw):
        if path == "/apis":
            return {"groups": [{"name": "policy", "preferredVersion": {"groupVersion": "policy/v1beta1"}}]}
        if path == "/api/v1":
            return {"resources": [{"name": "pods/eviction", "kind": "Eviction"}] if self.eviction else []}
        if method == "POST" and path.endswith("/pods/bar/eviction"):
            self.evicted = True
            self.pods = [p for p in self.pods if m.name_of(p) != "bar"]
            return {}
        raise AssertionError(f"unexpected request {method} {path}")

    @staticmethod
    def resource_info(res):
        from amdkube.api.scheme import SCHEME
        return SCHEME.resolve(res)

    @staticmethod
    def path(ri, ns="", name=None, sub=""):
        return f"/api/v1/namespaces/{ns}/pods/{name}/{sub}"


def _args(*argv):
    from amdkube.kubectl import main as km
    a, extra = km.parser().parse_known_args(list(argv))
    a.args = list(a.args) + extra
    return a


async def _run(cmd, client, *argv):
    import contextlib
    out, err = io.StringIO(), io.StringIO()
    a = _args(cmd, *argv)
    with contextlib.redirect_stdout(out), contextlib.redirect_stderr(err):
        fn = {"drain": D.cmd_drain, "cordon": D.cmd_cordon, "uncordon": D.cmd_uncordon}[cmd]
        rc = await fn(client, a)
    return rc, out.getvalue(), err.getvalue()


@pytest.mark.parametrize("node,expected,cmd,arg,fatal", [
    (CORDONED, NODE, "uncordon", "node/node", False),
    (CORDONED, NODE, "uncordon", "node", False),
    (NODE, NODE, "uncordon", "node", False),
    (CORDONED, CORDONED, "cordon", "node", False),
    (NODE, CORDONED, "cordon", "node", False),
    (NODE, NODE, "cordon", "bar", True),
    (NODE, NODE, "uncordon", "bar", True),
], ids=["node/node syntax", "uncordon for real", "uncordon does nothing", "cordon does nothing", "cordon for real",
        "cordon missing node", "uncordon missing node"])
def test_cordon(node, expected, cmd, arg, fatal):
    async def go():
        c = FakeClient(node, [], set())
        if fatal:
            with pytest.raises(m.StatusError):
                await _run(cmd, c, arg)
            assert c.patched is None
            return
        rc, out, _ = await _run(cmd, c, arg)
        assert rc == 0
        if expected["spec"] != node["spec"]:
            assert c.patched == expected["spec"]
            assert out == f'node "node" {cmd}ed\n'
        else:
            assert c.patched is None and out == f'node "node" already {cmd}ed\n'
    run(go())


CTRL = {("replicationcontrollers", "rc"), ("daemonsets", "ds"), ("jobs", "job"), ("replicasets", "rs")}

DRAIN_CASES = [
    ("RC-managed pod", [RC_POD], CTRL, ["node"], False, True),
    ("DS-managed pod", [DS_POD], CTRL, ["node"], True, False),
    ("orphaned DS-managed pod", [ORPHANED_DS_POD], set(), ["node"], True, False),
    ("orphaned DS-managed pod with --force", [ORPHANED_DS_POD], set(), ["node", "--force"], False, True),
    ("DS-managed pod with --ignore-daemonsets", [DS_POD], CTRL, ["node", "--ignore-daemonsets"], False, False),
    ("Job-managed pod", [JOB_POD], CTRL, ["node"], False, True),
    ("RS-managed pod", [RS_POD], CTRL, ["node"], False, True),
    ("naked pod", [NAKED_POD], set(), ["node"], True, False),
    ("naked pod with --force", [NAKED_POD], set(), ["node", "--force"], False, True),
    ("pod with EmptyDir", [EMPTYDIR_POD], set(), ["node", "--force"], True, False),
    ("pod with EmptyDir and --delete-local-data", [EMPTYDIR_POD], set(), ["node", "--force", "--delete-local-data"], False, True),
    ("empty node", [], CTRL, ["node"], False, False),
]


@pytest.mark.parametrize("eviction", [True, False], ids=["eviction", "delete"])
@pytest.mark.parametrize("desc,pods,ctrls,args,fatal,expect_delete", DRAIN_CASES, ids=[c[0] for c in DRAIN_CASES])
def test_drain(desc, pods, ctrls, args, fatal, expect_delete, eviction):
    async def go():
        c = FakeClient(NODE, pods, ctrls, eviction=eviction)
        rc, out, err = await _run("drain", c, *args)
        assert c.patched == CORDONED["spec"], desc                      # always cordoned first
        assert (rc != 0) == fatal, (desc, out, err)
        removed = c.evicted if eviction else c.deleted
        assert removed == expect_delete, desc
        if expect_delete:
            assert (c.evicted, c.deleted) == ((True, False) if eviction else (False, True))
            assert f'pod "bar" {"evicted" if eviction else "deleted"}' in out and 'node "node" drained' in out
    run(go())


def test_drain_messages():
    async def go():
        rc, _, err = await _run("drain", FakeClient(NODE, [DS_POD], CTRL), "node")
        assert rc == 1 and f"error: {D.K_DAEMONSET_FATAL}: bar" in err
        assert 'error: unable to drain node "node", aborting command...' in err
        rc, out, err = await _run("drain", FakeClient(NODE, [DS_POD], CTRL), "node", "--ignore-daemonsets")
        assert rc == 0 and f"WARNING: {D.K_DAEMONSET_WARNING}: bar" in err and 'node "node" drained' in out
        rc, _, err = await _run("drain", FakeClient(NODE, [NAKED_POD], set()), "node", "--force")
        assert f"WARNING: {D.K_UNMANAGED_WARNING}: bar" in err
        # a controller that is gone: fatal, or a warning naming the error with --force
        rc, _, err = await _run("drain", FakeClient(NODE, [RC_POD], set()), "node")
        assert rc == 1 and 'replicationcontrollers "rc" not found: bar' in err
        rc, _, err = await _run("drain", FakeClient(NODE, [RC_POD], set()), "node", "--force")
        assert rc == 0 and 'WARNING: replicationcontrollers "rc" not found: bar' in err
        # mirror pods are never evicted; every filter still runs on them (no short circuit in
        # getPodsForDeletion), so a mirror pod without a controller needs --force in v1.9
        mirror = _pod(annotations={D.MIRROR_ANNOTATION: "x"})
        c = FakeClient(NODE, [mirror], set())
        assert (await _run("drain", c, "node"))[0] == 1 and not c.evicted
        rc, _, err = await _run("drain", c, "node", "--force")
        assert rc == 0 and not c.evicted and not c.deleted
        c = FakeClient(NODE, [_pod(phase="Succeeded")], set())
        assert (await _run("drain", c, "node"))[0] == 0 and c.evicted
        # --dry-run changes nothing
        c = FakeClient(NODE, [RC_POD], CTRL)
        rc, out, _ = await _run("drain", c, "node", "--dry-run")
        assert rc == 0 and c.patched is None and not c.evicted and out == 'node "node" cordoned (dry run)\nnode "node" drained (dry run)\n'
        # usage
        rc, _, err = await _run("drain", c, "node", "-l", "a=b")
        assert rc == 1 and "cannot specify both a node name and a --selector option" in err
    run(go())


def test_wait_for_delete():
    """TestDeletePods: waitForDelete over eight pods."""
    pods = [{"metadata": {"name": f"pod{i}", "namespace": "default", "uid": f"{i}{i}", "generation": i}} for i in range(8)]

    class Getter:
        def __init__(self, fn):
            self.fn = fn

        async def get_or_none(self, res, name, ns=""):
            return self.fn(name)

    called = {}

    def finishing(name):
        i = int(name[3:])
        if name not in called:
            called[name] = True
            return pods[i]
        if i < 4:
            return {"metadata": {"name": name, "uid": str(i)}}          # replaced by a new pod
        return None

    async def go():
        d = D.Drainer(Getter(finishing), out=io.StringIO(), interval=0.05)
        assert await d.wait_for_delete(pods, "deleted", 10) == []
        d = D.Drainer(Getter(lambda n: pods[int(n[3:])]), out=io.StringIO(), interval=0.05)
        with pytest.raises(TimeoutError):
            await d.wait_for_delete(pods, "deleted", 0.3)

        def broken(name):
            raise m.StatusError(500, "InternalError", "This is a random error for testing")
        d = D.Drainer(Getter(broken), out=io.StringIO(), interval=0.05)
        with pytest.raises(m.StatusError):
            await d.wait_for_delete(pods, "deleted", 5)
    run(go())


def test_drain_through_the_cluster_waits_for_the_disruption_budget():
    from amdkube.localcluster import LocalCluster, wait_pod

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "web"},
                            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "web"}},
                                     "template": {"metadata": {"labels": {"app": "web"}},
                                                  "spec": {"terminationGracePeriodSeconds": 1, "containers": [
                                                      {"name": "w", "image": "busybox", "command": ["sleep", "300"]}]}}}},
                           "default")
            await c.create({"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget", "metadata": {"name": "web"},
                            "spec": {"minAvailable": 1, "selector": {"matchLabels": {"app": "web"}}}}, "default")
            await c.create({"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "agent"},
                            "spec": {"selector": {"matchLabels": {"app": "agent"}},
                                     "template": {"metadata": {"labels": {"app": "agent"}},
                                                  "spec": {"containers": [{"name": "a", "image": "busybox", "command": ["sleep", "300"]}]}}}},
                           "default")
            for _ in range(200):
                pods, _ = await c.list("pods", "default")
                if len([p for p in pods if (p.get("status") or {}).get("phase") == "Running"]) >= 2:
                    break
                await asyncio.sleep(0.1)
            node = lc.node_name
            d = D.Drainer(c, ignore_daemonsets=True, out=io.StringIO(), err=io.StringIO(), interval=0.2, eviction_retry=0.3)
            task = asyncio.ensure_future(d.drain([await c.get("nodes", node)]))
            await asyncio.sleep(1.5)
            assert not task.done()                                  # the budget refuses the eviction (429)
            assert (await c.get("nodes", node))["spec"].get("unschedulable") is True
            web = [p for p in (await c.list("pods", "default", "app=web"))[0]]
            assert len(web) == 1 and not (web[0]["metadata"].get("deletionTimestamp"))
            # the budget goes away (its spec is immutable in v1.9): the retried eviction goes through
            await c.delete("poddisruptionbudgets", "web", "default")
            await asyncio.wait_for(task, 60)
            out = d.out.getvalue()
            assert f'pod "{m.name_of(web[0])}" evicted' in out and f'node "{node}" drained' in out
            assert "WARNING: Ignoring DaemonSet-managed pods" in d.err.getvalue()
            left = [m.name_of(p) for p in (await c.list("pods", "default"))[0] if not (p["metadata"].get("deletionTimestamp"))]
            assert any(n.startswith("agent") for n in left)         # DaemonSet pods stay
    run(go(), 120)
