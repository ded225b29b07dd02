"""kubectl taint against the reference's tables.

Transcribed from pkg/util/taints/taints_test.go (TestReorganizeTaints :446-585, TestParseTaints
:588-690, TestDeleteTaint :241-313, TestDeleteTaintByKey :316-373, TestCheckIfTaintsAlreadyExists
:376-446) and pkg/kubectl/cmd/taint_test.go (TestTaint :79-330, TestValidateFlags :336-380);
the command cases run against an in-memory node and once against a live apiserver.
"""
from __future__ import annotations

import copy

import pytest

from amdkube.kubectl import taint as T
from amdkube.kubectl.metacmds import UsageError
from tests.conftest import run
from tests.test_kubectl_commands_parity import _kubectl

NS, PNS, NE = "NoSchedule", "PreferNoSchedule", "NoExecute"
FOO = {"key": "foo", "value": "bar", "effect": NS}


@pytest.mark.parametrize("name,overwrite,add,remove,expected,op,err", [
    ("no changes with overwrite is true", True, [], [], [FOO], T.MODIFIED, False),
    ("no changes with overwrite is false", False, [], [], [FOO], T.UNTAINTED, False),
    ("add new taint", False, [{"key": "foo_1", "effect": NE}], [], [{"key": "foo_1", "effect": NE}, FOO], T.TAINTED, False),
    ("delete taint with effect", False, [], [{"key": "foo", "effect": NS}], [], T.UNTAINTED, False),
    ("delete taint with no effect", False, [], [{"key": "foo"}], [], T.UNTAINTED, False),
    ("delete non-exist taint", False, [], [{"key": "foo_1", "effect": NS}], [FOO], T.UNTAINTED, True),
    ("add new taint and delete old one", False, [{"key": "foo_1", "effect": NS}], [{"key": "foo", "effect": NS}],
     [{"key": "foo_1", "effect": NS}], T.MODIFIED, False),
])
def test_reorganize_taints(name, overwrite, add, remove, expected, op, err):
    got_op, new, errs = T.reorganize([dict(FOO)], overwrite, add, remove)
    assert (new, got_op, bool(errs)) == (expected, op, err), name


@pytest.mark.parametrize("name,spec,add,remove,err", [
    ("invalid spec format", ["foo=abc"], None, None, True),
    ("invalid spec effect for adding taint", ["foo=abc:invalid_effect"], None, None, True),
    ("invalid spec effect for deleting taint", ["foo:invalid_effect-"], None, None, True),
    ("add new taints", ["foo=abc:NoSchedule", "bar=abc:NoSchedule"],
     [{"key": "foo", "value": "abc", "effect": NS}, {"key": "bar", "value": "abc", "effect": NS}], [], False),
    ("delete taints", ["foo:NoSchedule-", "bar:NoSchedule-"], [], [{"key": "foo", "effect": NS}, {"key": "bar", "effect": NS}], False),
    ("add taints and delete taints", ["foo=abc:NoSchedule", "bar=abc:NoSchedule", "foo:NoSchedule-", "bar:NoSchedule-"],
     [{"key": "foo", "value": "abc", "effect": NS}, {"key": "bar", "value": "abc", "effect": NS}],
     [{"key": "foo", "effect": NS}, {"key": "bar", "effect": NS}], False),
])
def test_parse_taints(name, spec, add, remove, err):
    if err:
        with pytest.raises(UsageError):
            T.parse_taints(spec)
        return
    assert T.parse_taints(spec) == (add, remove), name


@pytest.mark.parametrize("spec,msg", [
    ("foo=abc", "unknown taint spec: foo=abc"),
    ("foo=abc:invalid_effect", "invalid taint effect: invalid_effect, unsupported taint effect"),
    ("foo:invalid_effect-", "invalid taint effect: invalid_effect, unsupported taint effect"),
    ("nospecialchars^@=banana:NoSchedule", "invalid taint spec: nospecialchars^@=banana:NoSchedule"),
    ("foo=b@r:NoSchedule", "invalid taint spec: foo=b@r:NoSchedule, a valid label must be"),
    ("a=b=c:NoSchedule", "invalid taint spec: a=b=c:NoSchedule"),
    ("foo=bar:NoSchedule:x", "invalid taint spec: foo=bar:NoSchedule:x, "),
    ("foo", "unknown taint spec: foo"),
])
def test_parse_taint_messages(spec, msg):
    with pytest.raises(UsageError) as e:
        T.parse_taints([spec])
    assert str(e.value).startswith(msg)


def test_empty_taint_value_is_a_label_value():
    assert T.parse_taints(["foo=:NoSchedule"]) == ([{"key": "foo", "value": "", "effect": NS}], [])


def test_duplicated_taint_message():
    with pytest.raises(UsageError) as e:
        T.parse_taints(["foo=bar:NoSchedule", "foo=barz:NoSchedule"])
    assert str(e.value) == "duplicated taints with the same key and effect: {foo barz NoSchedule <nil>}"
    # the same key with another effect is a different taint
    assert len(T.parse_taints(["foo=bar:NoSchedule", "foo=bar:NoExecute"])[0]) == 2


@pytest.mark.parametrize("old,add,expected", [
    ([], [{"key": "foo_1", "effect": NS}], ""),
    ([{"key": "foo_1", "effect": NS}, {"key": "foo_2", "effect": NS}], [{"key": "foo_1", "effect": NE}], ""),
    ([{"key": "foo_1", "effect": NS}, {"key": "foo_2", "effect": NS}], [{"key": "foo_2", "effect": NS}], "foo_2"),
    ([{"key": "foo_1", "effect": NS}, {"key": "foo_2", "effect": NS}, {"key": "foo_3", "effect": NS}],
     [{"key": "foo_2", "effect": NS}, {"key": "foo_3", "effect": NS}], "foo_2,foo_3"),
])
def test_check_if_taints_already_exist(old, add, expected):
    assert T.already_exists(old, add) == expected


@pytest.mark.parametrize("old,remove,expected,removed", [
    ([{"key": "foo", "effect": NS}], {"key": "foo_1", "effect": NS}, [{"key": "foo", "effect": NS}], False),
    ([{"key": "foo", "effect": NS}], {"key": "foo", "effect": NE}, [{"key": "foo", "effect": NS}], False),
    ([{"key": "foo", "effect": NS}], {"key": "foo", "effect": NS}, [], True),
    ([], {"key": "foo", "effect": NS}, [], False),
    ([{"key": "foo", "effect": NS}, {"key": "foo", "effect": NE}], {"key": "foo"}, [], True),     # by key
    ([{"key": "foo", "effect": NS}], {"key": "foo_1"}, [{"key": "foo", "effect": NS}], False),
])
def test_delete_taint(old, remove, expected, removed):
    _, new, errs = T.reorganize(old, False, [], [remove])
    assert new == expected and (not errs) == removed
    if errs:
        assert errs == [f'taint "{T.to_string(remove)}" not found']


class FakeNodes:
    """An apiserver holding named nodes: get, list (label selector) and patch of spec.taints."""

    def __init__(self, **nodes):
        self.nodes = {n: {"apiVersion": "v1", "kind": "Node", "metadata": {"name": n, "labels": lbl},
                          "spec": {"taints": copy.deepcopy(t)} if t else {}} for n, (lbl, t) in nodes.items()}
        self.patches = []

    async def get(self, res, name, ns=""):
        from amdkube.api import meta as m
        if name not in self.nodes:
            raise m.not_found("nodes", name)
        return copy.deepcopy(self.nodes[name])

    async def list(self, res, ns="", selector=None, *a):
        from amdkube.api.labels import parse_selector
        sel = parse_selector(selector or "")
        return [copy.deepcopy(n) for n in self.nodes.values() if sel.matches(n["metadata"]["labels"])], "1"

    async def patch(self, res, name, body, *a, **k):
        self.patches.append((name, body))
        self.nodes[name]["spec"]["taints"] = body["spec"]["taints"]
        return copy.deepcopy(self.nodes[name])


DED_NS = {"key": "dedicated", "value": "namespaceA", "effect": NS}
DED_PNS = {"key": "dedicated", "value": "namespaceA", "effect": PNS}


@pytest.mark.parametrize("desc,old,new,args,fatal,tainted", [
    ("taints a node with effect NoSchedule", [], [{"key": "foo", "value": "bar", "effect": NS}],
     ["node", "node-name", "foo=bar:NoSchedule"], False, True),
    ("taints a node with effect PreferNoSchedule", [], [{"key": "foo", "value": "bar", "effect": PNS}],
     ["node", "node-name", "foo=bar:PreferNoSchedule"], False, True),
    ("update an existing taint on the node, change the value from bar to barz", [FOO],
     [{"key": "foo", "value": "barz", "effect": NS}], ["node", "node-name", "foo=barz:NoSchedule", "--overwrite"], False, True),
    ("taints a node with two taints", [], [DED_NS, {"key": "foo", "value": "bar", "effect": PNS}],
     ["node", "node-name", "dedicated=namespaceA:NoSchedule", "foo=bar:PreferNoSchedule"], False, True),
    ("remove one of two taints with the same key by key and effect", [DED_NS, DED_PNS], [DED_PNS],
     ["node", "node-name", "dedicated:NoSchedule-"], False, True),
    ("remove all taints of a key with the wildcard", [DED_NS, DED_PNS], [], ["node", "node-name", "dedicated-"], False, True),
    ("update one taint and remove the other", [DED_NS, {"key": "foo", "value": "bar", "effect": PNS}],
     [{"key": "foo", "value": "barz", "effect": PNS}],
     ["node", "node-name", "dedicated:NoSchedule-", "foo=barz:PreferNoSchedule", "--overwrite"], False, True),
    ("invalid taint key", [], None, ["node", "node-name", "nospecialchars^@=banana:NoSchedule"], True, False),
    ("invalid taint effect", [], None, ["node", "node-name", "foo=bar:NoExcute"], True, False),
    ("duplicated taints with the same key and effect should be rejected", [], None,
     ["node", "node-name", "foo=bar:NoExcute", "foo=barz:NoExcute"], True, False),
    ("can't update existing taint on the node, since 'overwrite' flag is not set", [FOO], None,
     ["node", "node-name", "foo=bar:NoSchedule"], True, False),
])
def test_taint(desc, old, new, args, fatal, tainted):
    c = FakeNodes(**{"node-name": ({}, old)})
    rc, out, err = run(_kubectl(c, "taint", *args))
    assert (rc != 0) == fatal, (desc, err)
    assert bool(c.patches) == tainted, desc
    if tainted:
        assert (c.nodes["node-name"]["spec"]["taints"] or []) == new, desc


@pytest.mark.parametrize("args,expected", [
    (["nodes", "n1", "foo=bar:NoSchedule"], 'node "n1" tainted\n'),
    (["no", "n1", "foo=bar:NoSchedule", "--overwrite"], 'node "n1" modified\n'),
    (["node", "n2", "foo:NoSchedule-"], 'node "n2" untainted\n'),
    (["node", "n2", "x=y:NoExecute", "foo:NoSchedule-"], 'node "n2" modified\n'),
    (["node", "n1", "n2", "gpu=mi355x:NoExecute"], 'node "n1" tainted\nnode "n2" tainted\n'),
    (["node", "-l", "pool=gpu", "gpu=mi355x:NoExecute"], 'node "n2" tainted\n'),
    (["node", "--all", "gpu-"], ""),
])
def test_taint_output(args, expected):
    c = FakeNodes(n1=({}, []), n2=({"pool": "gpu"}, [FOO]))
    rc, out, err = run(_kubectl(c, "taint", *args))
    if expected:
        assert (rc, out, err) == (0, expected, "")
    else:      # removing a key no node has: both report it, neither is patched
        assert rc == 1 and err.count('taint "gpu" not found') == 2 and not c.patches


@pytest.mark.parametrize("args,msg", [
    ([], "one or more resources must be specified as <resource> <name>"),
    (["node", "n1"], "at least one taint update is required"),
    (["node", "foo=bar:NoSchedule", "n1"], "all resources must be specified before taint changes: n1"),
    (["pods", "p", "foo=bar:NoSchedule"], 'invalid resource type pods, only ["nodes" "no" "node"] are supported'),
    (["node/n1", "foo=bar:NoSchedule"], 'invalid resource type node/n1'),
    (["node", "n1", "foo=bar:NoSchedule", "foo-"],
     'can not both modify and remove the following taint(s) in the same command: {"foo":""}'),
    (["node", "n1", "foo=bar:NoSchedule", "foo:NoSchedule-"],
     'can not both modify and remove the following taint(s) in the same command: {"foo":"NoSchedule"}'),
    # TestValidateFlags
    (["node", "-l", "myLabel=X", "--all", "foo=bar:NoSchedule"], "setting 'all' parameter with a non empty selector is prohibited."),
    (["node", "foo=bar:NoSchedule"], "at least one resource name must be specified since 'all' parameter is not set"),
])
def test_taint_usage_errors(args, msg):
    c = FakeNodes(n1=({}, []))
    rc, out, err = run(_kubectl(c, "taint", *args))
    assert rc == 1 and msg in err and not c.patches, err


def test_taint_validate_flags_pass():
    for args in (["node", "-l", "myLabel=X", "foo=bar:NoSchedule"], ["node", "--all", "foo=bar:NoSchedule"],
                 ["node", "n1", "foo=bar:NoSchedule"]):
        c = FakeNodes(n1=({"myLabel": "X"}, []))
        assert run(_kubectl(c, "taint", *args))[0] == 0, args


def test_taint_missing_node_does_not_stop_the_others():
    c = FakeNodes(n1=({}, []))
    rc, out, err = run(_kubectl(c, "taint", "node", "ghost", "n1", "foo=bar:NoSchedule"))
    assert rc == 1 and out == 'node "n1" tainted\n' and 'nodes "ghost" not found' in err


def test_taint_live():
    from amdkube.localcluster import LocalCluster

    async def body():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "gpu-0", "labels": {"pool": "gpu"}}})
            assert (await _kubectl(c, "taint", "nodes", "gpu-0", "dedicated=ml:NoSchedule"))[1] == 'node "gpu-0" tainted\n'
            assert (await _kubectl(c, "taint", "nodes", "-l", "pool=gpu", "maint=yes:NoExecute"))[1] == 'node "gpu-0" tainted\n'
            taints = (await c.get("nodes", "gpu-0"))["spec"]["taints"]
            assert [(t["key"], t["effect"]) for t in taints] == [("maint", NE), ("dedicated", NS)]
            rc, out, err = await _kubectl(c, "taint", "nodes", "gpu-0", "dedicated=ml:NoSchedule")
            assert rc == 1 and "already has dedicated taint(s) with same effect(s) and --overwrite is false" in err
            assert (await _kubectl(c, "taint", "nodes", "gpu-0", "dedicated-", "maint:NoExecute-"))[1] == 'node "gpu-0" untainted\n'
            assert not (await c.get("nodes", "gpu-0"))["spec"].get("taints")
    run(body())
