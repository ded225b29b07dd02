"""Strategic merge patch: the reference's own table tests, then the API-typed cases the round-3
review reproduced (Service ports merge by `port`, Container ports by `containerPort`).

The table comes from staging/src/k8s.io/apimachinery/pkg/util/strategicpatch/patch_test.go
(TestCustomStrategicMergePatch, TestStrategicMergePatch), extracted into
tests/fixtures/strategicpatch_cases.json by hack/extract_smp_cases.py, and runs over the same
`mergeItem` struct schema the reference uses (patch_test.go:96-119), given as StructNodes.
"""
import copy
import json
import os

import pytest

from amdkube.api import strategicpatch as smp
from amdkube.api.strategicpatch import StructNode

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "strategicpatch_cases.json")))

MERGE_ITEM = StructNode("mergeItem")
RETAIN_ITEM = StructNode("retainKeysMergeItem")
MERGE_ITEM.fields = {
    "mergingList": (MERGE_ITEM, "merge", "name"),
    "nonMergingList": (MERGE_ITEM, "", ""),
    "mergingIntList": (None, "merge", ""),
    "nonMergingIntList": (None, "", ""),
    "mergeItemPtr": (MERGE_ITEM, "merge", "name"),
    "simpleMap": (("map", None), "", ""),
    "replacingItem": (None, "replace", ""),
    "retainKeysMap": (RETAIN_ITEM, "retainKeys", ""),
    "retainKeysMergingList": (MERGE_ITEM, "merge,retainKeys", "name"),
}
RETAIN_ITEM.fields = {
    "simpleMap": (("map", None), "", ""),
    "mergingIntList": (None, "merge", ""),
    "mergingList": (MERGE_ITEM, "merge", "name"),
    "nonMergingList": (MERGE_ITEM, "", ""),
}


def _sort(obj, node):
    """patch.go sortMergeListsByNameMap: merge lists in key order, scalar merge lists sorted."""
    if not isinstance(obj, dict):
        return obj
    out = {}
    for k, v in obj.items():
        if k == smp.RETAIN_KEYS or k.startswith(smp.DELETE_PRIMITIVE + "/"):
            v = sorted(v, key=smp._gostr)
        elif k.startswith(smp.SET_ORDER + "/") or k == smp.DIRECTIVE:
            pass
        elif isinstance(v, dict):
            v = _sort(v, smp._lookup(node, k)[0])
        elif isinstance(v, list):
            child, strat, mk, _ = smp._lookup(node, k)
            if strat == smp.MERGE and v:
                if isinstance(v[0], dict):
                    v = sorted((_sort(e, child) for e in v), key=lambda e: smp._gostr(e.get(mk)))
                else:
                    v = sorted(smp._dedup(v), key=smp._gostr)
        out[k] = v
    return out


def _prep(c, field, default=None):
    v = c.get(field, default)
    if v is None:
        return {} if default is None else default
    return _sort(v, MERGE_ITEM) if c.get("sorted") else v


@pytest.mark.parametrize("c", CASES["apply"], ids=lambda c: c["description"])
def test_reference_patch_application(c):
    original, patch = _prep(c, "original"), _prep(c, "twoWay")
    expected = _prep(c, "twoWayResult") if c.get("twoWayResult") is not None else _prep(c, "modified")
    if c.get("expectedError"):
        with pytest.raises(smp.PatchError) as ei:
            smp.apply(original, patch, MERGE_ITEM)
        assert c["expectedError"] in str(ei.value)
        return
    assert smp.apply(original, patch, MERGE_ITEM) == expected


@pytest.mark.parametrize("c", CASES["create"], ids=lambda c: c["description"])
def test_reference_two_way_patch(c):
    original, modified = _prep(c, "original"), _prep(c, "modified")
    expected_patch = _prep(c, "twoWay")
    expected = _prep(c, "twoWayResult") if c.get("twoWayResult") is not None else modified
    patch = smp.create_two_way(original, modified, MERGE_ITEM)
    assert patch == expected_patch
    assert smp.apply(original, patch, MERGE_ITEM) == expected


@pytest.mark.parametrize("c", CASES["create"], ids=lambda c: c["description"])
def test_reference_three_way_patch(c):
    original, modified, current = _prep(c, "original"), _prep(c, "modified"), _prep(c, "current")
    expected, result = _prep(c, "threeWay"), c.get("result")
    result = None if result is None else _prep(c, "result")
    try:
        patch = smp.create_three_way(original, modified, current, MERGE_ITEM, overwrite=False)
    except smp.ConflictError:
        assert "conflict" in c["description"], "unexpected conflict"
        if result is None:
            return
        patch = smp.create_three_way(original, modified, current, MERGE_ITEM, overwrite=True)
    else:
        assert "conflict" not in c["description"] and result is not None, "expected a conflict"
    assert patch == expected
    assert smp.apply(current, patch, MERGE_ITEM) == result


# ---------------------------------------------------------------------- API-typed cases
def _svc(ports, **extra):
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default", **extra},
            "spec": {"selector": {"app": "web"}, "ports": ports}}


def test_service_ports_merge_by_port_not_container_port():
    """round-3 review: a strategic PATCH of Service spec.ports raised KeyError: 'containerPort'."""
    node = smp.schema_for("v1", "Service")
    live = _svc([{"name": "http", "port": 80, "targetPort": 8080, "protocol": "TCP"},
                 {"name": "https", "port": 443, "targetPort": 8443, "protocol": "TCP"}])
    out = smp.apply(live, {"spec": {"ports": [{"port": 443, "targetPort": 9443}]}}, node)
    assert out["spec"]["ports"] == [{"name": "http", "port": 80, "targetPort": 8080, "protocol": "TCP"},
                                    {"name": "https", "port": 443, "targetPort": 9443, "protocol": "TCP"}]


def test_three_way_apply_of_a_two_port_service_keeps_both_ports():
    node = smp.schema_for("v1", "Service")
    original = _svc([{"name": "http", "port": 80, "targetPort": 8080}, {"name": "https", "port": 443, "targetPort": 8443}])
    current = copy.deepcopy(original)
    current["spec"]["clusterIP"] = "10.0.0.7"
    for p in current["spec"]["ports"]:
        p["protocol"] = "TCP"
    modified = _svc([{"name": "http", "port": 80, "targetPort": 8081}, {"name": "https", "port": 443, "targetPort": 8443}])
    patch = smp.create_three_way(original, modified, current, node)
    assert patch == {"spec": {"$setElementOrder/ports": [{"port": 80}, {"port": 443}],
                              "ports": [{"port": 80, "targetPort": 8081}]}}
    out = smp.apply(current, patch, node)
    assert out["spec"]["ports"] == [{"name": "http", "port": 80, "targetPort": 8081, "protocol": "TCP"},
                                    {"name": "https", "port": 443, "targetPort": 8443, "protocol": "TCP"}]
    assert out["spec"]["clusterIP"] == "10.0.0.7"


def test_deployment_apply_drops_exactly_one_env_var_and_one_mount():
    node = smp.schema_for("apps/v1", "Deployment")

    def dep(env, mounts, vols):
        return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"},
                "spec": {"replicas": 1, "selector": {"matchLabels": {"a": "b"}}, "template": {
                    "metadata": {"labels": {"a": "b"}},
                    "spec": {"containers": [{"name": "c", "image": "img:1", "env": env, "volumeMounts": mounts,
                                             "ports": [{"containerPort": 80}]}],
                             "volumes": vols}}}}
    env = [{"name": "A", "value": "1"}, {"name": "B", "value": "2"}, {"name": "C", "value": "3"}]
    mounts = [{"name": "v1", "mountPath": "/a"}, {"name": "v2", "mountPath": "/b"}]
    vols = [{"name": "v1", "emptyDir": {}}, {"name": "v2", "emptyDir": {}}]
    original = dep(env, mounts, vols)
    current = copy.deepcopy(original)
    c = current["spec"]["template"]["spec"]["containers"][0]
    c["env"].append({"name": "INJECTED", "value": "by-webhook"})
    c["terminationMessagePath"] = "/dev/termination-log"
    modified = dep([env[0], env[2]], [mounts[0]], vols)
    patch = smp.create_three_way(original, modified, current, node)
    out = smp.apply(current, patch, node)
    oc = out["spec"]["template"]["spec"]["containers"][0]
    assert [e["name"] for e in oc["env"]] == ["A", "C", "INJECTED"]
    assert oc["volumeMounts"] == [{"name": "v1", "mountPath": "/a"}]
    assert oc["terminationMessagePath"] == "/dev/termination-log"
    assert len(out["spec"]["template"]["spec"]["volumes"]) == 2


def test_finalizers_merge_as_a_set_and_delete_from_primitive_list():
    node = smp.schema_for("v1", "ConfigMap")
    live = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x", "finalizers": ["a", "b"]}}
    out = smp.apply(live, {"metadata": {"finalizers": ["b", "c"]}}, node)
    assert out["metadata"]["finalizers"] == ["a", "b", "c"]
    out = smp.apply(out, {"metadata": {"$deleteFromPrimitiveList/finalizers": ["a"]}}, node)
    assert out["metadata"]["finalizers"] == ["b", "c"]


def test_volumes_retain_keys_switch_source():
    """PodSpec.volumes is merge,retainKeys: switching a volume's source clears the old one."""
    node = smp.schema_for("v1", "Pod")
    original = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"},
                "spec": {"containers": [{"name": "c", "image": "i"}], "volumes": [{"name": "v", "emptyDir": {}}]}}
    modified = copy.deepcopy(original)
    modified["spec"]["volumes"] = [{"name": "v", "hostPath": {"path": "/data"}}]
    patch = smp.create_three_way(original, modified, original, node)
    vp = patch["spec"]["volumes"][0]
    assert vp["$retainKeys"] == ["hostPath", "name"] and vp["emptyDir"] is None
    out = smp.apply(original, patch, node)
    assert out["spec"]["volumes"] == [{"name": "v", "hostPath": {"path": "/data"}}]


def test_directive_errors_and_replace():
    node = smp.schema_for("v1", "Pod")
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "labels": {"a": "1", "b": "2"}},
           "spec": {"containers": [{"name": "c", "image": "i"}, {"name": "d", "image": "j"}]}}
    out = smp.apply(pod, {"spec": {"containers": [{"$patch": "replace"}, {"name": "e", "image": "k"}]}}, node)
    assert out["spec"]["containers"] == [{"name": "e", "image": "k"}]
    out = smp.apply(pod, {"metadata": {"labels": {"$patch": "replace", "z": "9"}}}, node)
    assert out["metadata"]["labels"] == {"z": "9"}
    with pytest.raises(smp.PatchError):
        smp.apply(pod, {"spec": {"containers": [{"image": "no-merge-key"}]}}, node)
    with pytest.raises(smp.PatchError):
        smp.apply(pod, {"metadata": {"$patch": "bogus"}}, node)


def test_crd_three_way_is_json_merge():
    """Kinds without a schema (custom resources) get a JSON merge three-way patch: lists replaced."""
    orig = {"apiVersion": "ex.com/v1", "kind": "Thing", "spec": {"a": 1, "b": 2, "l": [1, 2]}}
    cur = {"apiVersion": "ex.com/v1", "kind": "Thing", "spec": {"a": 1, "b": 2, "l": [1, 2], "live": True}}
    mod = {"apiVersion": "ex.com/v1", "kind": "Thing", "spec": {"a": 5, "l": [3]}}
    assert smp.create_three_way_json_merge(orig, mod, cur) == {"spec": {"a": 5, "b": None, "l": [3]}}
