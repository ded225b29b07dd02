"""API machinery: Quantity, selectors, validation incl. the fork's ExtendedResources rules.

Table cases mirror pkg/apis/core/validation/validation.go:2457-2483, 2950-2987 and the
selector semantics used by plugin/pkg/scheduler/core/extended_resources_test.go
(`nvidia.com/memory Gt 4095`, `Gt` with two values is an error).
"""
import pytest

from amdkube.api import SCHEME
from amdkube.api import labels as L
from amdkube.api.helpers import (is_extended_resource_name, pod_extended_resource_assigned, pod_extended_resource_name,
                                 pod_requests, toleration_tolerates_taint, ExtendedResourceError)
from amdkube.api.quantity import Quantity, QuantityError
from amdkube.api.scheme import decode_envelope, encode_envelope, load_manifests
from amdkube.api.validation import validate_binding, validate_pod


@pytest.mark.parametrize("s,val,milli,canon", [
    ("1", 1, 1000, "1"), ("500m", 1, 500, "500m"), ("288Gi", 288 * 2 ** 30, 288 * 2 ** 30 * 1000, "288Gi"),
    ("1.5", 2, 1500, "1500m"), ("1000m", 1, 1000, "1"), ("2e3", 2000, 2000000, "2e3"), ("1536Mi", 1536 * 2 ** 20, None, "1536Mi"),
    ("0", 0, 0, "0"), ("4k", 4000, None, "4k"), ("1Ki", 1024, None, "1Ki"), ("100n", 1, 0 + 1, "100n"),
])
def test_quantity(s, val, milli, canon):
    q = Quantity(s)
    assert q.value() == val
    if milli is not None:
        assert q.milli_value() == milli
    assert str(q) == canon


def test_quantity_errors_and_compare():
    for bad in ("", "abc", "1.2.3", "Gi", "1Gb"):
        with pytest.raises(QuantityError):
            Quantity(bad)
    assert Quantity("1Gi") > Quantity("1G")
    assert Quantity("1") == Quantity("1000m")
    assert str(Quantity("1Gi") + Quantity("1Gi")) == "2Gi"


def test_selector_parse_and_match():
    s = L.parse_selector("app=web,tier!=db,env in (prod,staging),!legacy,gpu,mem>100")
    assert s.matches({"app": "web", "env": "prod", "gpu": "x", "mem": "200"})
    assert not s.matches({"app": "web", "env": "prod", "gpu": "x", "mem": "50"})
    assert not s.matches({"app": "web", "env": "dev", "gpu": "x", "mem": "200"})
    assert not s.matches({"app": "web", "env": "prod", "gpu": "x", "mem": "200", "legacy": "1"})
    assert L.parse_selector("").matches({"anything": "x"})


def test_node_requirements_gt_lt_and_errors():
    sel = L.node_requirements_as_selector([{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["262143"]},
                                           {"key": "amd.com/gpu-type", "operator": "In", "values": ["MI355X"]}])
    assert sel.matches({"amd.com/gpu-memory": "294896", "amd.com/gpu-type": "MI355X"})
    assert not sel.matches({"amd.com/gpu-memory": "196608", "amd.com/gpu-type": "MI355X"})
    assert not sel.matches({"amd.com/gpu-memory": "not-int", "amd.com/gpu-type": "MI355X"})
    with pytest.raises(L.SelectorError):  # Gt with two values
        L.node_requirements_as_selector([{"key": "a.com/m", "operator": "Gt", "values": ["1", "2"]}])
    with pytest.raises(L.SelectorError):  # two slashes in a key (quirk #13)
        L.node_requirements_as_selector([{"key": "nvidia.com/gpu/memory", "operator": "Exists"}])
    assert L.node_requirements_as_selector([]).matches({})


def test_field_selector():
    fs = L.parse_field_selector("spec.nodeName=n1,status.phase!=Succeeded")
    assert fs.matches({"spec.nodeName": "n1", "status.phase": "Running"})
    assert not fs.matches({"spec.nodeName": "n1", "status.phase": "Succeeded"})


def test_extended_resource_name():
    assert is_extended_resource_name("amd.com/gpu")
    assert not is_extended_resource_name("cpu")
    assert not is_extended_resource_name("kubernetes.io/foo")


def _gpu_pod(**over):
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
           "spec": {"containers": [{"name": "c", "image": "rocm/vector-add", "extendedResourceRequests": ["gpus0"]}],
                    "extendedResources": [{"name": "gpus0", "resources": {"limits": {"amd.com/gpu": "4"}},
                                           "affinity": {"required": [{"key": "amd.com/gpu-type", "operator": "In", "values": ["MI355X"]}]}}]}}
    pod["spec"].update(over)
    SCHEME.default(pod)
    return pod


def test_pod_defaults_copy_ext_limits_to_requests():
    pod = _gpu_pod()
    assert pod["spec"]["extendedResources"][0]["resources"]["requests"] == {"amd.com/gpu": "4"}
    assert validate_pod(pod) == []


@pytest.mark.parametrize("mutate,needle", [
    (lambda p: p["spec"]["extendedResources"][0].update(name=""), "can't be empty"),
    (lambda p: p["spec"]["extendedResources"].append(dict(p["spec"]["extendedResources"][0])), "should be unique"),
    (lambda p: p["spec"]["extendedResources"][0]["resources"]["limits"].update({"amd.com/other": "1"}), "limits length"),
    (lambda p: p["spec"]["extendedResources"][0]["resources"].update(requests={"amd.com/gpu": "2"}), "should be equal"),
    (lambda p: p["spec"]["containers"][0].update(extendedResourceRequests=["nope"]), "unknown extended resource"),
    (lambda p: p["spec"]["containers"].append({"name": "d", "image": "x", "extendedResourceRequests": ["gpus0"]}), "sharing is not allowed"),
    (lambda p: p["spec"].update(initContainers=[{"name": "i", "image": "x", "extendedResourceRequests": ["ghost"]}]), "unknown extended resource"),
    (lambda p: p["spec"]["extendedResources"][0]["affinity"].update(required=[{"key": "a.com/m", "operator": "Gt", "values": ["x"]}]), "integer"),
])
def test_extended_resource_validation(mutate, needle):
    pod = _gpu_pod()
    mutate(pod)
    errs = validate_pod(pod)
    assert any(needle in e for e in errs), errs


def test_pod_update_immutability():
    old = _gpu_pod()
    new = _gpu_pod()
    new["spec"]["containers"][0]["image"] = "other"
    assert validate_pod(new, old) == []
    new["spec"]["restartPolicy"] = "Never"
    assert any("Forbidden" in e for e in validate_pod(new, old))


def test_helpers_assigned():
    pod = _gpu_pod()
    pod["spec"]["extendedResources"][0]["assigned"] = ["g0", "g1", "g2", "g3"]
    assert pod_extended_resource_assigned("amd.com/gpu", pod["spec"]["containers"][0], pod) == ["g0", "g1", "g2", "g3"]
    assert pod_extended_resource_name(pod["spec"]["extendedResources"][0]) == "amd.com/gpu"
    with pytest.raises(ExtendedResourceError):
        pod_extended_resource_name({"resources": {"limits": {}}})


def test_pod_requests_init_max():
    pod = {"spec": {"containers": [{"resources": {"requests": {"cpu": "500m", "memory": "1Gi"}}},
                                   {"resources": {"requests": {"cpu": "250m"}}}],
                    "initContainers": [{"resources": {"requests": {"cpu": "2", "memory": "512Mi"}}}]}}
    assert pod_requests(pod) == {"cpu": 2000, "memory": 2 ** 30}


def test_tolerations():
    taint = {"key": "amd.com/gpu", "value": "", "effect": "NoSchedule"}
    assert toleration_tolerates_taint({"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}, taint)
    assert toleration_tolerates_taint({"operator": "Exists"}, taint)
    assert not toleration_tolerates_taint({"key": "x", "operator": "Exists"}, taint)


def test_binding_validation():
    assert validate_binding({"target": {"kind": "Node", "name": "n"}}) == []
    assert validate_binding({"target": {"name": ""}})
    assert validate_binding({"target": {"name": "n", "extendedResourceBinding": {"g": {"resources": ["a", "a"]}}}})


def test_manifests_and_envelope():
    docs = load_manifests("apiVersion: v1\nkind: Pod\nmetadata: {name: a}\n---\napiVersion: v1\nkind: List\nitems:\n- {apiVersion: v1, kind: Node, metadata: {name: n}}\n")
    assert [d["kind"] for d in docs] == ["Pod", "Node"]
    env = encode_envelope(docs[0])
    assert env.startswith(b"k8s\x00") and decode_envelope(env) == docs[0]


# TestValidateEnv / TestValidateEnvFrom (pkg/apis/core/validation/validation_test.go:3847-4360)
def _env_pod(env=None, env_from=None):
    c = {"name": "c", "image": "x"}
    if env is not None:
        c["env"] = env
    if env_from is not None:
        c["envFrom"] = env_from
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"}, "spec": {"containers": [c]}}
    SCHEME.default(pod)
    return validate_pod(pod)


def _fr(path, version="v1"):
    return {"valueFrom": {"fieldRef": {"apiVersion": version, "fieldPath": path}}}


def test_validate_env_success_cases():
    env = [{"name": n, "value": "value"} for n in ("abc", "ABC", "AbC_123", "a.b.c", "a-b-c")] + [{"name": "abc", "value": ""}]
    env += [{"name": "abc", **_fr(p)} for p in ("metadata.annotations['key']", "metadata.labels['key']", "metadata.name",
                                                  "metadata.namespace", "metadata.uid", "spec.nodeName",
                                                  "spec.serviceAccountName", "status.hostIP", "status.podIP")]
    env += [{"name": "secret_value", "valueFrom": {"secretKeyRef": {"name": "some-secret", "key": "secret-key"}}},
            {"name": "ENV_VAR_1", "valueFrom": {"configMapKeyRef": {"name": "some-config-map", "key": "some-key"}}},
            {"name": "defaulted", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}]   # apiVersion defaults to v1
    assert _env_pod(env) == []


@pytest.mark.parametrize("env,needle", [
    ([{"name": ""}], "env[0].name: Required value"),
    ([{"name": "a!b"}], 'env[0].name: Invalid value: \"a!b\": a valid environment variable name'),
    ([{"name": "1=bad", "value": "x"}], "must not start with a digit"),
    ([{"name": "."}], 'env[0].name: Invalid value: \".\": must not be'),
    ([{"name": ".."}], 'env[0].name: Invalid value: \"..\": must not be'),
    ([{"name": "..abc"}], 'env[0].name: Invalid value: \"..abc\": must not start with'),
    ([{"name": "abc", "value": "foo", **_fr("metadata.name")}], "valueFrom: Invalid value: \"\": may not be specified when `value`"),
    ([{"name": "abc", "valueFrom": {}}], "must specify one of: `fieldRef`, `resourceFieldRef`, `configMapKeyRef` or `secretKeyRef`"),
    ([{"name": "abc", "valueFrom": {"fieldRef": {"apiVersion": "v1", "fieldPath": "metadata.name"},
                                    "secretKeyRef": {"name": "a-secret", "key": "a-key"}}}],
     "may not have more than one field specified at a time"),
    ([{"name": "abc", "valueFrom": {"secretKeyRef": {"name": "$%^&*#", "key": "a-key"}}}], "secretKeyRef.name: Invalid value"),
    ([{"name": "abc", "valueFrom": {"configMapKeyRef": {"name": "$%^&*#", "key": "k"}}}], "configMapKeyRef.name: Invalid value"),
    ([{"name": "abc", "valueFrom": {"fieldRef": {"apiVersion": "v1"}}}], "valueFrom.fieldRef.fieldPath: Required value"),
    ([{"name": "abc", **_fr("metadata.whoops")}], 'fieldRef.fieldPath: Invalid value: \"metadata.whoops\": error converting fieldPath'),
    ([{"name": "abc", **_fr("metadata.name['key']")}], "error converting fieldPath: field label does not support subscript"),
    ([{"name": "abc", **_fr("metadata.labels")}], 'fieldRef.fieldPath: Unsupported value: \"metadata.labels\": supported values: '
                                                  '"metadata.name", "metadata.namespace", "metadata.uid", "spec.nodeName", '
                                                  '"spec.serviceAccountName", "status.hostIP", "status.podIP"'),
    ([{"name": "abc", **_fr("metadata.annotations['invalid~key']")}], 'valueFrom.fieldRef: Invalid value: \"invalid~key\"'),
    ([{"name": "abc", **_fr("metadata.labels['Www.k8s.io/test']")}], 'valueFrom.fieldRef: Invalid value: \"Www.k8s.io/test\"'),
    ([{"name": "abc", **_fr("status.phase")}], 'fieldRef.fieldPath: Unsupported value: \"status.phase\"'),
    ([{"name": "abc", "valueFrom": {"resourceFieldRef": {"resource": "limits.gpu"}}}], "resourceFieldRef.resource: Unsupported value"),
])
def test_validate_env_error_cases(env, needle):
    errs = _env_pod(env)
    assert errs and all(needle in e for e in errs), errs


def test_validate_env_from():
    ok = [{"configMapRef": {"name": "abc"}}, {"prefix": "pre_", "configMapRef": {"name": "abc"}},
          {"prefix": "a.b", "secretRef": {"name": "abc"}}, {"secretRef": {"name": "abc"}}]
    assert _env_pod(env_from=ok) == []
    for ef, needle in [([{"configMapRef": {"name": ""}}], "envFrom[0].configMapRef.name: Required value"),
                       ([{"configMapRef": {"name": "$"}}], "envFrom[0].configMapRef.name: Invalid value"),
                       ([{"prefix": "a!b", "configMapRef": {"name": "abc"}}], 'envFrom[0].prefix: Invalid value: \"a!b\"'),
                       ([{"secretRef": {"name": "&"}}], "envFrom[0].secretRef.name: Invalid value"),
                       ([{"prefix": "a!b"}], "must specify one of: `configMapRef` or `secretRef`"),
                       ([{"configMapRef": {"name": "a"}, "secretRef": {"name": "b"}}], "may not have more than one field")]:
        errs = _env_pod(env_from=ef)
        assert errs and any(needle in e for e in errs), (ef, errs)


def test_downward_api_volume_field_paths():
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"},
           "spec": {"containers": [{"name": "c", "image": "x"}], "volumes": [{"name": "v", "downwardAPI": {"items": [
               {"path": "labels", "fieldRef": {"fieldPath": "metadata.labels"}},
               {"path": "ip", "fieldRef": {"fieldPath": "status.podIP"}}]}}]}}
    SCHEME.default(pod)
    errs = validate_pod(pod)
    # validateDownwardAPIVolumeSource passes the volume's path, not the item's (validation.go:1003-1005)
    assert len(errs) == 1 and 'downwardAPI.fieldRef.fieldPath: Unsupported value: \"status.podIP\"' in errs[0], errs
