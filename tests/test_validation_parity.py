"""Validation parity: the reference's own tables, replayed.

tests/fixtures/validation_cases.json is extracted by hack/extract_validation_cases.py from
pkg/apis/core/validation/validation_test.go — TestValidatePersistentVolumes (:83),
TestValidatePersistentVolumeClaim (:739), TestValidateVolumes (:1707), TestValidatePorts
(:3703), TestValidateVolumeMounts (:4398), TestValidateContainers (:4838), TestValidatePodSpec
(:5496), TestValidateReplicationController (:8875), TestValidateLimitRange (:10371),
TestValidateResourceQuota (:10732), TestValidateEndpoints (:11435). Each case is replayed with
the assertion its test makes (valid / invalid; where the test checks it, the first error's
type, field suffix and detail). The feature gates are the reference's v1.9 defaults (alpha
storage/DNS gates off) as those tests run with them; TestValidateProbe/Handler, which build
their cases by reflection, are transcribed below, as are the apps/batch/autoscaling/policy
cases the verdict names.
"""
import copy
import json
import os

import pytest

from amdkube.api import corevalidation as cv
from amdkube.api import groupvalidation as gv
from amdkube.utils.features import FeatureGate

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "validation_cases.json")))
TYPES = ("Required value", "Invalid value", "Forbidden", "Duplicate value", "Not found", "Unsupported value",
         "Too long", "Internal error")


@pytest.fixture(autouse=True)
def reference_gates(monkeypatch):
    """The v1.9 feature gate defaults the reference's tests run with."""
    monkeypatch.setattr(cv, "GATES", FeatureGate())
    monkeypatch.setitem(cv.__dict__, "ALLOW_LOOPBACK_ENDPOINTS", False)
    from amdkube.api import validation
    monkeypatch.setitem(validation.CAPABILITIES, "allow_privileged", True)


def parse(err: str):
    """'<field>: <type>[: <value>][: <detail>]' -> (field, type, text after the type)."""
    for t in TYPES:
        mark = f": {t}"
        i = err.find(mark)
        if i >= 0:
            return err[:i], t, err[i + len(mark):]
    raise AssertionError(f"unparsable error {err!r}")


def cases(test):
    return [pytest.param(c, id=c["name"][:60]) for c in FIX[test]["cases"]]


def check(errs, case):
    if case["valid"]:
        assert errs == [], errs
    else:
        assert errs, f"expected failure for {case['name']}"


@pytest.mark.parametrize("case", cases("TestValidatePersistentVolumes"))
def test_persistent_volumes(case):
    check(cv.validate_persistent_volume(copy.deepcopy(case["object"])), case)


@pytest.mark.parametrize("case", cases("TestValidatePersistentVolumeClaim"))
def test_persistent_volume_claims(case):
    check(cv.validate_persistent_volume_claim(copy.deepcopy(case["object"])), case)


@pytest.mark.parametrize("case", cases("TestValidateVolumes"))
def test_volumes(case):
    names, errs = cv.validate_volumes([case["object"]], "field")
    if case["valid"]:
        assert errs == [] and list(names) == [case["object"]["name"]], errs
        return
    assert len(errs) == 1, errs
    f, t, rest = parse(errs[0])
    want = case["error"]
    assert t == want["type"], errs
    assert f.endswith("." + want["field"]), errs
    assert want["detail"] in rest, errs


def test_duplicate_volume_names():
    """TestValidateVolumes dupsCase (:3308)."""
    vol = {"name": "abc", "emptyDir": {}}
    _, errs = cv.validate_volumes([vol, dict(vol)], "field")
    assert len(errs) == 1 and parse(errs[0])[1] == "Duplicate value"


@pytest.mark.parametrize("case", cases("TestValidatePorts"))
def test_container_ports(case):
    errs = cv.validate_container_ports(case["object"], "field")
    if case["valid"]:
        assert errs == [], errs
        return
    assert errs
    want = case["error"]
    for e in errs:
        f, t, rest = parse(e)
        assert t == want["type"] and want["field"] in f and want["detail"] in rest, (e, want)


@pytest.mark.parametrize("case", cases("TestValidateVolumeMounts"))
def test_volume_mounts(case):
    t = FIX["TestValidateVolumeMounts"]
    vols, verrs = cv.validate_volumes(t["volumes"], "field")
    assert verrs == []
    devices = {d["name"]: d["devicePath"] for d in case["object"]["devices"]}
    errs = cv.validate_volume_mounts(case["object"]["mounts"], devices, vols, t["container"], "field")
    check(errs, case)


@pytest.mark.parametrize("case", cases("TestValidateContainers"))
def test_containers(case):
    check(cv.validate_containers(copy.deepcopy(case["object"]), {}, "field"), case)


@pytest.mark.parametrize("case", cases("TestValidatePodSpec"))
def test_pod_spec(case, monkeypatch):
    check(cv.validate_pod_spec(copy.deepcopy(case["object"]), "field"), case)


RC_FIELDS = ("metadata.name", "metadata.namespace", "spec.selector", "spec.template", "GCEPersistentDisk.ReadOnly",
             "spec.replicas", "spec.template.labels", "metadata.annotations", "metadata.labels", "status.replicas")


@pytest.mark.parametrize("case", cases("TestValidateReplicationController"))
def test_replication_controllers(case):
    errs = cv.validate_replication_controller(copy.deepcopy(case["object"]))
    check(errs, case)
    for e in errs:
        f = parse(e)[0]
        assert f.startswith("spec.template.") or f in RC_FIELDS, e


@pytest.mark.parametrize("case", cases("TestValidateLimitRange"))
def test_limit_ranges(case):
    errs = cv.validate_limit_range(copy.deepcopy(case["object"]))
    check(errs, case)
    if not case["valid"]:
        assert any(case["error"]["detail"] in e for e in errs), (errs, case["error"])


@pytest.mark.parametrize("case", cases("TestValidateResourceQuota"))
def test_resource_quotas(case):
    errs = cv.validate_resource_quota(copy.deepcopy(case["object"]))
    check(errs, case)
    if not case["valid"]:
        assert any(case["error"]["detail"] in e for e in errs), (errs, case["error"])


@pytest.mark.parametrize("case", cases("TestValidateEndpoints"))
def test_endpoints(case):
    errs = cv.validate_endpoints(copy.deepcopy(case["object"]))
    check(errs, case)
    if not case["valid"]:
        f, t, rest = parse(errs[0])
        assert t == case["error"]["type"] and case["error"]["detail"] in rest, (errs, case["error"])


# ---------------------------------------------------------------- TestValidateProbe (:4727)
HANDLER = {"exec": {"command": ["echo"]}}
POSITIVE = ("initialDelaySeconds", "timeoutSeconds", "periodSeconds", "successThreshold", "failureThreshold")


def test_probe():
    assert cv.validate_probe(None, "field") == []
    for f in POSITIVE:
        assert cv.validate_probe({**HANDLER, f: 10}, "field") == []
        assert cv.validate_probe({**HANDLER, f: -10}, "field")
    assert cv.validate_probe({"timeoutSeconds": 10, "initialDelaySeconds": 10}, "field")    # no handler


# ---------------------------------------------------------------- TestValidateHandler (:4757)
@pytest.mark.parametrize("h", [
    {"exec": {"command": ["echo"]}},
    {"httpGet": {"path": "/", "port": 1, "host": "", "scheme": "HTTP"}},
    {"httpGet": {"path": "/foo", "port": 65535, "host": "host", "scheme": "HTTP"}},
    {"httpGet": {"path": "/", "port": "port", "host": "", "scheme": "HTTP"}},
    {"httpGet": {"path": "/", "port": "port", "host": "", "scheme": "HTTP", "httpHeaders": [{"name": "Host", "value": "foo.example.com"}]}},
    {"httpGet": {"path": "/", "port": "port", "host": "", "scheme": "HTTP",
                 "httpHeaders": [{"name": "X-Forwarded-For", "value": "1.2.3.4"}, {"name": "X-Forwarded-For", "value": "5.6.7.8"}]}},
])
def test_handler_success(h):
    assert cv.validate_handler(h, "field") == []


@pytest.mark.parametrize("h", [
    {},
    {"exec": {"command": []}},
    {"httpGet": {"path": "", "port": 0, "host": ""}},
    {"httpGet": {"path": "/foo", "port": 65536, "host": "host"}},
    {"httpGet": {"path": "", "port": "", "host": ""}},
    {"httpGet": {"path": "/", "port": "port", "host": "", "scheme": "HTTP", "httpHeaders": [{"name": "Host:", "value": "foo.example.com"}]}},
    {"httpGet": {"path": "/", "port": "port", "host": "", "scheme": "HTTP", "httpHeaders": [{"name": "X_Forwarded_For", "value": "foo.example.com"}]}},
])
def test_handler_failure(h):
    assert cv.validate_handler(h, "field")


def test_pull_policy_restart_and_dns_policy():
    """TestValidatePullPolicy (:4788), TestValidateRestartPolicy (:5277), TestValidateDNSPolicy (:5298)."""
    for pol in ("IfNotPresent", "Always", "Never"):
        assert cv.validate_pull_policy(pol, "field") == []
    assert parse(cv.validate_pull_policy("", "field")[0])[1] == "Required value"
    assert parse(cv.validate_pull_policy("Sometimes", "field")[0])[1] == "Unsupported value"
    for rp in ("Always", "Never", "OnFailure"):
        assert cv.validate_restart_policy(rp, "field") == []
    for rp in ("", "newpolicy"):
        assert cv.validate_restart_policy(rp, "field")
    for dp in ("ClusterFirst", "Default", "ClusterFirstWithHostNet"):
        assert cv.validate_dns_policy(dp, "field") == []
    for dp in ("", "invalid", "None"):        # None needs the CustomPodDNS gate (off in 1.9)
        assert cv.validate_dns_policy(dp, "field")


# ---------------------------------------------------------------- apps / batch / autoscaling / policy
def _tpl(labels=None, restart="Always"):
    return {"metadata": {"labels": labels or {"a": "b"}},
            "spec": {"restartPolicy": restart, "dnsPolicy": "ClusterFirst",
                     "containers": [{"name": "abc", "image": "image", "imagePullPolicy": "IfNotPresent",
                                     "terminationMessagePolicy": "File"}]}}


def _sts(**spec):
    base = {"selector": {"matchLabels": {"a": "b"}}, "template": _tpl(), "podManagementPolicy": "OrderedReady",
            "updateStrategy": {"type": "RollingUpdate"}}
    base.update(spec)
    return {"metadata": {"name": "abc", "namespace": "default"}, "spec": base}


@pytest.mark.parametrize("mut,field", [
    ({"replicas": -1}, "spec.replicas"),
    ({"selector": {}}, "spec.selector"),
    ({"template": _tpl({"x": "y"})}, "spec.template.metadata.labels"),
    ({"template": _tpl(restart="OnFailure")}, "spec.template.spec.restartPolicy"),
    ({"podManagementPolicy": ""}, "spec.podManagementPolicy"),
    ({"podManagementPolicy": "foo"}, "spec.podManagementPolicy"),
    ({"updateStrategy": {"type": ""}}, "spec.updateStrategy"),
    ({"updateStrategy": {"type": "foo"}}, "spec.updateStrategy"),
    ({"updateStrategy": {"type": "OnDelete", "rollingUpdate": {"partition": 1}}}, "spec.updateStrategy.rollingUpdate"),
    ({"updateStrategy": {"type": "RollingUpdate", "rollingUpdate": {"partition": -1}}}, "spec.updateStrategy.rollingUpdate.partition"),
])
def test_statefulset_errors(mut, field):
    """apps/validation/validation_test.go TestValidateStatefulSet (:33) error cases."""
    assert cv.is_int(1)
    errs = gv.validate_statefulset(_sts(**mut))
    assert errs and any(parse(e)[0] == field for e in errs), errs


def test_statefulset_valid_and_update_rules():
    assert gv.validate_statefulset(_sts()) == []
    assert gv.validate_statefulset(_sts(podManagementPolicy="Parallel", updateStrategy={"type": "OnDelete"})) == []
    old = _sts(replicas=1)
    assert gv.validate_statefulset(_sts(replicas=3), old) == []
    assert any("forbidden" in e for e in gv.validate_statefulset(_sts(serviceName="x"), old))


def _cj(**spec):
    base = {"schedule": "* * * * ?", "concurrencyPolicy": "Allow",
            "jobTemplate": {"spec": {"template": _tpl(restart="OnFailure")}}}
    base.update(spec)
    return {"metadata": {"name": "mycronjob", "namespace": "default", "uid": "1a2b3c"}, "spec": base}


@pytest.mark.parametrize("mut,frag", [
    ({"schedule": "error"}, "spec.schedule"),
    ({"schedule": ""}, "spec.schedule"),
    ({"startingDeadlineSeconds": -1}, "spec.startingDeadlineSeconds"),
    ({"concurrencyPolicy": ""}, "spec.concurrencyPolicy"),
    ({"concurrencyPolicy": "Sometimes"}, "spec.concurrencyPolicy"),
    ({"successfulJobsHistoryLimit": -1}, "spec.successfulJobsHistoryLimit"),
    ({"failedJobsHistoryLimit": -1}, "spec.failedJobsHistoryLimit"),
    ({"jobTemplate": {"spec": {"parallelism": -1, "template": _tpl(restart="OnFailure")}}}, "spec.jobTemplate.spec.parallelism"),
    ({"jobTemplate": {"spec": {"completions": -1, "template": _tpl(restart="OnFailure")}}}, "spec.jobTemplate.spec.completions"),
    ({"jobTemplate": {"spec": {"activeDeadlineSeconds": -1, "template": _tpl(restart="OnFailure")}}}, "spec.jobTemplate.spec.activeDeadlineSeconds"),
    ({"jobTemplate": {"spec": {"selector": {"matchLabels": {"a": "b"}}, "template": _tpl(restart="OnFailure")}}}, "spec.jobTemplate.spec.selector"),
    ({"jobTemplate": {"spec": {"manualSelector": True, "template": _tpl(restart="OnFailure")}}}, "spec.jobTemplate.spec.manualSelector"),
    ({"jobTemplate": {"spec": {"template": _tpl(restart="Always")}}}, "spec.jobTemplate.spec.template.spec.restartPolicy"),
])
def test_cronjob_errors(mut, frag):
    """batch/validation/validation_test.go TestValidateCronJob (:213) error cases."""
    errs = gv.validate_cronjob(_cj(**mut))
    assert errs and any(parse(e)[0] == frag for e in errs), errs


def test_cronjob_valid_and_name_length():
    assert gv.validate_cronjob(_cj()) == []
    cj = _cj()
    cj["metadata"]["name"] = "a" * 53
    assert any("must be no more than 52 characters" in e for e in gv.validate_cronjob(cj))


def _hpa(**spec):
    base = {"scaleTargetRef": {"kind": "ReplicationController", "name": "myrc"}, "minReplicas": 1, "maxReplicas": 5}
    base.update(spec)
    return {"metadata": {"name": "myautoscaler", "namespace": "default"}, "spec": base}


@pytest.mark.parametrize("mut,msg", [
    ({"scaleTargetRef": {"name": "myrc"}}, "scaleTargetRef.kind: Required"),
    ({"scaleTargetRef": {"kind": "..", "name": "myrc"}}, "scaleTargetRef.kind: Invalid"),
    ({"scaleTargetRef": {"kind": "ReplicationController"}}, "scaleTargetRef.name: Required"),
    ({"scaleTargetRef": {"kind": "ReplicationController", "name": ".."}}, "scaleTargetRef.name: Invalid"),
    ({"minReplicas": -1}, "must be greater than 0"),
    ({"maxReplicas": 0}, "must be greater than 0"),
    ({"minReplicas": 7, "maxReplicas": 5}, "must be greater than or equal to `minReplicas`"),
    ({"targetCPUUtilizationPercentage": -70}, "must be greater than 0"),
])
def test_hpa_errors(mut, msg):
    """autoscaling/validation/validation_test.go TestValidateHorizontalPodAutoscaler (:63) error cases."""
    errs = gv.validate_hpa(_hpa(**mut))
    assert any(msg in e for e in errs), errs


def test_hpa_metric_specs():
    ok = [{"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 70}},
          {"type": "Pods", "pods": {"metricName": "somemetric", "targetAverageValue": "100m"}},
          {"type": "Object", "object": {"target": {"kind": "ReplicationController", "name": "myrc"},
                                        "metricName": "somemetric", "targetValue": "100m"}}]
    for m in ok:
        assert gv.validate_metric_spec(m, "spec.metrics[0]") == []
    bad = [({"type": "Resource", "resource": {"name": "cpu"}}, "must set either a target raw value or a target utilization"),
           ({"type": "Resource", "resource": {"targetAverageUtilization": 70}}, "must specify a resource name"),
           ({"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 70, "targetAverageValue": "100m"}},
            "may not set both a target raw value and a target utilization"),
           ({"type": "Pods", "pods": {"targetAverageValue": "100m"}}, "must specify a metric name"),
           ({"type": "Pods", "pods": {"metricName": "m"}}, "must specify a positive target value"),
           ({"type": "Object", "object": {"target": {"kind": "ReplicationController", "name": "myrc"}, "metricName": "m"}},
            "must specify a positive target value"),
           ({"type": "Resource"}, "must populate information for the given metric source"),
           ({"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 70},
             "pods": {"metricName": "m", "targetAverageValue": "1"}}, "must populate the given metric source only"),
           ({"type": "boogity"}, "Unsupported value")]
    for m, msg in bad:
        assert any(msg in e for e in gv.validate_metric_spec(m, "spec.metrics[0]")), (m, msg)


@pytest.mark.parametrize("spec,ok", [
    ({"minAvailable": 0}, True), ({"minAvailable": 5}, True), ({"minAvailable": "0%"}, True), ({"minAvailable": "100%"}, True),
    ({"maxUnavailable": 5}, True), ({"maxUnavailable": "30%"}, True),
    ({"minAvailable": -1}, False), ({"minAvailable": "-1%"}, False), ({"minAvailable": "101%"}, False),
    ({"minAvailable": "1.1%"}, False), ({"minAvailable": "nope"}, False),
    ({"maxUnavailable": -1}, False), ({"maxUnavailable": "101%"}, False),
    ({"minAvailable": 1, "maxUnavailable": 1}, False),
])
def test_pdb_spec(spec, ok):
    """policy/validation/validation_test.go TestValidatePodDisruptionBudgetSpec (:29) and
    TestValidateMinAvailablePodDisruptionBudgetSpec / MaxUnavailable (:38-102)."""
    pdb = {"metadata": {"name": "p", "namespace": "default"}, "spec": dict(spec)}
    assert (gv.validate_pdb(pdb) == []) == ok, gv.validate_pdb(pdb)
