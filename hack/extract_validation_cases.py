"""Extract the reference's validation test tables into tests/fixtures/validation_cases.json
(replayed by tests/test_validation_parity.py).

Sources: pkg/apis/core/validation/validation_test.go (TestValidatePersistentVolumes,
TestValidatePersistentVolumeClaim, TestValidateVolumes, TestValidatePorts,
TestValidateVolumeMounts, TestValidateContainers, TestValidatePodSpec,
TestValidateReplicationController, TestValidateLimitRange, TestValidateResourceQuota,
TestValidateEndpoints), pkg/apis/apps/validation/validation_test.go
(TestValidateStatefulSet), pkg/apis/batch/validation/validation_test.go (TestValidateCronJob),
pkg/apis/autoscaling/validation/validation_test.go (TestValidateHorizontalPodAutoscaler),
pkg/apis/policy/validation/validation_test.go (TestValidatePodDisruptionBudgetSpec).

The tables are internal-type Go literals; they are evaluated with hack/goexpr.py, turned into
the v1 JSON the apiserver serves (k8s_hook + the few internal-only shapes fixed below), and
written with the expectation the reference test asserts (success / failure, and where the
test checks it, the first error's type, field and detail).

    python hack/extract_validation_cases.py [REFERENCE_ROOT]
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import goexpr  # noqa: E402
from goexpr import Evaluator, func_body, go_string_constants, k8s_hook, statement_extent  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "validation_cases.json")
CORE = "pkg/apis/core/validation/validation_test.go"

# internal field names whose JSON spelling json_key() cannot derive
goexpr.JSON_FIELD.update({"CephFS": "cephfs", "StorageOS": "storageos", "DataDiskURI": "diskURI", "WWIDs": "wwids",
                          "DiscoveryCHAPAuth": "chapAuthDiscovery", "SessionCHAPAuth": "chapAuthSession",
                          "EndpointsName": "endpoints", "RadosUser": "user", "PodAffinityTerm": "podAffinityTerm",
                          "Template": "template", "JobTemplate": "jobTemplate"})


def _rl(**kv):
    return {k: v for k, v in kv.items() if v != ""}


def _sprintf(fmt, *args):
    import re as _re
    return _re.sub(r"%[vsdq]", lambda m, it=iter(args): str(next(it)), fmt)


def _with_affinity(pv, aff):
    """helper.StorageNodeAffinityToAlphaAnnotation: the affinity as JSON in an annotation."""
    if aff is not None:
        pv["metadata"]["annotations"] = {"volume.alpha.kubernetes.io/node-affinity": json.dumps(aff, sort_keys=True)}
    return pv


def funcs():
    def test_volume(name, ns, spec):
        md = {"name": name}
        if ns:
            md["namespace"] = ns
        return {"metadata": md, "spec": spec}

    def test_claim(name, ns, spec):
        return {"metadata": {"name": name, "namespace": ns}, "spec": spec}

    def test_claim_ann(name, ns, ann, annval, spec):
        return {"metadata": {"name": name, "namespace": ns, "annotations": {ann: annval}}, "spec": spec}
    ident = lambda x: x        # noqa: E731
    return {
        "resource.MustParse": ident, "core.ResourceName": ident, "intstr.FromInt": ident, "intstr.FromString": ident,
        "int64": ident, "int32": ident, "int": ident, "string": ident, "core.HostPathType": ident,
        "core.PersistentVolumeMode": ident, "core.ResourceQuotaScope": ident, "core.Protocol": ident,
        "core.LimitType": ident, "api.LimitType": ident, "core.PullPolicy": ident, "newInt32": ident, "boolPtr": ident,
        "newHostPathType": ident, "testVolume": test_volume,
        "testVolumeWithNodeAffinity": lambda t, name, ns, aff, spec: _with_affinity(test_volume(name, ns, spec), aff), "testVolumeClaim": test_claim,
        "testVolumeClaimAnnotation": test_claim_ann,
        "testVolumeClaimStorageClass": lambda n, ns, v, spec: test_claim_ann(n, ns, "volume.beta.kubernetes.io/storage-class", v, spec),
        "getResourceList": lambda cpu, mem: _rl(cpu=cpu, memory=mem),
        "getResourceLimits": lambda cpu, mem: {"cpu": cpu, "memory": mem},
        "getStorageResourceList": lambda s: _rl(storage=s),
        "fakeValidSecurityContext": lambda priv: {"privileged": priv},
        "utilpointer.Int32Ptr": ident, "utilpointer.Int64Ptr": ident,
        "validation.InclusiveRangeError": lambda lo, hi: f"must be between {lo} and {hi}, inclusive",
        "strings.Repeat": lambda x, n: x * n, "fmt.Sprintf": _sprintf, "core.DNSPolicy": ident,
        "core.RestartPolicy": ident, "core.TerminationMessagePolicy": ident, "core.StorageMedium": ident,
        "core.AzureDataDiskCachingMode": ident, "core.AzureDataDiskKind": ident, "core.MountPropagationMode": ident,
        "core.PersistentVolumeReclaimPolicy": ident, "core.PersistentVolumeAccessMode": ident, "core.URIScheme": ident,
        "core.Capability": ident, "core.TaintEffect": ident, "core.TolerationOperator": ident, "uint": ident,
    }


def names():
    n = {"math.MaxInt32": 2 ** 31 - 1, "t": None, "math.MaxInt64": 2 ** 63 - 1}
    # validation.go's message constants (:61-67)
    n.update({"isNegativeErrorMsg": "must be greater than or equal to 0", "isInvalidQuotaResource":
              "must be a standard resource for quota", "fieldImmutableErrorMsg": "field is immutable",
              "isNotIntegerErrorMsg": "must be an integer", "isNotPositiveErrorMsg": "must be greater than zero",
              "fileModeErrorMsg": "must be a number between 0 and 0777 (octal), both inclusive",
              "pdPartitionErrorMsg": "must be between 1 and 255, inclusive"})
    # the test file's own message prefixes (validation_test.go:41-45)
    n.update(dict(re.findall(r'^\t(\w+ErrMsg)\s*=\s*"([^"]*)"', open(os.path.join(REF, CORE)).read(), re.M)))
    # field.ErrorType values, as ErrorType.String() renders them in the message
    for k, v in (("NotFound", "Not found"), ("Required", "Required value"), ("Duplicate", "Duplicate value"),
                 ("Invalid", "Invalid value"), ("NotSupported", "Unsupported value"), ("Forbidden", "Forbidden"),
                 ("TooLong", "Too long"), ("Internal", "Internal error")):
        n["field.ErrorType" + k] = v
    n.update(go_string_constants(os.path.join(REF, "pkg/apis/core/types.go"), "core."))
    n.update(go_string_constants(os.path.join(REF, "pkg/apis/core/types.go"), "api."))
    n.update(go_string_constants(os.path.join(REF, "pkg/apis/apps/types.go"), "apps."))
    n.update(go_string_constants(os.path.join(REF, "pkg/apis/batch/types.go"), "batch."))
    n.update(go_string_constants(os.path.join(REF, "pkg/apis/autoscaling/types.go"), "autoscaling."))
    n.update(go_string_constants(os.path.join(REF, "staging/src/k8s.io/apimachinery/pkg/apis/meta/v1/types.go"), "metav1."))
    for k in list(n):
        if k.startswith("core.Resource") and not k.startswith("core.ResourceQuota"):
            n["api." + k[5:]] = n[k]
    return n


class DotEvaluator(Evaluator):
    """goexpr plus `var.Field` access into an evaluated local (validPodTemplate.Template)."""

    def unary(self):
        kind, val = self.peek()
        if kind == "ident" and "." in val and val not in self.names and val not in self.funcs and \
                self.peek(1)[1] not in ("(", "{"):
            head, *rest = val.split(".")
            if head in self.names:
                self.take()
                v = self.names[head]
                for f in rest:
                    v = v[goexpr.json_key(f)]
                return v
        return super().unary()


def evaluate_locals(src, ev, start, end, wanted=None):
    """Every `\\tname := expr` of the function body in order; returns the names that failed."""
    failed = {}
    for mt in re.finditer(r"^\t(\w+) :?= ", src[start:end], re.M):     # declarations and reassignments, in order
        i = start + mt.end()
        j = statement_extent(src, i)
        name = mt.group(1)
        try:
            ev.names[name] = ev.eval(src[i:j])
        except (SyntaxError, NameError, KeyError, ValueError, TypeError, IndexError) as e:
            near = " ".join(t[1] for t in ev.toks[max(0, ev.i - 12):ev.i + 4])
            failed[name] = f"{type(e).__name__}: {e}"[:160] + f" near: {near}"
    if wanted:
        for w in wanted:
            if w in failed:
                print(f"  ! {w}: {failed[w]}", file=sys.stderr)
    return failed


# -------------------------------------------------------------- internal → v1 JSON fixes
def fix_pod_spec(spec):
    if not isinstance(spec, dict):
        return spec
    sc = spec.get("securityContext")
    if isinstance(sc, dict):
        for k in ("hostNetwork", "hostPID", "hostIPC"):
            if k in sc:
                v = sc.pop(k)
                if v:
                    spec[k] = v
    return spec


def fix(obj, kind):
    if kind == "PodSpec":
        return fix_pod_spec(obj)
    if kind in ("Pod",):
        fix_pod_spec(obj.get("spec"))
    if kind in ("ReplicationController", "StatefulSet", "Job"):
        tpl = (obj.get("spec") or {}).get("template")
        if isinstance(tpl, dict):
            fix_pod_spec(tpl.get("spec"))
    if kind == "CronJob":
        tpl = (((obj.get("spec") or {}).get("jobTemplate") or {}).get("spec") or {}).get("template")
        if isinstance(tpl, dict):
            fix_pod_spec(tpl.get("spec"))
    return obj


TYPES = {"FieldValueNotFound": "Not found", "FieldValueRequired": "Required value", "FieldValueDuplicate": "Duplicate value",
         "FieldValueInvalid": "Invalid value", "FieldValueNotSupported": "Unsupported value",
         "FieldValueForbidden": "Forbidden", "FieldValueTooLong": "Too long", "InternalError": "Internal error"}


def rec(v, fields):
    """A positional struct literal as {field: value}."""
    return dict(zip(fields, v)) if isinstance(v, list) else v


def items(v):
    if isinstance(v, dict):
        return sorted(v.items())
    return [(str(i), x) for i, x in enumerate(v)]


def main():
    out = {}
    F, N = funcs(), names()

    def load(path, test, wanted):
        src = open(os.path.join(REF, path)).read()
        ev = DotEvaluator(F, dict(N), hook=k8s_hook)
        start, end = func_body(src, test)
        evaluate_locals(src, ev, start, end, wanted)
        return ev.names, goexpr.line_of(src, start)

    def put(test, path, line, kind, cases):
        out[test] = {"source": f"{path}:{line}", "kind": kind, "cases": cases}
        print(f"{test}: {len(cases)} cases", file=sys.stderr)

    # ---- PVs / PVCs: scenarios {isExpectedFailure, volume|claim}
    ns, line = load(CORE, "TestValidatePersistentVolumes", ["scenarios"])
    put("TestValidatePersistentVolumes", CORE, line, "PersistentVolume",
        [{"name": k, "object": v["volume"], "valid": not v.get("isExpectedFailure")} for k, v in items(ns["scenarios"])])
    ns, line = load(CORE, "TestValidatePersistentVolumeClaim", ["scenarios"])
    put("TestValidatePersistentVolumeClaim", CORE, line, "PersistentVolumeClaim",
        [{"name": k, "object": v["claim"], "valid": not v.get("isExpectedFailure")} for k, v in items(ns["scenarios"])])
    # ---- volumes: testCases {name, vol, errtype, errfield, errdetail}
    ns, line = load(CORE, "TestValidateVolumes", ["testCases"])
    cases = []
    for tc in ns["testCases"]:
        c = {"name": tc["name"], "object": tc["vol"], "valid": not tc.get("errtype")}
        if tc.get("errtype"):
            c["error"] = {"type": tc["errtype"], "field": tc.get("errfield", ""), "detail": tc.get("errdetail", "")}
        cases.append(c)
    put("TestValidateVolumes", CORE, line, "Volume", cases)
    # ---- ports: successCase, nonCanonicalCase, errorCases {P, T, F, D}
    ns, line = load(CORE, "TestValidatePorts", ["successCase", "nonCanonicalCase", "errorCases"])
    cases = [{"name": "success", "object": ns["successCase"], "valid": True},
             {"name": "non-canonical", "object": ns["nonCanonicalCase"], "valid": True}]
    for k, v in items(ns["errorCases"]):
        v = rec(v, ("P", "T", "F", "D"))
        cases.append({"name": k, "object": v["P"], "valid": False,
                      "error": {"type": v["T"], "field": v["F"], "detail": v["D"]}})
    put("TestValidatePorts", CORE, line, "ContainerPorts", cases)
    # ---- volume mounts
    ns, line = load(CORE, "TestValidateVolumeMounts",
                    ["volumes", "container", "successCase", "goodVolumeDevices", "errorCases", "badVolumeDevice"])
    cases = [{"name": "success", "object": {"mounts": ns["successCase"], "devices": ns["goodVolumeDevices"]}, "valid": True}]
    for k, v in items(ns["errorCases"]):
        cases.append({"name": k, "object": {"mounts": v, "devices": ns["badVolumeDevice"]}, "valid": False})
    out["TestValidateVolumeMounts"] = {"source": f"{CORE}:{line}", "kind": "VolumeMounts", "volumes": ns["volumes"],
                                       "container": ns["container"], "cases": cases}
    # ---- containers
    ns, line = load(CORE, "TestValidateContainers", ["successCase", "errorCases"])
    cases = [{"name": "success", "object": ns["successCase"], "valid": True}]
    cases += [{"name": k, "object": v, "valid": False} for k, v in items(ns["errorCases"])]
    put("TestValidateContainers", CORE, line, "Containers", cases)
    # ---- pod spec
    ns, line = load(CORE, "TestValidatePodSpec", ["successCases", "failureCases"])
    cases = [{"name": f"success-{i}", "object": fix(v, "PodSpec"), "valid": True} for i, v in enumerate(ns["successCases"])]
    cases += [{"name": k, "object": fix(v, "PodSpec"), "valid": False} for k, v in items(ns["failureCases"])]
    put("TestValidatePodSpec", CORE, line, "PodSpec", cases)
    # ---- replication controllers: errorCases fields checked by prefix
    ns, line = load(CORE, "TestValidateReplicationController", ["successCases", "errorCases"])
    cases = [{"name": f"success-{i}", "object": fix(v, "ReplicationController"), "valid": True}
             for i, v in enumerate(ns["successCases"])]
    cases += [{"name": k, "object": fix(v, "ReplicationController"), "valid": False} for k, v in items(ns["errorCases"])]
    put("TestValidateReplicationController", CORE, line, "ReplicationController", cases)
    # ---- limit ranges
    ns, line = load(CORE, "TestValidateLimitRange", ["successCases", "errorCases"])
    cases = [{"name": v["name"], "object": {"metadata": {"name": v["name"], "namespace": "foo"}, "spec": v["spec"]},
              "valid": True} for v in ns["successCases"]]
    cases += [{"name": k, "object": rec(v, "RD")["R"], "valid": False, "error": {"detail": rec(v, "RD")["D"]}}
              for k, v in items(ns["errorCases"])]
    put("TestValidateLimitRange", CORE, line, "LimitRange", cases)
    # ---- resource quotas
    ns, line = load(CORE, "TestValidateResourceQuota", ["successCases", "errorCases"])
    cases = [{"name": f"success-{i}", "object": v, "valid": True} for i, v in enumerate(ns["successCases"])]
    cases += [{"name": k, "object": rec(v, "RD")["R"], "valid": False, "error": {"detail": rec(v, "RD")["D"]}}
              for k, v in items(ns["errorCases"])]
    put("TestValidateResourceQuota", CORE, line, "ResourceQuota", cases)
    # ---- endpoints
    ns, line = load(CORE, "TestValidateEndpoints", ["successCases", "errorCases"])
    cases = [{"name": k, "object": v, "valid": True} for k, v in items(ns["successCases"])]
    cases += [{"name": k, "object": v["endpoints"], "valid": False,
               "error": {"type": TYPES.get(v.get("errorType"), v.get("errorType")), "detail": v.get("errorDetail", "")}}
              for k, v in items(ns["errorCases"])]
    put("TestValidateEndpoints", CORE, line, "Endpoints", cases)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
