"""Extract the LimitRanger admission tables from the reference into a JSON fixture.

Source: plugin/pkg/admission/limitranger/admission_test.go — TestPodLimitFunc (successCases /
errorCases), TestPersistentVolumeClaimLimitFunc (successCases / errorCases), and the fixtures
validLimitRange / validLimitRangeNoDefaults. The helper functions of that file
(getComputeResourceList, getLocalStorageResourceList, getStorageResourceList,
getResourceRequirements, createLimitRange, validPod, validPodInit, validPersistentVolumeClaim)
are re-expressed below over JSON objects; the tables themselves are read by hack/goexpr.py.

  python hack/extract_limitranger_cases.py [REFERENCE_ROOT]  ->  tests/fixtures/limitranger_cases.json
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, block_after, line_of  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = "plugin/pkg/admission/limitranger/admission_test.go"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "limitranger_cases.json")


def rl(x):
    return dict(x) if isinstance(x, dict) else {}


def compute(cpu, mem):
    out = {}
    if cpu:
        out["cpu"] = cpu
    if mem:
        out["memory"] = mem
    return out


def requirements(req, lim):
    out = {}
    if req is not None:
        out["requests"] = rl(req)
    if lim is not None:
        out["limits"] = rl(lim)
    return out


def limit_range(ltype, mn, mx, default, dreq, ratio):
    item = {"type": ltype}
    for k, v in (("min", mn), ("max", mx), ("default", default), ("defaultRequest", dreq),
                 ("maxLimitRequestRatio", ratio)):
        if rl(v):
            item[k] = rl(v)
    return {"apiVersion": "v1", "kind": "LimitRange", "metadata": {"name": "abc", "namespace": "test"},
            "spec": {"limits": [item]}}


def valid_pod(name, n, res):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "test"},
            "spec": {"containers": [{"name": f"foo-{i}", "image": f"foo:V{i}", "resources": json.loads(json.dumps(res or {}))}
                                    for i in range(n)]}}


def valid_pod_init(pod, *resources):
    pod = json.loads(json.dumps(pod))
    for i, res in enumerate(resources):
        pod["spec"].setdefault("initContainers", []).append(
            {"name": f"foo-{i}", "image": f"foo:V{i}", "resources": json.loads(json.dumps(res or {}))})
    return pod


def valid_pvc(name, res):
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": "test"},
            "spec": {"resources": res}}


FUNCS = {
    "getComputeResourceList": compute,
    "getLocalStorageResourceList": lambda x: {"ephemeral-storage": x} if x else {},
    "getStorageResourceList": lambda x: {"storage": x} if x else {},
    "getResourceRequirements": requirements,
    "createLimitRange": limit_range,
    "validPod": valid_pod,
    "validPodInit": valid_pod_init,
    "validPersistentVolumeClaim": valid_pvc,
}
NAMES = {"api.LimitTypeContainer": "Container", "api.LimitTypePod": "Pod",
         "api.LimitTypePersistentVolumeClaim": "PersistentVolumeClaim"}


def main():
    src = open(os.path.join(REF, SRC)).read()
    ev = Evaluator(FUNCS, NAMES)
    out = {"source": SRC, "pod": {}, "pvc": {}}
    for test, kind, obj in (("func TestPodLimitFunc(", "pod", "pod"),
                            ("func TestPersistentVolumeClaimLimitFunc(", "pvc", "pvc")):
        at = src.index(test)
        for table in ("successCases", "errorCases"):
            body, end = block_after(src, f"{table} := []testCase{{", at)
            cases = ev.eval(body)
            out[kind][table] = [{"name": c[obj]["metadata"]["name"], "line": line_of(src, src.index(table, at)),
                                 "object": c[obj], "limitRange": c["limitRange"]} for c in cases]
    # fixtures used by the default/merge tests
    for fn in ("validLimitRange", "validLimitRangeNoDefaults"):
        at = src.index(f"func {fn}()")
        body, _ = block_after(src, "Spec: api.LimitRangeSpec{", at)
        spec = ev.eval(body.replace("Limits:", "Limits:", 1))
        items = []
        for it in spec["Limits"]:
            item = {"type": it["Type"]}
            for gk, jk in (("Max", "max"), ("Min", "min"), ("Default", "default"), ("DefaultRequest", "defaultRequest")):
                if it.get(gk):
                    item[jk] = it[gk]
            items.append(item)
        out[fn] = {"apiVersion": "v1", "kind": "LimitRange", "metadata": {"name": "abc", "namespace": "test"},
                   "spec": {"limits": items}}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    n = sum(len(v) for k in ("pod", "pvc") for v in out[k].values())
    print(f"wrote {OUT}: {n} cases")


if __name__ == "__main__":
    main()
