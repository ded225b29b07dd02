"""Extract the scheduler predicate tables from the reference into a JSON fixture.

Source: plugin/pkg/scheduler/algorithm/predicates/predicates_test.go. Every table-driven test
whose cases are plain data is read by hack/goexpr.py (Go struct literals become the JSON the
apiserver serves, via goexpr.k8s_hook; core/v1 and meta/v1 constants are read from the
reference's types.go; Err* failure reasons from error.go). The file's helper constructors
(newResourcePod, makeResources, newPod, ...) are re-expressed below over JSON objects. A
`schedulercache.NewNodeInfo(pods...)` becomes {"nodeInfoPods": [...]} and the test replays it
into an amdkube NodeInfo.

  python hack/extract_predicates_cases.py [REFERENCE_ROOT]  ->  tests/fixtures/predicates_cases.json
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, eval_locals, func_body, k8s_hook, k8s_names, table  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
PKG = "plugin/pkg/scheduler/algorithm/predicates"
SRC = PKG + "/predicates_test.go"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "predicates_cases.json")


# ------------------------------------------------------------------ helpers of predicates_test.go
def resource_list(r: dict) -> dict:
    """schedulercache.Resource.ResourceList()."""
    out = {"cpu": f"{r.get('milliCPU', 0)}m", "memory": str(r.get("memory", 0)),
           "alpha.kubernetes.io/nvidia-gpu": str(r.get("nvidiaGPU", 0)),
           "ephemeral-storage": str(r.get("ephemeralStorage", 0))}
    for k, v in (r.get("scalarResources") or {}).items():
        out[k] = str(v)
    return out


def new_resource_pod(*usage):
    return {"metadata": {}, "spec": {"containers": [{"resources": {"requests": resource_list(u)}} for u in usage]}}


def new_resource_init_pod(pod, *usage):
    pod = json.loads(json.dumps(pod))
    pod["spec"]["initContainers"] = new_resource_pod(*usage)["spec"]["containers"]
    return pod


def allocatable(milli_cpu, memory, gpus, pods, ext_a, storage, hugepage_a):
    return {"cpu": f"{milli_cpu}m", "memory": str(memory), "pods": str(pods),
            "alpha.kubernetes.io/nvidia-gpu": str(gpus), "example.com/aaa": str(ext_a),
            "ephemeral-storage": str(storage), "hugepages-2Mi": str(hugepage_a)}


def new_port_pod(host, *infos):
    ports = []
    for info in infos:
        proto, ip, port = info.split("/")
        ports.append({"hostIP": ip, "hostPort": int(port), "protocol": proto})
    return {"metadata": {}, "spec": {"nodeName": host, "containers": [{"ports": ports}]}}


def new_pod_with_port(*ports):
    return {"metadata": {}, "spec": {"containers": [{"ports": [{"hostPort": p} for p in ports]}]}}


def node_info(*pods):
    return {"nodeInfoPods": list(pods)}


def empty_node_info(node):
    return {"nodeInfoPods": [], "node": node}


def pod_with_volume(name, vol, claim):
    return {"metadata": {"name": name, "namespace": "default"},
            "spec": {"volumes": [{"name": vol, "persistentVolumeClaim": {"claimName": claim}}]}}


def insufficient(name, requested, used, capacity):
    return f"Insufficient {name}"


FUNCS = {
    "newResourcePod": new_resource_pod, "newResourceInitPod": new_resource_init_pod,
    "makeAllocatableResources": allocatable, "makeResourcesCapacity": allocatable,
    "newPod": new_port_pod, "newPodWithPort": new_pod_with_port,
    "schedulercache.NewNodeInfo": node_info, "makeEmptyNodeInfo": empty_node_info,
    "NewInsufficientResourceError": insufficient, "createPodWithVolume": pod_with_volume,
    "resource.NewMilliQuantity": lambda v, fmt=None: f"{v}m", "resource.NewQuantity": lambda v, fmt=None: str(v),
    "resource.MustParse": lambda s: s, "v1.ResourceName": lambda s: s, "v1.Protocol": lambda s: s,
    "v1helper.HugePageResourceName": lambda q: f"hugepages-{q}", "int64": int, "int32": int, "int": int,
    "strconv.Itoa": str,
}


def error_reasons(ref: str) -> dict:
    """Err* = newPredicateFailureError("Name") in error.go: GetReason() is the name."""
    src = open(os.path.join(ref, PKG, "error.go")).read()
    return dict(re.findall(r"(Err\w+)\s*=\s*newPredicateFailureError\(\"(\w+)\"\)", src))


# ------------------------------------------------------------------ reading the test file
def preprocess(src: str) -> str:
    src = re.sub(r"new\(([\w.]+)\)", r"&\1{}", src)
    return re.sub(r"makeResources\(([^()]*)\)\.Capacity", r"makeResourcesCapacity(\1)", src)


TABLES = [   # (test function, table variable, fixture key)
    ("TestPodFitsResources", "enoughPodsTests", "PodFitsResources/enough"),
    ("TestPodFitsResources", "notEnoughPodsTests", "PodFitsResources/notEnoughPods"),
    ("TestPodFitsResources", "storagePodsTests", "PodFitsResources/storage"),
    ("TestPodFitsHost", "tests", "PodFitsHost"),
    ("TestPodFitsHostPorts", "tests", "PodFitsHostPorts"),
    ("TestGetUsedPorts", "tests", "GetUsedPorts"),
    ("TestGCEDiskConflicts", "tests", "DiskConflicts/GCE"),
    ("TestAWSDiskConflicts", "tests", "DiskConflicts/AWS"),
    ("TestRBDDiskConflicts", "tests", "DiskConflicts/RBD"),
    ("TestISCSIDiskConflicts", "tests", "DiskConflicts/ISCSI"),
    ("TestPodFitsSelector", "tests", "PodFitsSelector"),
    ("TestNodeLabelPresence", "tests", "NodeLabelPresence"),
    ("TestServiceAffinity", "tests", "ServiceAffinity"),
    ("TestEBSVolumeCountConflicts", "tests", "EBSVolumeCount"),
    ("TestRunGeneralPredicates", "resourceTests", "GeneralPredicates"),
    ("TestInterPodAffinity", "tests", "InterPodAffinity"),
    ("TestInterPodAffinityWithMultipleNodes", "tests", "InterPodAffinityWithMultipleNodes"),
    ("TestPodToleratesTaints", "podTolerateTaintsTests", "PodToleratesTaints"),
    ("TestPodSchedulesOnNodeWithMemoryPressureCondition", "tests", "MemoryPressure"),
    ("TestPodSchedulesOnNodeWithDiskPressureCondition", "tests", "DiskPressure"),
    ("TestNodeConditionPredicate", "tests", "NodeCondition"),
    ("TestVolumeZonePredicate", "tests", "VolumeZone"),
    ("TestVolumeZonePredicateMultiZone", "tests", "VolumeZoneMultiZone"),
    ("TestVolumeZonePredicateWithVolumeBinding", "tests", "VolumeZoneWithBinding"),
    ("TestGetMaxVols", "tests", "GetMaxVols"),
]
# harness data the replay needs besides the table (ServiceAffinity's node list, EBS's PV infos)
LOCALS = {"TestServiceAffinity": ["node1", "node2", "node3", "node4", "node5"],
          "TestEBSVolumeCountConflicts": ["pvInfo", "pvcInfo"],
          "TestVolumeZonePredicate": ["pvInfo", "pvcInfo"], "TestVolumeZonePredicateMultiZone": ["pvInfo", "pvcInfo"],
          "TestVolumeZonePredicateWithVolumeBinding": ["pvInfo", "pvcInfo", "classInfo"]}


def main():
    src = preprocess(open(os.path.join(REF, SRC)).read())
    names = {**k8s_names(REF), **error_reasons(REF)}
    names.update({"resource.DecimalSI": "DecimalSI", "resource.BinarySI": "BinarySI",
                  "extendedResourceA": "example.com/aaa", "extendedResourceB": "example.com/bbb",
                  "hugePageResourceA": "hugepages-2Mi"})
    out = {"source": SRC}
    n = 0
    for fn, var, key in TABLES:
        ev = Evaluator(FUNCS, names, hook=k8s_hook)
        ev.map_types = frozenset({"v1.ResourceList"})
        start, end = func_body(src, fn)
        eval_locals(src, ev, start, end)
        cases, line = table(src, ev, var, start)
        entry = {"line": line, "cases": cases}
        for lv in LOCALS.get(fn, []):
            entry.setdefault("locals", {})[lv] = ev.names[lv]
        out[key] = entry
        n += len(cases)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: {n} cases in {len(TABLES)} tables")


if __name__ == "__main__":
    main()
