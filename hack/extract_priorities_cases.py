"""Extract the scheduler priority tables from the reference into a JSON fixture.

Sources (plugin/pkg/scheduler/algorithm/priorities/): least_requested_test.go TestLeastRequested,
balanced_resource_allocation_test.go TestBalancedResourceAllocation, most_requested_test.go
TestMostRequested, node_affinity_test.go TestNodeAffinityPriority, taint_toleration_test.go
TestTaintAndToleration, interpod_affinity_test.go TestInterPodAffinityPriority and
TestHardPodAffinitySymmetricWeight, node_prefer_avoid_pods_test.go TestNodePreferAvoidPriority.
Each table is read by hack/goexpr.py; the files' helpers (makeNode in test_util.go,
nodeWithTaints, podWithTolerations) are re-expressed below over JSON objects, and the one
struct-copy idiom (`cpuOnly2 := cpuOnly; cpuOnly2.NodeName = "machine2"`) is rewritten to a call.

  python hack/extract_priorities_cases.py [REFERENCE_ROOT]  ->  tests/fixtures/priorities_cases.json
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, eval_locals, func_body, k8s_hook, k8s_names, table  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
PKG = "plugin/pkg/scheduler/algorithm/priorities"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "priorities_cases.json")


def make_node(name, milli_cpu, memory):
    res = {"cpu": f"{milli_cpu}m", "memory": str(memory)}
    return {"metadata": {"name": name}, "status": {"capacity": dict(res), "allocatable": dict(res)}}


def node_with_taints(name, taints):
    return {"metadata": {"name": name}, "spec": {"taints": taints}}


def pod_with_tolerations(tols):
    return {"spec": {"tolerations": tols}}


def with_node_name(spec, node):
    return {**spec, "nodeName": node}


FUNCS = {
    "makeNode": make_node, "nodeWithTaints": node_with_taints, "podWithTolerations": pod_with_tolerations,
    "withNodeName": with_node_name, "resource.MustParse": lambda s: s, "int32": int, "int64": int, "int": int,
}

TABLES = [   # (file, test function, table variable, fixture key)
    ("least_requested_test.go", "TestLeastRequested", "tests", "LeastRequested"),
    ("balanced_resource_allocation_test.go", "TestBalancedResourceAllocation", "tests", "BalancedResourceAllocation"),
    ("most_requested_test.go", "TestMostRequested", "tests", "MostRequested"),
    ("node_affinity_test.go", "TestNodeAffinityPriority", "tests", "NodeAffinity"),
    ("taint_toleration_test.go", "TestTaintAndToleration", "tests", "TaintToleration"),
    ("interpod_affinity_test.go", "TestInterPodAffinityPriority", "tests", "InterPodAffinity"),
    ("interpod_affinity_test.go", "TestHardPodAffinitySymmetricWeight", "tests", "HardPodAffinitySymmetricWeight"),
    ("node_prefer_avoid_pods_test.go", "TestNodePreferAvoidPriority", "tests", "NodePreferAvoidPods"),
]


def preprocess(src: str) -> str:
    src = re.sub(r"\t(\w+) := (\w+)\n\t\1\.NodeName = (\"\w+\")", r"\t\1 := withNodeName(\2, \3)", src)
    return re.sub(r"new\(([\w.]+)\)", r"&\1{}", src)


def main():
    names = dict(k8s_names(REF))
    names.update({"schedulerapi.MaxPriority": 10, "v1.DefaultHardPodAffinitySymmetricWeight": 1,
                  "v1.PreferAvoidPodsAnnotationKey": "scheduler.alpha.kubernetes.io/preferAvoidPods"})
    out = {"source": PKG}
    total = 0
    for fname, fn, var, key in TABLES:
        src = preprocess(open(os.path.join(REF, PKG, fname)).read())
        ev = Evaluator(FUNCS, names, hook=k8s_hook)
        ev.map_types = frozenset({"v1.ResourceList"})
        start, end = func_body(src, fn)
        eval_locals(src, ev, start, end)
        cases, line = table(src, ev, var, start)
        for c in cases:
            c["expectedList"] = [[h["host"], h["score"]] for h in c["expectedList"]]
        out[key] = {"file": f"{PKG}/{fname}", "line": line, "cases": cases}
        total += len(cases)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: {total} cases in {len(TABLES)} tables")


if __name__ == "__main__":
    main()
