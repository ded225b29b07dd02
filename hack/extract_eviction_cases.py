"""Extract the kubelet eviction helper tables from the reference into a JSON fixture.

Source: pkg/kubelet/eviction/helpers_test.go — the data-only tables TestParseThresholdConfig,
TestThresholdsMet, TestThresholdsUpdatedStats, TestPercentageThresholdsMet, TestNodeConditions,
TestHasNodeConditions, TestGetStarvedResources, read by hack/goexpr.py. Thresholds become
{"signal", "operator", "value": {"quantity" | "percentage"}, "minReclaim", "gracePeriod"} (bytes,
float32 fractions, seconds); signalObservations {signal: {"available", "capacity", "time"}} with
times as epoch seconds. The tests whose cases are built from times relative to `now` or whose
maps are keyed by threshold values are transcribed in tests/test_eviction.py instead.

  python hack/extract_eviction_cases.py [REFERENCE_ROOT]  ->  tests/fixtures/eviction_cases.json
"""
from __future__ import annotations

import calendar
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, eval_locals, func_body, go_string_constants, k8s_hook, k8s_names, table  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
PKG = "pkg/kubelet/eviction"
SRC = PKG + "/helpers_test.go"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "eviction_cases.json")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def quantity(s):
    from amdkube.api.quantity import Quantity
    return Quantity(s).value()


def hook(type_name, v):
    out = k8s_hook(type_name, v)
    if "percentage" in out:                       # ThresholdValue.Percentage is a float32
        out["percentage"] = float(np.float32(out["percentage"]))
    return out


FUNCS = {"quantityMustParse": quantity, "resource.MustParse": quantity,
         "resource.NewQuantity": lambda v, fmt=None: int(v),
         "metav1.Date": lambda y, mo, d, h, mi, s, ns, loc=None: calendar.timegm((y, mo, d, h, mi, s)) + ns / 1e9}
ORDER_TESTS = ["TestOrderedByExceedsRequestMemory", "TestOrderedByExceedsRequestDisk", "TestOrderedByPriority",
               "TestOrderedByPriorityDisabled", "TestOrderedbyDisk", "TestOrderedbyDiskDisableLocalStorage",
               "TestOrderedbyInodes", "TestOrderedByPriorityDisk", "TestOrderedByPriorityInodes", "TestOrderedByMemory",
               "TestOrderedByPriorityMemory"]


def _container(name, requests, limits):
    res = {}
    if requests:
        res["requests"] = requests
    if limits:
        res["limits"] = limits
    return {"name": name, "resources": res}


def _pod(name, priority, containers, volumes):
    """newPod: the name is the UID."""
    return {"metadata": {"name": name, "uid": name}, "spec": {"containers": containers or [], "volumes": volumes or [],
                                                             "priority": priority}}


def _resource_list(cpu, mem, disk):
    out = {}
    for k, v in (("cpu", cpu), ("memory", mem), ("ephemeral-storage", disk)):
        if v:
            out[k] = v
    return out


def _local_volume_names(pod):
    return [v["name"] for v in pod["spec"]["volumes"]
            if "hostPath" in v or ("emptyDir" in v and (v["emptyDir"] or {}).get("medium") != "Memory")
            or "configMap" in v or "gitRepo" in v]


def _fs_stats(pod, root, logs, per_volume, key):
    return {"podRef": {"name": pod["metadata"]["name"], "uid": pod["metadata"]["uid"]},
            "containers": [{"rootfs": {key: root}, "logs": {key: logs}} for _ in pod["spec"]["containers"]],
            "volume": [{"name": n, key: per_volume} for n in _local_volume_names(pod)]}


def _memory_stats(pod, working_set):
    return {"podRef": {"name": pod["metadata"]["name"], "uid": pod["metadata"]["uid"]},
            "containers": [{"memory": {"workingSetBytes": working_set}} for _ in pod["spec"]["containers"]]}


ORDER_FUNCS = {
    "newPod": _pod, "newContainer": _container, "newResourceList": _resource_list,
    "newVolume": lambda name, source: {"name": name, **source},
    "newPodMemoryStats": _memory_stats,
    "newPodDiskStats": lambda pod, r, lg, v: _fs_stats(pod, r, lg, v, "usedBytes"),
    "newPodInodeStats": lambda pod, r, lg, v: _fs_stats(pod, r, lg, v, "inodesUsed"),
    # comparator descriptors for orderedBy(...)
    "exceedMemoryRequests": lambda stats: ["exceedMemoryRequests"], "memory": lambda stats: ["memory"],
    "exceedDiskRequests": lambda stats, measure, res: ["exceedDiskRequests", measure, res],
    "disk": lambda stats, measure, res: ["disk", measure, res],
}
ORDER_NAMES = {"lowPriority": -1, "defaultPriority": 0, "highPriority": 1, "statsFn": None, "priority": ["priority"],
               "fsStatsRoot": "root", "fsStatsLogs": "logs", "fsStatsLocalVolumeSource": "localVolumeSource",
               "resourceDisk": "disk", "resourceInodes": "inodes"}


def order_test(src, fn, base_names):
    """One TestOrdered* function: its pods (input order), the stats, the comparator chain, the
    feature gates it sets and the expected order (by pod name)."""
    import re
    ev = Evaluator({**FUNCS, **ORDER_FUNCS}, {**base_names, **ORDER_NAMES}, hook=hook)
    ev.map_types = frozenset({"v1.ResourceList"})
    start, end = func_body(src, fn)
    eval_locals(src, ev, start, end)
    body = src[start:end]
    gates = {g: v == "true" for v, g in re.findall(r'Sprintf\("%s=(true|false)", features\.(\w+)\)', body)}
    cmps = re.search(r"orderedBy\((.*)\)\.Sort\(pods\)", body).group(1)
    chain = ev.eval("[]x{" + cmps + "}")
    stats = ev.names["stats"] if "stats" in ev.names else []
    return {"line": src.count("\n", 0, start) + 1, "gates": gates, "chain": chain,
            "pods": ev.names["pods"], "stats": [v for _k, v in stats],
            "expected": [p["metadata"]["name"] for p in ev.names["expected"]]}


TABLES = [("TestParseThresholdConfig", "testCases"), ("TestThresholdsMet", "testCases"),
          ("TestThresholdsUpdatedStats", "testCases"), ("TestPercentageThresholdsMet", "testCases"),
          ("TestNodeConditions", "testCases"), ("TestHasNodeConditions", "testCases"),
          ("TestGetStarvedResources", "testCases")]


def main():
    src = open(os.path.join(REF, SRC)).read()
    names = {**k8s_names(REF), **go_string_constants(os.path.join(REF, PKG, "api/types.go"), "evictionapi.")}
    names.update({"cm.NodeAllocatableEnforcementKey": "pods", "locationUTC": "UTC", "gracePeriod": 30.0,
                  "resourceImageFs": "imagefs", "resourceNodeFs": "nodefs", "resource.BinarySI": "BinarySI",
                  "resource.DecimalSI": "DecimalSI"})
    out = {"source": SRC}
    n = 0
    for fn, var in TABLES:
        ev = Evaluator(FUNCS, dict(names), hook=hook)
        ev.map_types = frozenset({"signalObservations"})
        start, end = func_body(src, fn)
        eval_locals(src, ev, start, end)
        cases, line = table(src, ev, var, start)
        out[fn] = {"line": line, "cases": sorted(cases, key=lambda c: c["name"])}
        n += len(cases)
    out["ordering"] = {fn: order_test(src, fn, names) for fn in ORDER_TESTS}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: {n} cases in {len(TABLES)} tables")


if __name__ == "__main__":
    main()
