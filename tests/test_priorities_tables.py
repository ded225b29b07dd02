"""The default priorities held to their reference tables, extracted from
plugin/pkg/scheduler/algorithm/priorities/*_test.go by hack/extract_priorities_cases.py into
tests/fixtures/priorities_cases.json and replayed here:

  least_requested_test.go:30 TestLeastRequested, balanced_resource_allocation_test.go:30
  TestBalancedResourceAllocation, most_requested_test.go:30 TestMostRequested,
  node_affinity_test.go:29 TestNodeAffinityPriority (map + NormalizeReduce),
  taint_toleration_test.go:52 TestTaintAndToleration (map + reversed NormalizeReduce),
  interpod_affinity_test.go:42 TestInterPodAffinityPriority (hardPodAffinityWeight 1) and :529
  TestHardPodAffinitySymmetricWeight, node_prefer_avoid_pods_test.go:30 TestNodePreferAvoidPriority.

Each case builds the NodeInfos the reference's CreateNodeNameToInfoMap builds (pods placed by
spec.nodeName) and compares the exact integer HostPriority list.
"""
from __future__ import annotations

import json
import os

import pytest

from amdkube.scheduler import priorities as P
from amdkube.scheduler.cache import NodeInfo
from amdkube.scheduler.generic import Context
from amdkube.scheduler.predicates import PodInfo

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "priorities_cases.json")))


def node_infos(nodes, pods):
    out = {}
    for n in nodes:
        ni = NodeInfo(n["metadata"]["name"])
        ni.set_node(n)
        out[ni.name] = ni
    for i, p in enumerate(pods or []):
        p = {**p, "metadata": {**(p.get("metadata") or {}), "name": f"p{i}"}}
        p.setdefault("spec", {})
        ni = out.get(p["spec"].get("nodeName"))
        if ni is not None:
            ni.add_pod(f"{p['metadata'].get('namespace', '')}/p{i}", p)
    return [out[n["metadata"]["name"]] for n in nodes]


def _pod(p):
    p = json.loads(json.dumps(p))
    p.setdefault("metadata", {})
    p.setdefault("spec", {})
    return PodInfo(p)


def _run(fn, case, hard_weight=1):
    nis = node_infos(case["nodes"], case.get("pods"))
    ctx = Context(nis, False, any_affinity=True, hard_weight=hard_weight, any_pref_affinity=True)
    got = fn(_pod(case["pod"]), nis, ctx)
    assert all(type(s) is int for s in got), got
    return [[ni.name, s] for ni, s in zip(nis, got)]


TABLES = [("LeastRequested", P.least_requested), ("BalancedResourceAllocation", P.balanced_allocation),
          ("MostRequested", P.most_requested), ("NodeAffinity", P.node_affinity),
          ("TaintToleration", P.taint_toleration), ("InterPodAffinity", P.inter_pod_affinity),
          ("NodePreferAvoidPods", P.node_prefer_avoid_pods)]
CASES = [(key, fn, i) for key, fn in TABLES for i in range(len(FIX[key]["cases"]))]


@pytest.mark.parametrize("key,fn,i", CASES, ids=[f"{k}-{i}" for k, _, i in CASES])
def test_priority_table(key, fn, i):
    case = FIX[key]["cases"][i]
    assert _run(fn, case) == case["expectedList"], case["test"]


@pytest.mark.parametrize("i", range(len(FIX["HardPodAffinitySymmetricWeight"]["cases"])))
def test_hard_pod_affinity_symmetric_weight(i):
    case = FIX["HardPodAffinitySymmetricWeight"]["cases"][i]
    assert _run(P.inter_pod_affinity, case, case["hardPodAffinityWeight"]) == case["expectedList"], case["test"]


def test_fixture_covers_every_table():
    assert sum(len(FIX[k]["cases"]) for k in FIX if k != "source") == 50
