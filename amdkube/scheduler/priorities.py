"""Priority (scoring) functions; each returns 0..10 per node, combined by weight.

Reference: plugin/pkg/scheduler/algorithm/priorities/* — least_requested.go,
balanced_resource_allocation.go, most_requested.go, selector_spreading.go,
node_affinity.go, taint_toleration.go, node_prefer_avoid_pods.go (weight 10000),
interpod_affinity.go, image_locality.go; defaults in algorithmprovider/defaults/
defaults.go:217-260. New: GPUTopologyPriority (xGMI/NUMA subset quality + best fit, see
extended.topology_score) — the reference has no topology awareness.
"""
from __future__ import annotations

import json

from ..api import meta as m
from ..api.helpers import tolerations_tolerate_taint
from . import extended

MAX = 10.0


def _cpu_mem(pi):
    nz = getattr(pi, "_nz", None)
    if nz is None:
        from .cache import nonzero_requests
        nz = pi._nz = nonzero_requests(pi.pod)
    return nz


def least_requested(pi, nodes, ctx=None):
    cpu, mem = _cpu_mem(pi)
    out = []
    for ni in nodes:
        cc, mc = ni.allocatable.get("cpu", 0), ni.allocatable.get("memory", 0)
        s1 = ((cc - ni.nonzero[0] - cpu) * MAX / cc) if cc and ni.nonzero[0] + cpu <= cc else 0.0
        s2 = ((mc - ni.nonzero[1] - mem) * MAX / mc) if mc and ni.nonzero[1] + mem <= mc else 0.0
        out.append((s1 + s2) / 2)
    return out


def most_requested(pi, nodes, ctx=None):
    cpu, mem = _cpu_mem(pi)
    out = []
    for ni in nodes:
        cc, mc = ni.allocatable.get("cpu", 0), ni.allocatable.get("memory", 0)
        s1 = ((ni.nonzero[0] + cpu) * MAX / cc) if cc and ni.nonzero[0] + cpu <= cc else 0.0
        s2 = ((ni.nonzero[1] + mem) * MAX / mc) if mc and ni.nonzero[1] + mem <= mc else 0.0
        out.append((s1 + s2) / 2)
    return out


def balanced_allocation(pi, nodes, ctx=None):
    cpu, mem = _cpu_mem(pi)
    out = []
    for ni in nodes:
        cc, mc = ni.allocatable.get("cpu", 0), ni.allocatable.get("memory", 0)
        if not cc or not mc:
            out.append(0.0)
            continue
        f1, f2 = (ni.nonzero[0] + cpu) / cc, (ni.nonzero[1] + mem) / mc
        out.append(0.0 if f1 >= 1 or f2 >= 1 else MAX - abs(f1 - f2) * MAX)
    return out


def selector_spread(pi, nodes, ctx=None):
    if pi.owner is None:
        return [MAX] * len(nodes)
    uid = pi.owner.get("uid")
    counts = [ni.owners.get(uid, 0) for ni in nodes]
    mx = max(counts) if counts else 0
    return [MAX * (mx - c) / mx if mx else MAX for c in counts]


def node_affinity(pi, nodes, ctx=None):
    if not pi.preferred_terms:
        return [0.0] * len(nodes)
    raw = [sum(w for w, sel in pi.preferred_terms if sel.matches(ni.labels)) for ni in nodes]
    mx = max(raw) if raw else 0
    return [MAX * r / mx if mx else 0.0 for r in raw]


def taint_toleration(pi, nodes, ctx=None):
    tols = [t for t in pi.tolerations if t.get("effect") in (None, "", "PreferNoSchedule")]
    raw = [sum(1 for t in ni.taints if t.get("effect") == "PreferNoSchedule" and not tolerations_tolerate_taint(tols, t))
           if ni.taints else 0 for ni in nodes]
    mx = max(raw) if raw else 0
    return [MAX * (1 - r / mx) if mx else MAX for r in raw]


def node_prefer_avoid_pods(pi, nodes, ctx=None):
    out = []
    ref = pi.owner
    for ni in nodes:
        ann = m.annotations_of(ni.node or {}).get("scheduler.alpha.kubernetes.io/preferAvoidPods")
        score = MAX
        if ann and ref and ref.get("kind") in ("ReplicationController", "ReplicaSet"):
            try:
                for e in (json.loads(ann).get("preferAvoidPods") or []):
                    pc = (e.get("podSignature") or {}).get("podController") or {}
                    if pc.get("kind") == ref.get("kind") and pc.get("uid") == ref.get("uid"):
                        score = 0.0
            except ValueError:
                pass
        out.append(score)
    return out


def _symmetric_hard(pi, nodes, ctx) -> list[int]:
    """interpod_affinity.go: an existing pod's *required* affinity term that matches the incoming
    pod pulls it into that pod's topology domain with hardPodAffinitySymmetricWeight."""
    from .predicates import _term_selector, _term_namespaces
    out = [0] * len(nodes)
    for o in ctx.nodes:
        for p in o.pods.values():
            terms = ((((p.get("spec") or {}).get("affinity") or {}).get("podAffinity") or {})
                     .get("requiredDuringSchedulingIgnoredDuringExecution") or [])
            for term in terms:
                if m.namespace_of(pi.pod) not in _term_namespaces(term, p) or not _term_selector(term).matches(pi.labels):
                    continue
                key = term.get("topologyKey")
                val = o.labels.get(key)
                if val is None:
                    continue
                for i, ni in enumerate(nodes):
                    if ni.labels.get(key) == val:
                        out[i] += ctx.hard_weight
    return out


def inter_pod_affinity(pi, nodes, ctx=None):
    sym = ctx is not None and ctx.hard_weight and ctx.any_affinity
    if not (pi.pref_affinity or pi.pref_anti or sym):
        return [0.0] * len(nodes)
    from .predicates import _term_selector, _term_namespaces
    raw = []
    hard = _symmetric_hard(pi, nodes, ctx) if sym else [0] * len(nodes)
    for idx, ni in enumerate(nodes):
        s = hard[idx]
        for weighted, sign in ((pi.pref_affinity, 1), (pi.pref_anti, -1)):
            for wt in weighted:
                term = wt.get("podAffinityTerm") or {}
                key = term.get("topologyKey")
                val = ni.labels.get(key)
                sel, nss = _term_selector(term), _term_namespaces(term, pi.pod)
                for o in (ctx.nodes if ctx else [ni]):
                    if val is None or o.labels.get(key) != val:
                        continue
                    s += sign * int(wt.get("weight", 0)) * sum(
                        1 for p in o.pods.values() if m.namespace_of(p) in nss and sel.matches(m.labels_of(p)))
        raw.append(s)
    lo, hi = min(raw), max(raw)
    return [MAX * (r - lo) / (hi - lo) if hi > lo else 0.0 for r in raw]


def image_locality(pi, nodes, ctx=None):
    return [0.0] * len(nodes)


def gpu_topology(pi, nodes, ctx=None):
    return [extended.topology_score(pi, ni) for ni in nodes]


PRIORITIES = {
    "LeastRequestedPriority": least_requested,
    "MostRequestedPriority": most_requested,
    "BalancedResourceAllocation": balanced_allocation,
    "SelectorSpreadPriority": selector_spread,
    "NodeAffinityPriority": node_affinity,
    "TaintTolerationPriority": taint_toleration,
    "NodePreferAvoidPodsPriority": node_prefer_avoid_pods,
    "InterPodAffinityPriority": inter_pod_affinity,
    "ImageLocalityPriority": image_locality,
    "GPUTopologyPriority": gpu_topology,
}

DEFAULT_PRIORITIES = {"SelectorSpreadPriority": 1, "InterPodAffinityPriority": 1, "LeastRequestedPriority": 1,
                      "BalancedResourceAllocation": 1, "NodePreferAvoidPodsPriority": 10000, "NodeAffinityPriority": 1,
                      "TaintTolerationPriority": 1, "GPUTopologyPriority": 2}
