"""Priority (scoring) functions; each returns 0..10 per node, combined by weight.

Reference: plugin/pkg/scheduler/algorithm/priorities/* — least_requested.go,
balanced_resource_allocation.go, most_requested.go, selector_spreading.go,
node_affinity.go, taint_toleration.go, node_prefer_avoid_pods.go (weight 10000),
interpod_affinity.go, image_locality.go, resource_limits.go; EqualPriority and
ServiceSpreadingPriority (algorithmprovider/defaults/defaults.go:91-115); defaults at
defaults.go:217-260. Scores are the reference's integers 0..10, truncated where its map/reduce
truncates, and weighted totals are integers. New: GPUTopologyPriority (xGMI/NUMA subset quality + best fit, see
extended.topology_score) — the reference has no topology awareness.
"""
from __future__ import annotations

import json

from ..api import meta as m
from ..api.helpers import tolerations_tolerate_taint
from . import extended

MAX = 10            # schedulerapi.MaxPriority: every priority scores an integer 0..10


def _cpu_mem(pi):
    nz = getattr(pi, "_nz", None)
    if nz is None:
        from .cache import nonzero_requests
        nz = pi._nz = nonzero_requests(pi.pod)
    return nz


def unused_score(requested: int, capacity: int) -> int:
    """least_requested.go calculateUnusedScore: integer ((capacity - requested) * 10) / capacity."""
    if capacity == 0 or requested > capacity:
        return 0
    return (capacity - requested) * MAX // capacity


def used_score(requested: int, capacity: int) -> int:
    """most_requested.go calculateUsedScore: integer (requested * 10) / capacity."""
    if capacity == 0 or requested > capacity:
        return 0
    return requested * MAX // capacity


def least_requested(pi, nodes, ctx=None):
    """LeastRequestedPriority: the mean of the CPU and memory unused scores, integer-divided."""
    cpu, mem = _cpu_mem(pi)
    return [(unused_score(ni.nonzero[0] + cpu, ni.allocatable.get("cpu", 0)) +
             unused_score(ni.nonzero[1] + mem, ni.allocatable.get("memory", 0))) // 2 for ni in nodes]


def most_requested(pi, nodes, ctx=None):
    cpu, mem = _cpu_mem(pi)
    return [(used_score(ni.nonzero[0] + cpu, ni.allocatable.get("cpu", 0)) +
             used_score(ni.nonzero[1] + mem, ni.allocatable.get("memory", 0))) // 2 for ni in nodes]


def _fraction(requested: int, capacity: int) -> float:
    return 1.0 if capacity == 0 else requested / capacity


def balanced_allocation(pi, nodes, ctx=None):
    """balanced_resource_allocation.go: int((1 - |cpuFraction - memoryFraction|) * 10), 0 when
    either fraction reaches 1."""
    cpu, mem = _cpu_mem(pi)
    out = []
    for ni in nodes:
        f1 = _fraction(ni.nonzero[0] + cpu, ni.allocatable.get("cpu", 0))
        f2 = _fraction(ni.nonzero[1] + mem, ni.allocatable.get("memory", 0))
        out.append(0 if f1 >= 1 or f2 >= 1 else int((1 - abs(f1 - f2)) * float(MAX)))
    return out


def normalize_reduce(raw, reverse: bool) -> list[int]:
    """reduce.go NormalizeReduce(MaxPriority, reverse): integer MAX * score / maxCount."""
    mx = max([0, *raw])
    if mx == 0:
        return [MAX if reverse else 0 for _ in raw]
    return [(MAX - MAX * r // mx) if reverse else MAX * r // mx for r in raw]


ZONE_WEIGHTING = 2.0 / 3.0
ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"


def zone_key(labels: dict) -> str:
    """pkg/util/node/node.go GetZoneKey: region and zone joined; "" when the node has neither."""
    region, zone = labels.get(REGION_LABEL, ""), labels.get(ZONE_LABEL, "")
    if not region and not zone:
        return ""
    return region + ":\x00:" + zone


def pod_selectors(pi, ctx, services_only=False) -> list:
    """Selectors of the Services/RCs/RSs/StatefulSets that pick the pod, once per attempt."""
    attr = "_svc_sel" if services_only else "_spread_sel"
    sel = getattr(pi, attr, None)
    if sel is None:
        listers = getattr(ctx, "listers", None) if ctx is not None else None
        sel = listers.selectors(pi.pod, services_only) if listers is not None else []
        setattr(pi, attr, sel)
    return sel


def _spread_counts(pi, nodes, sels) -> list[int]:
    """CalculateSpreadPriorityMap: per node, the live pods of the pod's namespace that any of the
    selectors matches. Nodes keep pods grouped by (namespace, labels), so each distinct label set
    is matched once per call."""
    ns = (pi.pod.get("metadata") or {}).get("namespace") or ""
    memo: dict = {}
    out = []
    for ni in nodes:
        c = 0
        for (gns, lk), n in ni.groups.items():
            if gns != ns:
                continue
            hit = memo.get(lk)
            if hit is None:
                ls = dict(lk)
                hit = memo[lk] = any(s.matches(ls) for s in sels)
            if hit:
                c += n
        out.append(c)
    return out


def _spread_reduce(counts, nodes) -> list[int]:
    """CalculateSpreadPriorityReduce (selector_spreading.go:119-161): fewer matching pods on the
    node scores higher; with zone labels, 2/3 of the score comes from the node's zone total."""
    by_zone: dict[str, int] = {}
    zones = []
    for c, ni in zip(counts, nodes):
        z = zone_key(ni.labels)
        zones.append(z)
        if z:
            by_zone[z] = by_zone.get(z, 0) + c
    max_node = max(counts) if counts else 0
    max_zone = max(by_zone.values()) if by_zone else 0
    out = []
    for c, z in zip(counts, zones):
        f = float(MAX) * ((max_node - c) / max_node) if max_node > 0 else float(MAX)
        if by_zone and z:
            zs = float(MAX) * ((max_zone - by_zone[z]) / max_zone) if max_zone > 0 else float(MAX)
            f = f * (1.0 - ZONE_WEIGHTING) + ZONE_WEIGHTING * zs
        out.append(int(f))
    return out


def selector_spread(pi, nodes, ctx=None):
    """SelectorSpreadPriority: spread the pods selected by the same Service, RC, RS or StatefulSet
    over nodes and zones (selector_spreading.go:34-161)."""
    sels = pod_selectors(pi, ctx)
    if not sels:
        return [MAX] * len(nodes)
    return _spread_reduce(_spread_counts(pi, nodes, sels), nodes)


def service_spreading(pi, nodes, ctx=None):
    """ServiceSpreadingPriority: SelectorSpread over Services only (defaults.go:91-102)."""
    sels = pod_selectors(pi, ctx, services_only=True)
    if not sels:
        return [MAX] * len(nodes)
    return _spread_reduce(_spread_counts(pi, nodes, sels), nodes)


def equal(pi, nodes, ctx=None):
    """EqualPriority (core/generic_scheduler.go EqualPriorityMap): every node scores 1."""
    return [1] * len(nodes)


def node_affinity(pi, nodes, ctx=None):
    """node_affinity.go: the summed weights of the matching preferred terms (weight 0 skipped),
    normalised by NormalizeReduce."""
    if not pi.preferred_terms:
        return [0] * len(nodes)
    raw = [sum(w for w, sel in pi.preferred_terms if w and sel.matches(ni.labels)) for ni in nodes]
    return normalize_reduce(raw, reverse=False)


def taint_toleration(pi, nodes, ctx=None):
    """taint_toleration.go: intolerable PreferNoSchedule taints counted, NormalizeReduce reversed."""
    tols = [t for t in pi.tolerations if t.get("effect") in (None, "", "PreferNoSchedule")]
    raw = [sum(1 for t in ni.taints if t.get("effect") == "PreferNoSchedule" and not tolerations_tolerate_taint(tols, t))
           if ni.taints else 0 for ni in nodes]
    return normalize_reduce(raw, reverse=True)


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
                        score = 0
            except ValueError:
                pass
        out.append(score)
    return out


def _pod_affinity_terms(pod):
    aff = (pod.get("spec") or {}).get("affinity") or {}
    return aff.get("podAffinity") or {}, aff.get("podAntiAffinity") or {}


def inter_pod_affinity(pi, nodes, ctx=None):
    """InterPodAffinityPriority (interpod_affinity.go CalculateInterPodAffinityPriority :114-220):
    per candidate node, the weight of every (term, pod) match in its topology domain —
    the incoming pod's preferred affinity (+) and anti-affinity (-) terms against existing pods,
    and, by symmetry, existing pods' required affinity terms (hardPodAffinitySymmetricWeight),
    preferred affinity (+) and preferred anti-affinity (-) against the incoming pod. Counts are
    normalised between min(0, counts) and max(0, counts) and truncated: int(10 * (c - min) /
    (max - min))."""
    from .predicates import _term_namespaces, _term_selector
    from ..api.labels import SelectorError
    n = len(nodes)
    counts = [0.0] * n
    all_nodes = ctx.nodes if ctx is not None and ctx.nodes else nodes
    hard_w = ctx.hard_weight if ctx is not None else 0
    # existing pods' terms matter only if some pod carries them (the cache counts such pods)
    sym = ctx is None or (ctx.any_affinity and hard_w > 0) or ctx.any_pref_affinity
    if not (pi.pref_affinity or pi.pref_anti or sym):
        return [0] * n

    def add_domain(key, value, weight):
        if not key or value is None:
            return
        for i, ni in enumerate(nodes):
            if ni.labels.get(key) == value:
                counts[i] += weight

    # the incoming pod's preferred terms: matching pods counted per topology domain in one pass
    for weighted, sign in ((pi.pref_affinity, 1), (pi.pref_anti, -1)):
        for wt in weighted:
            term = wt.get("podAffinityTerm") or {}
            key = term.get("topologyKey")
            if not key:
                continue
            try:
                sel = _term_selector(term)
            except SelectorError:
                continue
            nss = _term_namespaces(term, pi.pod)
            w = float(int(wt.get("weight", 0)) * sign)
            dom: dict = {}
            for o in all_nodes:
                val = o.labels.get(key)
                if val is None:
                    continue
                c = sum(1 for p in o.pods.values() if m.namespace_of(p) in nss and sel.matches(m.labels_of(p)))
                if c:
                    dom[val] = dom.get(val, 0.0) + w * c
            if dom:
                for i, ni in enumerate(nodes):
                    v = ni.labels.get(key)
                    if v is not None and v in dom:
                        counts[i] += dom[v]

    # symmetry: the terms existing pods carry, checked against the incoming pod
    if sym:
        ns, labels = m.namespace_of(pi.pod), pi.labels

        def matches(term, definer) -> bool:
            if ns not in _term_namespaces(term, definer):
                return False
            try:
                return _term_selector(term).matches(labels)
            except SelectorError:
                return False
        for o in all_nodes:
            for p in o.pods.values():
                pa, paa = _pod_affinity_terms(p)
                if not pa and not paa:
                    continue
                if pa:
                    if hard_w > 0:
                        for term in pa.get("requiredDuringSchedulingIgnoredDuringExecution") or []:
                            if matches(term, p):
                                key = term.get("topologyKey")
                                add_domain(key, o.labels.get(key) if key else None, float(hard_w))
                    for wt in pa.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
                        term = wt.get("podAffinityTerm") or {}
                        if matches(term, p):
                            key = term.get("topologyKey")
                            add_domain(key, o.labels.get(key) if key else None, float(int(wt.get("weight", 0))))
                if paa:
                    for wt in paa.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
                        term = wt.get("podAffinityTerm") or {}
                        if matches(term, p):
                            key = term.get("topologyKey")
                            add_domain(key, o.labels.get(key) if key else None, -float(int(wt.get("weight", 0))))
    hi, lo = max([0.0, *counts]), min([0.0, *counts])
    if hi - lo <= 0:
        return [0] * n
    return [int(float(MAX) * ((c - lo) / (hi - lo))) for c in counts]


MB = 1024 * 1024
MIN_IMG_SIZE, MAX_IMG_SIZE = 23 * MB, 1000 * MB


def image_score(total: int) -> int:
    """image_locality.go calculateScoreFromSize: 0 below 23 MiB, 10 from 1000 MiB, linear
    (integer) buckets between."""
    if total == 0 or total < MIN_IMG_SIZE:
        return 0
    if total >= MAX_IMG_SIZE:
        return MAX
    return MAX * (total - MIN_IMG_SIZE) // (MAX_IMG_SIZE - MIN_IMG_SIZE) + 1


def image_locality(pi, nodes, ctx=None):
    """ImageLocalityPriority (image_locality.go:32-62): the summed size of the pod's container
    images already present on the node (node.status.images, reported by the kubelet)."""
    images = [c.get("image") for c in pi.spec.get("containers") or []]
    out = []
    for ni in nodes:
        sizes = {}
        for img in ((ni.node or {}).get("status") or {}).get("images") or []:
            for name in img.get("names") or []:
                sizes[name] = int(img.get("sizeBytes") or 0)
        out.append(image_score(sum(sizes.get(i, 0) for i in images)))
    return out


def _pod_limits(pod) -> tuple[int, int]:
    """resource_limits.go getResourceLimits: summed container limits, raised to the largest init
    container limit (milli-CPU, memory bytes)."""
    from ..api.quantity import Quantity
    spec = pod.get("spec") or {}
    cpu = mem = 0
    for c in spec.get("containers") or []:
        lim = (c.get("resources") or {}).get("limits") or {}
        if "cpu" in lim:
            cpu += Quantity(lim["cpu"]).milli_value()
        if "memory" in lim:
            mem += Quantity(lim["memory"]).value()
    for c in spec.get("initContainers") or []:
        lim = (c.get("resources") or {}).get("limits") or {}
        if "cpu" in lim:
            cpu = max(cpu, Quantity(lim["cpu"]).milli_value())
        if "memory" in lim:
            mem = max(mem, Quantity(lim["memory"]).value())
    return cpu, mem


def resource_limits(pi, nodes, ctx=None):
    """ResourceLimitsPriority (resource_limits.go:37-72, gate ResourceLimitsPriorityFunction):
    1 for a node whose allocatable CPU or memory covers the pod's limit, else 0."""
    lim = getattr(pi, "_limits", None)
    if lim is None:
        lim = pi._limits = _pod_limits(pi.pod)
    cpu, mem = lim
    out = []
    for ni in nodes:
        ac, am = ni.allocatable.get("cpu", 0), ni.allocatable.get("memory", 0)
        ok = (cpu and ac and cpu <= ac) or (mem and am and mem <= am)
        out.append(1 if ok else 0)
    return out


def gpu_topology(pi, nodes, ctx=None):
    """GPUTopologyPriority: subset quality plus best fit, an integer 0..10 (extended.topology_score)."""
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
    "ServiceSpreadingPriority": service_spreading,
    "EqualPriority": equal,
    "ResourceLimitsPriority": resource_limits,      # registered only with its feature gate
    "GPUTopologyPriority": gpu_topology,
}

# registered in the reference only when the named gate is on (defaults.go:113-115)
GATED_PRIORITIES = {"ResourceLimitsPriority": "ResourceLimitsPriorityFunction"}

DEFAULT_PRIORITIES = {"SelectorSpreadPriority": 1, "InterPodAffinityPriority": 1, "LeastRequestedPriority": 1,
                      "BalancedResourceAllocation": 1, "NodePreferAvoidPodsPriority": 10000, "NodeAffinityPriority": 1,
                      "TaintTolerationPriority": 1, "GPUTopologyPriority": 2}
