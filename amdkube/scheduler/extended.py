"""Device-granular extended-resource allocation (the fork's scheduler core).

Reference: plugin/pkg/scheduler/core/extended_resources.go — GetExtendedResources (:42-81)
runs after the predicates for every surviving node, hasExtendedResources (:83-111) allocates
each pod ExtendedResource from a copy of the node's available devices, allocateResources
(:113-150) takes the first N devices whose Attributes match the selector (isDeviceAMatch,
:152-167) in Go-map (random) order; failures become "Insufficient <res>".

amdkube keeps the contract (output: ExtendedResourceBinding per node, i.e. {pres name:
{"resources": [ids]}}) and changes the choice: among the matching healthy free devices the
subset is chosen by the native xGMI/NUMA topology allocator (amdkube.ops.topology) when the
node publishes a topology, otherwise deterministically by device ID. Feasibility is a count
check, so the (more expensive) subset choice runs only for the selected host.
"""
from __future__ import annotations

from ..ops import topology as topo


def matching_free(pi, ni, rname, selector, exclude=()) -> list[str]:
    avail = ni.available_devices(rname)
    if not avail:
        return []
    if selector.empty():
        return [d for d in avail if d not in exclude]
    return [d for d, dev in avail.items() if d not in exclude and selector.matches(dev.get("attributes") or {})]


def _shared_selectors(pi) -> bool:
    """True when two requests draw on one resource name and one of them has a selector: the
    per-request count check can then pass although no disjoint assignment exists."""
    seen: dict[str, bool] = {}
    for _, rname, _n, sel in pi.ext:
        if rname in seen and (not sel.empty() or seen[rname]):
            return True
        seen[rname] = seen.get(rname, False) or not sel.empty()
    return False


def _match(pi, ni, exclude=()) -> dict | None:
    """Exact feasibility: a disjoint assignment of devices to every request (each request of
    n devices is n slots; bipartite matching by augmenting paths — tiny graphs: ≤ 8 devices
    per resource on an MI355X node, 64 with CPX partitions). {pres name: [ids]} or None."""
    slots, cands = [], []
    for pname, rname, n, sel in pi.ext:
        c = matching_free(pi, ni, rname, sel, exclude)
        for _ in range(n):
            slots.append(pname)
            cands.append(c)
    owner: dict[str, int] = {}

    def augment(i, seen):
        for d in cands[i]:
            if d in seen:
                continue
            seen.add(d)
            if d not in owner or augment(owner[d], seen):
                owner[d] = i
                return True
        return False
    for i in range(len(slots)):
        if not augment(i, set()):
            return None
    out: dict[str, list[str]] = {}
    for d, i in sorted(owner.items()):
        out.setdefault(slots[i], []).append(d)
    return out


def fits(pi, ni) -> tuple[bool, list[str]]:
    if pi.ext_error:
        return False, [pi.ext_error]
    if not pi.ext:
        return True, []
    need: dict[str, int] = {}
    for _, rname, n, sel in pi.ext:
        cand = matching_free(pi, ni, rname, sel)
        need[rname] = need.get(rname, 0) + n
        if len(cand) < n or len(ni.available_devices(rname)) < need[rname]:
            return False, [f"Insufficient {rname}"]
    if _shared_selectors(pi) and _match(pi, ni) is None:
        # overlapping selectors on one resource name: the counts fit, no disjoint choice does
        return False, [f"Insufficient {pi.ext[0][1]}"]
    return True, []


def allocate(pi, ni, use_topology: bool = True) -> dict | None:
    """ExtendedResourceBinding for this node, or None if it does not fit."""
    if pi.ext_error:
        return None
    binding = {}
    taken: set[str] = set()
    t = ni.topology() if use_topology else None
    # most constrained request first, so a narrow selector is not starved by a wide one
    order = sorted(pi.ext, key=lambda e: len(matching_free(pi, ni, e[1], e[3]))) if _shared_selectors(pi) else pi.ext
    for pname, rname, n, sel in order:
        cand = matching_free(pi, ni, rname, sel, taken)
        if len(cand) < n:
            m = _match(pi, ni)       # the greedy order failed: take any disjoint assignment
            return {k: {"resources": v} for k, v in m.items()} if m is not None else None
        chosen = None
        if t is not None:
            ids, index, numa, link, parent = t
            if all(d in index for d in cand):
                free_all = [index[d] for d in ni.available_devices(rname) if d in index and d not in taken]
                sel_idx, cost = topo.select([index[d] for d in cand], n, link, numa, free_all, parent)
                if len(sel_idx) == n:
                    chosen = [ids[i] for i in sel_idx]
        if chosen is None:
            chosen = sorted(cand)[:n]
        taken.update(chosen)
        binding[pname] = {"resources": chosen}
    return binding


def topology_score(pi, ni) -> int:
    """0..10, an integer like every priority: how well the pod's GPUs fit this node
    (GPUTopologyPriority). Half comes from the placement quality of the chosen subset (xGMI links,
    NUMA; 0..5), half from how full the node's devices are once the pod is placed (best fit,
    0..5), so a GPU pod goes to the node it fills most and keeps empty nodes whole for large pods.
    CPU-only pods score GPU-less nodes 10 and GPU nodes 0."""
    if not pi.ext:
        return 10 if not ni.devices else 0
    names = {r for _, r, _, _ in pi.ext}
    total = sum(len(ni.devices.get(r) or {}) for r in names)
    free = sum(len(ni.available_devices(r)) for r in names)
    used_after = max(0, total - max(0, free - pi.gpu_count))
    fill = used_after * 5 // total if total else 0
    t = ni.topology()
    if t is None:
        return 2 + fill
    ids, index, numa, link, parent = t
    q = 0.0
    for _, rname, n, sel in pi.ext:
        cand = matching_free(pi, ni, rname, sel)
        if not all(d in index for d in cand):
            return 2 + fill
        free_all = [index[d] for d in ni.available_devices(rname) if d in index]
        q += topo.score([index[d] for d in cand], n, link, numa, free_all, parent)
    quality = int(max(0.0, min(10.0, q / len(pi.ext)))) // 2
    return quality + fill
