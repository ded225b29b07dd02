"""genericScheduler: filter → device allocation → prioritize → select host; preemption.

Reference: plugin/pkg/scheduler/core/generic_scheduler.go — Schedule (:109-159, traced with
LogIfLong(100ms) and steps "Computing predicates"/"Prioritizing"/"Selecting host"),
findNodesThatFit (:283-361, Parallelize(16) + extenders + the fork's GetExtendedResources
at :353-358), podFitsOnNode (:402), PrioritizeNodes (:509), selectHost round-robin among
the maxima (:178-193), Preempt (:199).

Fixes: #5 (no predicates configured no longer turns the node list into nils — the filtered
list is always the real nodes), #7 (preemption simulates the device allocator too).
"""
from __future__ import annotations

import logging

from ..api import meta as m
from ..utils.trace import Trace
from . import extended
from .predicates import (ERR_NODE_LABEL_PRESENCE_VIOLATED, ERR_NODE_NETWORK_UNAVAILABLE, ERR_NODE_NOT_READY,
                         ERR_NODE_SELECTOR_NOT_MATCH, ERR_NODE_UNKNOWN_CONDITION, ERR_NODE_UNSCHEDULABLE,
                         ERR_POD_NOT_MATCH_HOST_NAME, ERR_TAINTS_TOLERATIONS_NOT_MATCH, ERR_VOLUME_BIND_CONFLICT,
                         ERR_VOLUME_NODE_CONFLICT, ERR_VOLUME_ZONE_CONFLICT, ORDER, PREDICATES, PodInfo)
from .priorities import PRIORITIES, pod_selectors

log = logging.getLogger("amdkube.scheduler")


# priorities whose per-node value depends only on that node and the pod (cacheable per node generation)
LOCAL_PRIORITIES = {"LeastRequestedPriority", "MostRequestedPriority", "BalancedResourceAllocation",
                    "NodePreferAvoidPodsPriority", "ImageLocalityPriority", "GPUTopologyPriority",
                    "ResourceLimitsPriority", "EqualPriority"}


class FitError(Exception):
    def __init__(self, pod, n_nodes, failed: dict):
        self.pod, self.n_nodes, self.failed = pod, n_nodes, failed
        # FitError.Error (core/generic_scheduler.go:70-88): a histogram of reasons, "<n> <reason>"
        # strings sorted as strings
        counts: dict[str, int] = {}
        for reasons in failed.values():
            for r in reasons:
                counts[r] = counts.get(r, 0) + 1
        msg = ", ".join(sorted(f"{c} {r}" for r, c in counts.items()))
        super().__init__(f"0/{n_nodes} nodes are available: {msg}." if n_nodes else "no nodes available to schedule pods")


FIT_INDEX_CLASSES = 256    # equivalence classes kept (least recently used dropped first)


class _FitIndex:
    """One equivalence class's answer for every ready node, kept current by replaying the
    cache's node-change log: `fit` maps node name -> the node-local priority total, `failed`
    node name -> predicate failure reasons. A pod of the class costs O(nodes changed since the
    last pod of the class) instead of O(nodes) (scheduler_perf at 1000 nodes: each bind changes
    one node)."""
    __slots__ = ("pos", "fit", "failed")

    def __init__(self):
        self.pos = -1
        self.fit: dict[str, int] = {}
        self.failed: dict[str, list] = {}


class Context:
    __slots__ = ("nodes", "any_anti_affinity", "any_affinity", "hard_weight", "services", "listers", "any_pref_affinity")

    def __init__(self, nodes, any_anti_affinity, any_affinity=False, hard_weight=0, services=None, listers=None,
                 any_pref_affinity=False):
        self.nodes, self.any_anti_affinity = nodes, any_anti_affinity
        self.any_pref_affinity = any_pref_affinity
        self.any_affinity, self.hard_weight = any_affinity, hard_weight
        self.services = services or (lambda: [])
        self.listers = listers


class GenericScheduler:
    def __init__(self, cache, predicates: list[str], priorities: dict[str, int], extenders=(), use_topology=True,
                 trace_threshold: float = 0.1, volumes=None, volume_scheduling: bool = False, custom_predicates=None,
                 custom_priorities=None, services=None, hard_affinity_weight: int = 1, listers=None):
        from .listers import ControllerListers
        self.cache = cache
        # Services/RCs/RSs/StatefulSets for the spreading priorities (metadata.go getSelectors)
        self.listers = listers or ControllerListers(services=services)
        self.volumes = volumes                  # scheduler/volumes.VolumeLister (claims, volumes, classes)
        self.volume_scheduling = volume_scheduling
        self.volume_binds: dict[str, list] = {}  # pod key -> [(pvc, pv)] to pre-bind before the pod
        self.services = services
        self.configure(predicates, priorities, custom_predicates or {}, custom_priorities or {}, extenders,
                       hard_affinity_weight)
        self.use_topology = use_topology
        self.last_index = 0
        self.trace_threshold = trace_threshold
        self.ecache: dict[str, dict[str, tuple]] = {}
        self.ecache_hits = 0
        self.findex: dict[str, _FitIndex] = {}
        self.queue = None               # the SchedulingQueue (nominated pods), set by the Scheduler

    def configure(self, predicates, priorities, custom_predicates, custom_priorities, extenders, hard_affinity_weight):
        """(Re)build the algorithm from a policy: registered names plus policy-argument functions."""
        names = [p for p in ORDER if p in predicates] + [p for p in predicates if p not in ORDER]
        self.predicates = [(n, custom_predicates.get(n) or PREDICATES[n]) for n in names]
        self.priorities = [(n, custom_priorities.get(n) or PRIORITIES[n], w) for n, w in priorities.items() if w]
        self.extenders = list(extenders)
        self.hard_affinity_weight = hard_affinity_weight
        self.custom = bool(custom_predicates or custom_priorities)
        self.ecache = {}
        self.findex = {}

    @property
    def _lctx(self):
        """A node-less context carrying only the listers (selector lookups)."""
        return Context((), False, listers=self.listers)

    def _ctx(self, nodes):
        return Context(nodes, self.cache.anti_affinity_pods > 0, getattr(self.cache, "affinity_pods", 0) > 0,
                       self.hard_affinity_weight, self.services, self.listers,
                       getattr(self.cache, "pref_affinity_pods", 0) > 0)

    # Equivalence cache (reference plugin/pkg/scheduler/core/equivalence_cache.go:38): pods with the
    # same scheduling-relevant spec get the same per-node answer as long as the node is unchanged.
    # Keyed by (equivalence class, node) and validated by the node's generation, which moves on
    # every node update and every pod add/remove on that node — so only nodes that changed since
    # the last identical pod are re-evaluated. Pods with inter-pod (anti-)affinity, or any cluster
    # with anti-affinity pods, bypass it (their answer depends on other nodes).
    def _equiv_key(self, pi):
        if pi.pod_affinity or pi.pod_anti_affinity or pi.pref_affinity or pi.pref_anti or self.cache.anti_affinity_pods or \
                self.custom or (self.hard_affinity_weight and getattr(self.cache, "affinity_pods", 0)):
            return None
        if pi.ext_error:
            return None
        spec = pi.spec
        if any("persistentVolumeClaim" in v for v in spec.get("volumes") or []):
            return None     # the answer depends on claim/volume state, not just the node
        import json as _json
        # images are part of the class: ImageLocalityPriority is a node-local score
        rel = {"c": [(c.get("resources"), c.get("ports"), c.get("image")) for c in spec.get("containers") or []],
               "i": [c.get("resources") for c in spec.get("initContainers") or []],
               "ns": spec.get("nodeSelector"), "aff": spec.get("affinity"), "tol": spec.get("tolerations"),
               "nn": spec.get("nodeName"), "x": [(r.get("resources"), r.get("affinity")) for r in spec.get("extendedResources") or []],
               "v": [v for v in spec.get("volumes") or [] if len(v) > 1 and "emptyDir" not in v],
               "o": (pi.owner or {}).get("uid"), "be": pi.best_effort}
        return _json.dumps(rel, sort_keys=True, separators=(",", ":"))

    def pod_fits_on_node(self, pi, ni, ctx) -> tuple[bool, list[str]]:
        reasons = []
        for name, fn in self.predicates:
            ok, r = fn(pi, ni, ctx)
            if not ok:
                reasons += r       # every predicate runs and reports (podFitsOnNode, no early exit)
        if not reasons:
            ok, r = extended.fits(pi, ni)
            reasons += r
        return (not reasons), reasons

    # ------------------------------------------------------------ fast path
    def _uniform_others(self, pi) -> bool:
        """Whether every node-normalising priority gives all nodes the same score for this pod
        (so they cannot change the choice and need not run): no controller to spread, no
        preferred node or pod (anti-)affinity, no PreferNoSchedule taint anywhere."""
        for name, _fn, _w in self.priorities:
            if name in LOCAL_PRIORITIES:
                continue
            if name == "SelectorSpreadPriority" and not pod_selectors(pi, self._lctx):
                continue
            if name == "ServiceSpreadingPriority" and not pod_selectors(pi, self._lctx, services_only=True):
                continue
            if name == "NodeAffinityPriority" and not pi.preferred_terms:
                continue
            if name == "TaintTolerationPriority" and not self.cache.prefer_no_schedule:
                continue
            if name == "InterPodAffinityPriority" and not (pi.pref_affinity or pi.pref_anti) and \
                    not (self.hard_affinity_weight and getattr(self.cache, "affinity_pods", 0)) and \
                    not getattr(self.cache, "pref_affinity_pods", 0):
                continue
            return False
        return True

    def _eval_node(self, pi, ni, local) -> tuple[bool, list, int]:
        ok, reasons = self.pod_fits_on_node(pi, ni, None)
        score = 0
        if ok:
            for _name, fn, w in local:
                score += fn(pi, [ni], None)[0] * w
        return ok, reasons, score

    def _fit_index(self, pi, ek) -> _FitIndex:
        c = self.cache
        idx = self.findex.pop(ek, None)          # re-inserted below: the dict's order is recency (LRU)
        local = [(n, fn, w) for n, fn, w in self.priorities if n in LOCAL_PRIORITIES]
        if idx is None or idx.pos < c.log_base:
            while len(self.findex) >= FIT_INDEX_CLASSES:  # each class holds an entry per node
                self.findex.pop(next(iter(self.findex)))
            idx = _FitIndex()
            for ni in c.ready_nodes():
                ok, reasons, score = self._eval_node(pi, ni, local)
                if ok:
                    idx.fit[ni.name] = score
                else:
                    idx.failed[ni.name] = reasons
        else:
            changed = dict.fromkeys(c.log[idx.pos - c.log_base:])
            self.ecache_hits += max(0, len(idx.fit) + len(idx.failed) - len(changed))
            for name in changed:
                ni = c.nodes.get(name)
                if ni is None or ni.node is None:
                    idx.fit.pop(name, None)
                    idx.failed.pop(name, None)
                    continue
                ok, reasons, score = self._eval_node(pi, ni, local)
                if ok:
                    idx.failed.pop(name, None)
                    idx.fit[name] = score
                else:
                    idx.fit.pop(name, None)
                    idx.failed[name] = reasons
        idx.pos = c.seq
        self.findex[ek] = idx
        return idx

    async def find_nodes_that_fit(self, pi, nodes):
        ctx = self._ctx(nodes) if (pi.pod_affinity or pi.pod_anti_affinity) or self.custom or any(
            n == "MatchInterPodAffinity" for n, _ in self.predicates) else None
        fit, failed = [], {}
        ek = self._equiv_key(pi)
        pi.equiv = ek
        cache = self.ecache.setdefault(ek, {}) if ek is not None else None
        if cache is not None and len(self.ecache) > 4096:
            self.ecache.clear()
            cache = self.ecache.setdefault(ek, {})
        for ni in nodes:
            hit = cache.get(ni.name) if cache is not None else None
            if hit is not None and hit[0] == ni.generation:
                ok, reasons = hit[1], hit[2]
                self.ecache_hits += 1
            else:
                ok, reasons = self.pod_fits_on_node(pi, ni, ctx)
                if cache is not None:
                    cache[ni.name] = (ni.generation, ok, reasons, None)
            if ok:
                fit.append(ni)
            else:
                failed[ni.name] = reasons
        if fit and self.extenders:
            for ext in self.extenders:
                if not ext.filter_verb:
                    continue
                names, ext_failed = await ext.filter(pi.pod, [ni.node for ni in fit])
                failed.update({k: [v] for k, v in ext_failed.items()})
                keep = set(names)
                fit = [ni for ni in fit if ni.name in keep]
                if not fit:
                    break
        return fit, failed, ctx

    async def prioritize(self, pi, nodes, ctx) -> list[int]:
        """PrioritizeNodes: integer weighted totals (HostPriority.Score is an int)."""
        if not self.priorities and not self.extenders:
            return [1] * len(nodes)
        if ctx is None and (self.custom or (self.hard_affinity_weight and self.cache.affinity_pods) or
                            any(n not in LOCAL_PRIORITIES for n, _fn, _w in self.priorities)):
            ctx = self._ctx(self.cache.ready_nodes())
        total = [0] * len(nodes)
        # per-node scores depend only on (pod class, node state) unless a priority normalises across
        # nodes; only the normalising ones (spread, affinity, taints) are recomputed every time
        cache = self.ecache.get(pi.equiv) if getattr(pi, "equiv", None) is not None else None
        local = [(n, fn, w) for n, fn, w in self.priorities if n in LOCAL_PRIORITIES]
        others = [(n, fn, w) for n, fn, w in self.priorities if n not in LOCAL_PRIORITIES]
        need = []
        for i, ni in enumerate(nodes):
            hit = cache.get(ni.name) if cache is not None else None
            if hit is not None and hit[0] == ni.generation and hit[3] is not None:
                total[i] += hit[3]
            else:
                need.append(i)
        if need:
            sub = [nodes[i] for i in need]
            part = [0] * len(sub)
            for name, fn, w in local:
                for j, s in enumerate(fn(pi, sub, ctx)):
                    part[j] += s * w
            for j, i in enumerate(need):
                total[i] += part[j]
                if cache is not None and nodes[i].name in cache and cache[nodes[i].name][0] == nodes[i].generation:
                    g, ok, reasons, _ = cache[nodes[i].name]
                    cache[nodes[i].name] = (g, ok, reasons, part[j])
        for name, fn, w in others:
            scores = fn(pi, nodes, ctx)
            for i, s in enumerate(scores):
                total[i] += s * w
        for ext in self.extenders:
            if not ext.prioritize_verb:
                continue
            scores = await ext.prioritize(pi.pod, [ni.node for ni in nodes])
            for i, ni in enumerate(nodes):
                total[i] += scores.get(ni.name, 0) * ext.weight
        return total

    def select_host(self, nodes, scores):
        """selectHost (generic_scheduler.go): the list sorted by HostPriorityList's order reversed
        (score, then host name, descending); round-robin among the hosts with the top score."""
        best = max(scores)
        idx = sorted((i for i, s in enumerate(scores) if s == best), key=lambda i: nodes[i].name, reverse=True)
        pick = idx[self.last_index % len(idx)]
        self.last_index += 1
        return nodes[pick]

    async def schedule(self, pod: dict):
        """Returns (node name, extendedResourceBinding). Raises FitError."""
        trace = Trace(f"Scheduling {m.key_of(pod)}")
        pi = PodInfo(pod)
        if (pod.get("spec") or {}).get("volumes"):
            from .volumes import pod_volumes
            pi.lister, pi.volume_scheduling = self.volumes, self.volume_scheduling
            pi.vol = pod_volumes(pod, self.volumes)
        ek = None if self.extenders or self.custom else self._equiv_key(pi)
        if ek is not None and self._uniform_others(pi):
            # incremental path: the class's fit index, only changed nodes re-checked
            pi.equiv = ek
            trace.step("Computing predicates (fit index)")
            idx = self._fit_index(pi, ek)
            n_ready = len(idx.fit) + len(idx.failed)
            if not n_ready:
                raise FitError(pod, 0, {})
            if not idx.fit:
                raise FitError(pod, n_ready, dict(idx.failed))
            names = list(idx.fit)
            fit = [self.cache.nodes[n] for n in names]
            scores = list(idx.fit.values())
            if self.queue is not None and self.queue.nominated:
                failed = dict(idx.failed)
                keep = {ni.name for ni in self._filter_nominated(pi, fit, failed)}
                if len(keep) != len(fit):
                    scores = [s for ni, s in zip(fit, scores) if ni.name in keep]
                    fit = [ni for ni in fit if ni.name in keep]
                    if not fit:
                        raise FitError(pod, n_ready, failed)
            scores = scores if len(fit) > 1 else None
            n_nodes = n_ready
            host = fit[0] if scores is None else self.select_host(fit, scores)
        else:
            nodes = self.cache.ready_nodes()
            n_nodes = len(nodes)
            if not nodes:
                raise FitError(pod, 0, {})
            trace.step("Computing predicates")
            fit, failed, ctx = await self.find_nodes_that_fit(pi, nodes)
            fit = self._filter_nominated(pi, fit, failed, ctx)
            if not fit:
                raise FitError(pod, len(nodes), failed)
            trace.step("Prioritizing")
            scores = None
            if len(fit) == 1:
                host = fit[0]
            else:
                scores = await self.prioritize(pi, fit, ctx)
                trace.step("Selecting host")
                host = self.select_host(fit, scores)
        binding = extended.allocate(pi, self._with_nominated(pi, host) or host, self.use_topology) if pi.ext else {}
        if binding is None:
            # the device choice failed on the best host: the next-ranked hosts get their turn
            failed_alloc = {host.name: ["device allocation failed"]}
            order = sorted(range(len(fit)), key=lambda i: -scores[i]) if scores is not None else range(len(fit))
            for alt in (fit[i] for i in order if fit[i] is not host):
                binding = extended.allocate(pi, alt, self.use_topology)
                if binding is not None:
                    host = alt
                    break
                failed_alloc[alt.name] = ["device allocation failed"]
            if binding is None:
                raise FitError(pod, n_nodes, failed_alloc)
        vol = getattr(pi, "vol", None)
        if vol is not None and vol.delayed and self.volume_scheduling:
            from .volumes import match_delayed
            pairs = match_delayed(vol.delayed, self.volumes, host.labels)
            if pairs is None:
                raise FitError(pod, n_nodes, {host.name: [ERR_VOLUME_BIND_CONFLICT]})
            self.volume_binds[m.key_of(pod)] = pairs
        trace.log_if_long(self.trace_threshold)
        return host.name, binding

    # -------------------------------------------------------------- nominated pods
    def _nominated_for(self, pi, node_name: str) -> list:
        """Pods nominated to `node_name` (waiting for a preemption there) whose priority is at
        least this pod's: it must not take the room freed for them (addNominatedPods :367-400)."""
        q = self.queue
        if q is None:
            return []
        return [p for p in q.waiting_pods_for_node(node_name)
                if pod_priority(p) >= pi.priority and m.key_of(p) != pi.key]

    def _with_nominated(self, pi, ni):
        """A copy of the node with those nominated pods added — their devices simulated as
        taken (the device allocator picks them on the copy) — or None when there are none."""
        noms = self._nominated_for(pi, ni.name)
        if not noms:
            return None
        sim = ni.clone()
        for p in noms:
            npi = PodInfo(p)
            if npi.ext:
                b = extended.allocate(npi, sim, False)
                if b:
                    got = {name: list(v["resources"]) for name, v in b.items()}
                else:
                    # its victims are still terminating: the devices free so far are its own
                    got, taken = {}, set()
                    for pname, rname, n, _sel in npi.ext:
                        free = [d for d in sim.available_devices(rname) if d not in taken][:n]
                        taken.update(free)
                        got[pname] = free
                spec = dict(p.get("spec") or {})
                spec["extendedResources"] = [dict(r, assigned=got[r["name"]]) if r.get("name") in got else r
                                             for r in spec.get("extendedResources") or []]
                p = dict(p, spec=spec)
            sim.add_pod(m.key_of(p), p)
        return sim

    def fits_with_nominated(self, pi, ni, ctx=None) -> tuple[bool, list[str]]:
        """podFitsOnNode's first pass (:402-470): the node as it would be with the nominated
        pods of equal or higher priority running. The second pass (without them) is the normal
        evaluation; a node must pass both."""
        sim = self._with_nominated(pi, ni)
        if sim is None:
            return True, []
        return self.pod_fits_on_node(pi, sim, ctx)

    def _filter_nominated(self, pi, fit, failed, ctx=None):
        if self.queue is None or not self.queue.nominated:
            return fit
        out = []
        for ni in fit:
            ok, reasons = self.fits_with_nominated(pi, ni, ctx)
            if ok:
                out.append(ni)
            else:
                failed[ni.name] = reasons
        return out

    # -------------------------------------------------------------- preemption
    def select_victims_on_node(self, pi, ni, pdbs=()):
        """selectVictimsOnNode (generic_scheduler.go:872-955): remove every lower-priority pod;
        if the pod then fits (nominated pods counted), reprieve victims from the highest
        priority down — PDB-violating ones first — while it still fits. Returns
        (victims, number of PDB-violating victims, fits). The device allocator is part of the
        fit (fix #7)."""
        sim = ni.clone()
        potential = [p for p in ni.pods.values() if pod_priority(p) < pi.priority]
        for p in potential:
            sim.remove_pod(m.key_of(p))
        potential.sort(key=pod_priority, reverse=True)       # util.HigherPriorityPod

        ctx = None
        if self.custom or any(n == "MatchInterPodAffinity" for n, _ in self.predicates):
            # inter-pod (anti-)affinity sees the node as it would be after the preemption
            ctx = self._ctx([sim if x.name == ni.name else x for x in self.cache.ready_nodes()])

        def fits():
            ok, _ = self.pod_fits_on_node(pi, sim, ctx)
            return ok and self.fits_with_nominated(pi, sim, ctx)[0]
        if not fits():
            return None, 0, False
        violating, non_violating = filter_pods_with_pdb_violation(potential, pdbs)
        victims, n_violating = [], 0

        def reprieve(p) -> bool:
            sim.add_pod(m.key_of(p), p)
            if fits():
                return True
            sim.remove_pod(m.key_of(p))
            victims.append(p)
            return False
        for p in violating:
            if not reprieve(p):
                n_violating += 1
        for p in non_violating:
            reprieve(p)
        return victims, n_violating, True

    def select_nodes_for_preemption(self, pi, nodes, pdbs=()) -> dict:
        """selectNodesForPreemption (:820-852): node name -> (victims, PDB violations) for every
        node where the pod fits after preemption."""
        out = {}
        for ni in nodes:
            victims, nviol, ok = self.select_victims_on_node(pi, ni, pdbs)
            if ok:
                out[ni.name] = (victims, nviol)
        return out

    def preempt(self, pod: dict, failed: dict | None = None, pdbs=()):
        """(node, victims): the node pickOneNodeForPreemption chooses among the nodes where
        preemption might help (all ready nodes when `failed` is None), without extenders."""
        pi = PodInfo(pod)
        if pi.spec.get("preemptionPolicy") == "Never":
            return None, []
        nodes = self.cache.ready_nodes()
        if failed is not None:
            keep = set(nodes_where_preemption_might_help([ni.name for ni in nodes], failed))
            nodes = [ni for ni in nodes if ni.name in keep]
        cand = self.select_nodes_for_preemption(pi, nodes, pdbs)
        name = pick_one_node_for_preemption(cand)
        return (name, cand[name][0]) if name is not None else (None, [])

    async def preempt_async(self, pod: dict, failed: dict, pdbs=()):
        """genericScheduler.Preempt (generic_scheduler.go:199-262): (node, victims, pods whose
        nomination is to be cleared). A pod whose earlier preemption still has victims
        terminating on its nominated node is not eligible; when no node can help, the pod's own
        nomination is cleared; a chosen node must pass the extenders with its victims removed;
        lower-priority pods nominated to that node lose their nomination."""
        pi = PodInfo(pod)
        if pi.spec.get("preemptionPolicy") == "Never":
            return None, [], []
        if not pod_eligible_to_preempt_others(pod, self.cache):
            return None, [], []
        nodes = self.cache.ready_nodes()
        if not nodes:
            return None, [], []
        keep = set(nodes_where_preemption_might_help([ni.name for ni in nodes], failed))
        potential = [ni for ni in nodes if ni.name in keep]
        if not potential:
            return None, [], [pod]
        cand = self.select_nodes_for_preemption(pi, potential, pdbs)
        while cand:
            name = pick_one_node_for_preemption(cand)
            if name is None:
                break
            victims = cand[name][0]
            if await self._node_passes_extenders(pod, name, victims):
                lower = [p for p in (self.queue.waiting_pods_for_node(name) if self.queue is not None else [])
                         if pod_priority(p) < pi.priority]
                return name, victims, lower
            del cand[name]
        return None, [], []

    async def _node_passes_extenders(self, pod, name, victims) -> bool:
        """nodePassesExtendersForPreemption (:854-884): the node with its victims removed."""
        filters = [e for e in self.extenders if e.filter_verb]
        if not filters:
            return True
        ni = self.cache.nodes.get(name)
        if ni is None or ni.node is None:
            return False
        for ext in filters:
            try:
                names, ext_failed = await ext.filter(pod, [ni.node])
            except Exception as e:
                log.warning("extender filter during preemption on %s: %r", name, e)
                return False
            if name in ext_failed or name not in set(names):
                return False
        return True


def pod_priority(pod: dict) -> int:
    """util.GetPodPriority: spec.priority, 0 when unset (no default PriorityClass)."""
    return int((pod.get("spec") or {}).get("priority") or 0)


# nodesWherePreemptionMightHelp (:957-997): failures that removing pods cannot fix
UNRESOLVABLE = {ERR_NODE_SELECTOR_NOT_MATCH, ERR_POD_NOT_MATCH_HOST_NAME, ERR_TAINTS_TOLERATIONS_NOT_MATCH,
                ERR_NODE_LABEL_PRESENCE_VIOLATED, ERR_NODE_NOT_READY, ERR_NODE_NETWORK_UNAVAILABLE,
                ERR_NODE_UNSCHEDULABLE, ERR_NODE_UNKNOWN_CONDITION, ERR_VOLUME_ZONE_CONFLICT,
                ERR_VOLUME_NODE_CONFLICT, ERR_VOLUME_BIND_CONFLICT}


def nodes_where_preemption_might_help(names, failed: dict) -> list:
    return [n for n in names if n not in failed or not any(r in UNRESOLVABLE for r in failed[n])]


def pod_eligible_to_preempt_others(pod: dict, cache) -> bool:
    """podEligibleToPreemptOthers (:999-1011): not while a lower-priority pod on the node the pod
    is nominated to is still terminating (its earlier preemption is in progress)."""
    from .queue import NOMINATED_NODE_ANNOTATION
    node = ((pod.get("metadata") or {}).get("annotations") or {}).get(NOMINATED_NODE_ANNOTATION)
    if not node:
        return True
    ni = cache.nodes.get(node)
    if ni is None:
        return True
    prio = pod_priority(pod)
    return not any((p.get("metadata") or {}).get("deletionTimestamp") and pod_priority(p) < prio
                   for p in ni.pods.values())


def filter_pods_with_pdb_violation(pods, pdbs):
    """filterPodsWithPDBViolation (:889-917): a pod whose matching PDB allows no disruption is a
    violating victim; order is kept."""
    from ..api.labels import SelectorError, selector_from_label_selector
    violating, non_violating = [], []
    for p in pods:
        labels = m.labels_of(p)
        hit = False
        if labels:
            for pdb in pdbs or ():
                if m.namespace_of(pdb) != m.namespace_of(p):
                    continue
                try:
                    sel = selector_from_label_selector((pdb.get("spec") or {}).get("selector"))
                except SelectorError:
                    continue
                if sel.empty() or not sel.matches(labels):
                    continue
                st = pdb.get("status") or {}
                if int(st.get("disruptionsAllowed", st.get("podDisruptionsAllowed", 0)) or 0) <= 0:
                    hit = True
                    break
        (violating if hit else non_violating).append(p)
    return violating, non_violating


def pick_one_node_for_preemption(node_to_victims: dict):
    """pickOneNodeForPreemption (:657-760): a node needing no preemption; else fewest PDB
    violations, then the lowest highest-priority victim (victims[0]), then the smallest sum
    of priorities (each shifted by MaxInt32+1), then the fewest victims, then the first."""
    if not node_to_victims:
        return None
    cands = []
    for name, (victims, nviol) in node_to_victims.items():
        if not victims:
            return name
        cands.append(name)

    def narrow(names, key):
        best = min(key(n) for n in names)
        return [n for n in names if key(n) == best]
    cands = narrow(cands, lambda n: node_to_victims[n][1])
    if len(cands) > 1:
        cands = narrow(cands, lambda n: pod_priority(node_to_victims[n][0][0]))
    if len(cands) > 1:
        cands = narrow(cands, lambda n: sum(pod_priority(p) + 2 ** 31 for p in node_to_victims[n][0]))
    if len(cands) > 1:
        cands = narrow(cands, lambda n: len(node_to_victims[n][0]))
    return cands[0]
