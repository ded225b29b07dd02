"""Scheduler policy arguments (plugin/pkg/scheduler/api/types.go PredicateArgument /
PriorityArgument; factory/plugins.go RegisterCustomFitPredicate / RegisterCustomPriorityFunction):
policy entries that carry an `argument` build a predicate or priority of their own.

  predicates: {"name": N, "argument": {"serviceAffinity": {"labels": [...]}}}
                — pods of one service land on nodes that agree, for these labels, with the
                  nodes the service's first pods landed on (predicates.go ServiceAffinity)
              {"name": N, "argument": {"labelsPresence": {"labels": [...], "presence": bool}}}
                — the node has all (presence) or none (absence) of the labels
  priorities: {"name": N, "weight": W, "argument": {"serviceAntiAffinity": {"label": L}}}
                — spread a service's pods over the values of label L (selector_spreading.go)
              {"name": N, "weight": W, "argument": {"labelPreference": {"label": L, "presence": bool}}}
                — prefer nodes that have (or lack) label L (node_label.go)
"""
from __future__ import annotations

from ..api import meta as m
from ..api.labels import selector_from_set
from .predicates import ERR_NODE_LABEL_PRESENCE_VIOLATED, ERR_SERVICE_AFFINITY_VIOLATED, OK, _fail

MAX = 10


def _service_affinity_pods(pi, ni, ctx):
    """serviceAffinityMetadataProducer + FilterOutPods (predicates.go:829-847, :898): when a
    Service in the pod's namespace selects it, the placed pods of that namespace whose labels
    carry all of the pod's labels, as (pod, node) — pods the candidate node's NodeInfo does not
    hold are skipped."""
    ns = m.namespace_of(pi.pod)
    if not any(m.namespace_of(s) == ns and (s.get("spec") or {}).get("selector") is not None
               and selector_from_set((s.get("spec") or {}).get("selector") or {}).matches(pi.labels)
               for s in (ctx.services() if ctx else [])):
        return []
    own = selector_from_set(pi.labels)
    out = []
    for other in (ctx.nodes if ctx else [ni]):
        for p in other.pods.values():
            if m.namespace_of(p) == ns and own.matches(m.labels_of(p)):
                out.append((p, other))
    return out


def service_affinity(labels: list[str]):
    """checkServiceAffinity (predicates.go:886-922): labels the pod's nodeSelector does not pin
    are taken from the node of the first placed pod of its service."""
    def pred(pi, ni, ctx=None):
        want = {k: pi.node_selector[k] for k in labels if k in pi.node_selector}
        if len(want) < len(labels):
            placed = _service_affinity_pods(pi, ni, ctx)
            if placed:
                first = placed[0][1]
                for k in labels:
                    if k not in want and k in first.labels:
                        want[k] = first.labels[k]
        if all(ni.labels.get(k) == v for k, v in want.items()):
            return OK
        return _fail(ERR_SERVICE_AFFINITY_VIOLATED)
    return pred


def labels_presence(labels: list[str], presence: bool):
    def pred(pi, ni, ctx=None):
        has = all(k in ni.labels for k in labels) if presence else not any(k in ni.labels for k in labels)
        return OK if has else _fail(ERR_NODE_LABEL_PRESENCE_VIOLATED)
    return pred


def service_anti_affinity(label: str):
    """ServiceAntiAffinity.CalculateAntiAffinityPriority (selector_spreading.go:185-254): the
    first Service selecting the pod names the pods to spread; a labelled node scores
    10 * (service pods - service pods in its label value) / service pods, an unlabelled one 0.
    The denominator counts every service pod, wherever it runs; the per-value counts only those
    on the nodes being scored."""
    def prio(pi, nodes, ctx=None):
        ns = m.namespace_of(pi.pod)
        svcs = [s for s in (ctx.services() if ctx is not None else [])
                if m.namespace_of(s) == ns and (s.get("spec") or {}).get("selector")
                and selector_from_set(s["spec"]["selector"]).matches(pi.labels)]
        labeled = {ni.name: ni.labels[label] for ni in nodes if label in ni.labels}
        counts: dict[str, int] = {}
        total = 0
        if svcs:
            sel = selector_from_set(svcs[0]["spec"]["selector"])
            for ni in ctx.nodes:
                for p in ni.pods.values():
                    if m.namespace_of(p) != ns or not sel.matches(m.labels_of(p)):
                        continue
                    total += 1
                    v = labeled.get(ni.name)
                    if v is not None:
                        counts[v] = counts.get(v, 0) + 1
        out = []
        for ni in nodes:
            v = labeled.get(ni.name)
            if v is None:
                out.append(0)
            elif total == 0:
                out.append(MAX)
            else:
                out.append(int(float(MAX) * ((total - counts.get(v, 0)) / total)))
        return out
    return prio


def label_preference(label: str, presence: bool):
    def prio(pi, nodes, ctx=None):
        return [MAX if (label in ni.labels) == presence else 0 for ni in nodes]
    return prio


def build(policy: dict) -> tuple[list, dict, dict, dict]:
    """(predicate names, priority weights, custom predicates, custom priorities)."""
    from .predicates import DEFAULT_PREDICATES, PREDICATES
    from .priorities import DEFAULT_PRIORITIES, PRIORITIES
    cpreds, cprios = {}, {}
    preds = []
    if "predicates" in policy:
        for p in policy.get("predicates") or []:
            arg = p.get("argument") or {}
            if "serviceAffinity" in arg:
                cpreds[p["name"]] = service_affinity(list(arg["serviceAffinity"].get("labels") or []))
            elif "labelsPresence" in arg:
                lp = arg["labelsPresence"]
                cpreds[p["name"]] = labels_presence(list(lp.get("labels") or []), bool(lp.get("presence")))
            elif p["name"] not in PREDICATES:
                raise ValueError(f"unknown predicate {p['name']!r} and no argument to build it from")
            preds.append(p["name"])
    else:
        preds = list(DEFAULT_PREDICATES)
    prios = {}
    if "priorities" in policy:
        for p in policy.get("priorities") or []:
            arg = p.get("argument") or {}
            if "serviceAntiAffinity" in arg:
                cprios[p["name"]] = service_anti_affinity(arg["serviceAntiAffinity"]["label"])
            elif "labelPreference" in arg:
                lp = arg["labelPreference"]
                cprios[p["name"]] = label_preference(lp["label"], bool(lp.get("presence")))
            elif p["name"] not in PRIORITIES:
                raise ValueError(f"unknown priority {p['name']!r} and no argument to build it from")
            prios[p["name"]] = int(p.get("weight", 1))
    else:
        prios = dict(DEFAULT_PRIORITIES)
    return preds, prios, cpreds, cprios
