"""Fit predicates (filter phase).

Reference: plugin/pkg/scheduler/algorithm/predicates/predicates.go — PodFitsResources,
PodFitsHost, PodFitsHostPorts, PodMatchNodeSelector, GeneralPredicates (:965-1020),
PodToleratesNodeTaints, CheckNodeCondition, CheckNodeMemoryPressure/DiskPressure,
NoDiskConflict, MatchInterPodAffinity; registered names (policy-file compatibility) from
algorithmprovider/defaults/defaults.go:119-215. The volume predicates (NoVolumeZoneConflict,
Max{EBS,GCEPD,AzureDisk}VolumeCount, CheckVolumeBinding) live in scheduler/volumes.py and read
the claims/volumes the scheduler resolved for the pod (`pi.vol`).

A PodInfo pre-computes everything derived from the pod once per scheduling attempt, so the
per-node loop is dictionary lookups only.
"""
from __future__ import annotations

from ..api import meta as m
from ..api.helpers import (find_untolerated_taint, get_condition, pod_extended_resource_count, pod_extended_resource_name,
                           pod_host_ports, pod_requests, ExtendedResourceError, is_extended_resource_name)
from ..api.labels import node_requirements_as_selector, selector_from_label_selector, SelectorError


class PodInfo:
    def __init__(self, pod: dict):
        self.pod = pod
        self.key = m.key_of(pod)
        spec = pod.get("spec") or {}
        self.spec = spec
        self.requests = pod_requests(pod)
        self.ports = pod_host_ports(pod)
        self.node_selector = spec.get("nodeSelector") or {}
        na = ((spec.get("affinity") or {}).get("nodeAffinity") or {})
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution") or {}
        self.required_terms = [node_requirements_as_selector(t.get("matchExpressions")) for t in req.get("nodeSelectorTerms") or []]
        self.preferred_terms = [(int(t.get("weight", 0)), node_requirements_as_selector((t.get("preference") or {}).get("matchExpressions")))
                                for t in na.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
        self.tolerations = spec.get("tolerations") or []
        self.priority = int(spec.get("priority") or 0)
        self.qos = (pod.get("status") or {}).get("qosClass") or ""
        self.best_effort = not any((c.get("resources") or {}).get("requests") or (c.get("resources") or {}).get("limits")
                                   for c in spec.get("containers") or [])
        self.ext = []   # [(pres name, resource name, count, selector)]
        self.ext_error = None
        for pres in spec.get("extendedResources") or []:
            try:
                rn = pod_extended_resource_name(pres)
                self.ext.append((pres.get("name"), rn, pod_extended_resource_count(pres),
                                 node_requirements_as_selector((pres.get("affinity") or {}).get("required"))))
            except (ExtendedResourceError, SelectorError) as e:
                self.ext_error = str(e)
        self.gpu_count = sum(n for _, _, n, _ in self.ext)
        aff = spec.get("affinity") or {}
        self.pod_affinity = (aff.get("podAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or []
        self.pod_anti_affinity = (aff.get("podAntiAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or []
        self.pref_affinity = (aff.get("podAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or []
        self.pref_anti = (aff.get("podAntiAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or []
        self.owner = m.controller_ref(pod)
        self.labels = m.labels_of(pod)


def _fail(*reasons):
    return False, list(reasons)


OK = (True, [])


def pod_fits_resources(pi: PodInfo, ni, ctx=None):
    alloc = ni.allocatable
    reasons = []
    if len(ni.pods) + 1 > alloc.get("pods", 110):
        reasons.append("Insufficient pods")
    for k, v in pi.requests.items():
        if v <= 0:
            continue
        cap = alloc.get(k)
        if cap is None:
            if is_extended_resource_name(k) or k in ("cpu", "memory"):
                reasons.append(f"Insufficient {k}")
            continue
        if ni.requested.get(k, 0) + v > cap:
            reasons.append(f"Insufficient {k}")
    return (not reasons), reasons


def pod_fits_host(pi, ni, ctx=None):
    nn = pi.spec.get("nodeName")
    if nn and nn != ni.name:
        return _fail("node(s) didn't match the requested hostname")
    return OK


def pod_fits_host_ports(pi, ni, ctx=None):
    for hp in pi.ports:
        for used in ni.ports:
            if used[2] == hp[2] and used[1] == hp[1] and (used[0] == hp[0] or "0.0.0.0" in (used[0], hp[0])):
                return _fail("node(s) didn't have free ports for the requested pod ports")
    return OK


def pod_match_node_selector(pi, ni, ctx=None):
    labels = ni.labels
    for k, v in pi.node_selector.items():
        if labels.get(k) != v:
            return _fail("node(s) didn't match node selector")
    if pi.required_terms and not any(s.matches(labels) for s in pi.required_terms):
        return _fail("node(s) didn't match node selector")
    return OK


def general_predicates(pi, ni, ctx=None):
    reasons = []
    for p in (pod_fits_resources, pod_fits_host, pod_fits_host_ports, pod_match_node_selector):
        ok, r = p(pi, ni, ctx)
        reasons += r
    return (not reasons), reasons


def pod_tolerates_node_taints(pi, ni, ctx=None):
    t = find_untolerated_taint(ni.taints, pi.tolerations, ("NoSchedule", "NoExecute"))
    if t:
        return _fail("node(s) had taints that the pod didn't tolerate")
    return OK


def check_node_condition(pi, ni, ctx=None):
    node = ni.node or {}
    if (node.get("spec") or {}).get("unschedulable"):
        return _fail("node(s) were unschedulable")
    ready = get_condition(node, "Ready")
    if ready is None or ready.get("status") != "True":
        return _fail("node(s) were not ready")
    od = get_condition(node, "OutOfDisk")
    if od is not None and od.get("status") == "True":
        return _fail("node(s) were out of disk space")
    nu = get_condition(node, "NetworkUnavailable")
    if nu is not None and nu.get("status") == "True":
        return _fail("node(s) had unavailable network")
    return OK


def check_node_memory_pressure(pi, ni, ctx=None):
    if not pi.best_effort:
        return OK
    c = get_condition(ni.node or {}, "MemoryPressure")
    if c is not None and c.get("status") == "True":
        return _fail("node(s) had memory pressure")
    return OK


def check_node_disk_pressure(pi, ni, ctx=None):
    c = get_condition(ni.node or {}, "DiskPressure")
    if c is not None and c.get("status") == "True":
        return _fail("node(s) had disk pressure")
    return OK


def _vol_ids(pod):
    out = set()
    for v in (pod.get("spec") or {}).get("volumes") or []:
        for kind, idk in (("gcePersistentDisk", "pdName"), ("awsElasticBlockStore", "volumeID"), ("rbd", "image"), ("iscsi", "iqn")):
            if kind in v:
                out.add((kind, v[kind].get(idk), bool(v[kind].get("readOnly"))))
    return out


def no_disk_conflict(pi, ni, ctx=None):
    """isVolumeConflict: the same GCE PD / RBD image / iSCSI IQN may be shared only when every
    user mounts it read-only; an AWS EBS volume attaches to one instance, so never twice."""
    mine = _vol_ids(pi.pod)
    if not mine:
        return OK
    for p in ni.pods.values():
        for kind, vid, ro in _vol_ids(p):
            for k2, v2, ro2 in mine:
                if kind == k2 and vid == v2 and (kind == "awsElasticBlockStore" or not (ro and ro2)):
                    return _fail("node(s) had no available disk")
    return OK


def _topology_value(ni, key):
    return ni.labels.get(key) if key else None


def _term_selector(term):
    return selector_from_label_selector(term.get("labelSelector"))


def _term_namespaces(term, pod):
    return set(term.get("namespaces") or [m.namespace_of(pod)])


def match_inter_pod_affinity(pi, ni, ctx=None):
    """Required pod (anti-)affinity with topologyKey (hostname or any node label)."""
    nodes = ctx.nodes if ctx else None
    if not (pi.pod_affinity or pi.pod_anti_affinity) and not (ctx and ctx.any_anti_affinity):
        return OK
    all_nodes = nodes if nodes is not None else [ni]
    for term in pi.pod_anti_affinity:
        key = term.get("topologyKey")
        val = _topology_value(ni, key)
        sel, nss = _term_selector(term), _term_namespaces(term, pi.pod)
        for other in all_nodes:
            if val is None or _topology_value(other, key) != val:
                continue
            for p in other.pods.values():
                if m.namespace_of(p) in nss and sel.matches(m.labels_of(p)):
                    return _fail("node(s) didn't match pod anti-affinity rules")
    for term in pi.pod_affinity:
        key = term.get("topologyKey")
        val = _topology_value(ni, key)
        sel, nss = _term_selector(term), _term_namespaces(term, pi.pod)
        found = any(_topology_value(o, key) == val and val is not None and any(
            m.namespace_of(p) in nss and sel.matches(m.labels_of(p)) for p in o.pods.values()) for o in all_nodes)
        if not found:
            anywhere = any(m.namespace_of(p) in nss and sel.matches(m.labels_of(p)) for o in all_nodes for p in o.pods.values())
            if anywhere or not (sel.matches(pi.labels) and m.namespace_of(pi.pod) in nss):
                return _fail("node(s) didn't match pod affinity rules")
    if ctx and ctx.any_anti_affinity:  # existing pods' anti-affinity against this pod
        for other in all_nodes:
            for p in other.pods.values():
                terms = (((p.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {}).get(
                    "requiredDuringSchedulingIgnoredDuringExecution") or []
                for term in terms:
                    key = term.get("topologyKey")
                    if _topology_value(other, key) is None or _topology_value(other, key) != _topology_value(ni, key):
                        continue
                    if m.namespace_of(pi.pod) in _term_namespaces(term, p) and _term_selector(term).matches(pi.labels):
                        return _fail("node(s) didn't satisfy existing pods anti-affinity rules")
    return OK


def always_fit(pi, ni, ctx=None):
    return OK


def no_volume_zone_conflict(pi, ni, ctx=None):
    vol = getattr(pi, "vol", None)
    if vol is None:
        return OK
    if vol.missing:
        return _fail(f'persistentvolumeclaim "{vol.missing[0]}" not found')
    from .volumes import no_volume_zone_conflict as zc
    return OK if zc(vol.bound, ni.labels) else _fail("node(s) had no available volume zone")


def _max_pd(kind):
    def pred(pi, ni, ctx=None):
        from .volumes import MAX_PD, max_pd_limit, pod_volumes
        vol = getattr(pi, "vol", None)
        idk = MAX_PD[kind][0]
        mine = {src.get(idk) for k, src in (vol.sources if vol is not None else []) if k == kind}
        if not mine:
            return OK             # the reference's early exit: the pod adds no such disk
        have = set()
        for p in ni.pods.values():
            for k, src in pod_volumes(p, getattr(pi, "lister", None)).sources:
                if k == kind:
                    have.add(src.get(idk))
        if len(have | mine) > max_pd_limit(kind):
            return _fail("node(s) exceed max volume count")
        return OK
    pred.__name__ = f"max_{kind}_count"
    return pred


def check_volume_binding(pi, ni, ctx=None):
    vol = getattr(pi, "vol", None)
    if vol is None or not getattr(pi, "volume_scheduling", False):
        return OK
    from .volumes import match_delayed, pv_node_affinity_ok
    if vol.unbound:
        return _fail("pod has unbound PersistentVolumeClaims")
    for pvc, pv in vol.bound:
        if not pv_node_affinity_ok(pv, ni.labels):
            return _fail("node(s) had volume node affinity conflict")
    if vol.delayed and match_delayed(vol.delayed, pi.lister, ni.labels) is None:
        return _fail("node(s) didn't find available persistent volumes to bind")
    return OK


PREDICATES = {
    "PodFitsResources": pod_fits_resources,
    "PodFitsHost": pod_fits_host,
    "PodFitsHostPorts": pod_fits_host_ports,
    "PodFitsPorts": pod_fits_host_ports,
    "PodMatchNodeSelector": pod_match_node_selector,
    "HostName": pod_fits_host,
    "MatchNodeSelector": pod_match_node_selector,
    "GeneralPredicates": general_predicates,
    "PodToleratesNodeTaints": pod_tolerates_node_taints,
    "CheckNodeCondition": check_node_condition,
    "CheckNodeMemoryPressure": check_node_memory_pressure,
    "CheckNodeDiskPressure": check_node_disk_pressure,
    "NoDiskConflict": no_disk_conflict,
    "MatchInterPodAffinity": match_inter_pod_affinity,
    "NoVolumeZoneConflict": no_volume_zone_conflict,
    "MaxEBSVolumeCount": _max_pd("awsElasticBlockStore"),
    "MaxGCEPDVolumeCount": _max_pd("gcePersistentDisk"),
    "MaxAzureDiskVolumeCount": _max_pd("azureDisk"),
    "CheckVolumeBinding": check_volume_binding,
}

# evaluation order (cheap → expensive), predicates.go predicatesOrdering
ORDER = ["CheckNodeCondition", "GeneralPredicates", "HostName", "PodFitsHostPorts", "MatchNodeSelector", "PodFitsResources",
         "NoDiskConflict", "PodToleratesNodeTaints", "CheckNodeMemoryPressure", "CheckNodeDiskPressure", "MaxEBSVolumeCount",
         "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount", "CheckVolumeBinding", "NoVolumeZoneConflict", "MatchInterPodAffinity",
         "PodFitsHost", "PodMatchNodeSelector", "PodFitsPorts"]

DEFAULT_PREDICATES = ["NoVolumeZoneConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                      "MatchInterPodAffinity", "NoDiskConflict", "GeneralPredicates", "CheckNodeMemoryPressure",
                      "CheckNodeDiskPressure", "CheckNodeCondition", "PodToleratesNodeTaints", "CheckVolumeBinding"]
