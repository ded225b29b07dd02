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


# Failure reasons: algorithm/predicates/error.go — PredicateFailureError.GetReason() is the
# predicate's name (:33-57); InsufficientResourceError's is "Insufficient <resource>" (:84).
ERR_DISK_CONFLICT = "NoDiskConflict"
ERR_VOLUME_ZONE_CONFLICT = "NoVolumeZoneConflict"
ERR_NODE_SELECTOR_NOT_MATCH = "MatchNodeSelector"
ERR_POD_AFFINITY_NOT_MATCH = "MatchInterPodAffinity"
ERR_POD_AFFINITY_RULES_NOT_MATCH = "PodAffinityRulesNotMatch"
ERR_POD_ANTI_AFFINITY_RULES_NOT_MATCH = "PodAntiAffinityRulesNotMatch"
ERR_EXISTING_PODS_ANTI_AFFINITY_RULES_NOT_MATCH = "ExistingPodsAntiAffinityRulesNotMatch"
ERR_TAINTS_TOLERATIONS_NOT_MATCH = "PodToleratesNodeTaints"
ERR_POD_NOT_MATCH_HOST_NAME = "HostName"
ERR_POD_NOT_FITS_HOST_PORTS = "PodFitsHostPorts"
ERR_NODE_LABEL_PRESENCE_VIOLATED = "CheckNodeLabelPresence"
ERR_SERVICE_AFFINITY_VIOLATED = "CheckServiceAffinity"
ERR_MAX_VOLUME_COUNT_EXCEEDED = "MaxVolumeCount"
ERR_NODE_UNDER_MEMORY_PRESSURE = "NodeUnderMemoryPressure"
ERR_NODE_UNDER_DISK_PRESSURE = "NodeUnderDiskPressure"
ERR_NODE_OUT_OF_DISK = "NodeOutOfDisk"
ERR_NODE_NOT_READY = "NodeNotReady"
ERR_NODE_NETWORK_UNAVAILABLE = "NodeNetworkUnavailable"
ERR_NODE_UNSCHEDULABLE = "NodeUnschedulable"
ERR_NODE_UNKNOWN_CONDITION = "NodeUnknownCondition"
ERR_VOLUME_NODE_CONFLICT = "VolumeNodeAffinityConflict"
ERR_VOLUME_BIND_CONFLICT = "VolumeBindingNoMatch"

# PodFitsResources checks these whatever the pod asks (an overcommitted node fails a pod that
# requests none of it), then every scalar (extended or hugepages-*) resource it requests. The
# legacy in-kubelet accelerator is alpha.kubernetes.io/amd-gpu here (kubelet/gpu_legacy.py), in
# the slot the reference gives ResourceNvidiaGPU, which is kept for its tables.
FIXED_RESOURCES = ("cpu", "memory", "alpha.kubernetes.io/nvidia-gpu", "alpha.kubernetes.io/amd-gpu", "ephemeral-storage")


def is_scalar_resource(name: str) -> bool:
    """v1helper.IsScalarResourceName: an extended resource or hugepages-<size>."""
    return is_extended_resource_name(name) or name.startswith("hugepages-")


_NOTHING = object()     # a node selector term that matches no node


def _term_selector_or_nothing(exprs):
    """NodeSelectorRequirementsAsSelector: no requirements select nothing; a bad one is an error."""
    if not exprs:
        return _NOTHING
    try:
        return node_requirements_as_selector(exprs)
    except SelectorError:
        return None


class PodInfo:
    def __init__(self, pod: dict):
        from ..kubelet.qos import BEST_EFFORT, pod_qos
        self.pod = pod
        self.key = m.key_of(pod)
        spec = pod.get("spec") or {}
        self.spec = spec
        self.requests = pod_requests(pod)
        self.ports = pod_host_ports(pod)
        self.node_selector = spec.get("nodeSelector") or {}
        na = ((spec.get("affinity") or {}).get("nodeAffinity") or {})
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
        # None: no required node affinity (every node); else the ORed terms (_NOTHING / None =
        # parse error entries), an empty list matching no node (predicates.go:715-720)
        self.required_terms = None if req is None else [_term_selector_or_nothing(t.get("matchExpressions"))
                                                        for t in req.get("nodeSelectorTerms") or []]
        self.preferred_terms = []
        for t in na.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
            try:
                self.preferred_terms.append((int(t.get("weight", 0)), node_requirements_as_selector(
                    (t.get("preference") or {}).get("matchExpressions"))))
            except SelectorError:
                pass
        self.tolerations = spec.get("tolerations") or []
        self.priority = int(spec.get("priority") or 0)
        self.qos = (pod.get("status") or {}).get("qosClass") or ""
        # GetPodQOS == BestEffort: no cpu/memory request or limit (the full QoS parse only when
        # some container names one)
        self.best_effort = not any(k in ((c.get("resources") or {}).get(part) or {})
                                   for c in (spec.get("containers") or []) + (spec.get("initContainers") or [])
                                   for part in ("requests", "limits") for k in ("cpu", "memory")) \
            or pod_qos(pod) == BEST_EFFORT
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
    """PodFitsResources (predicates.go:630-687)."""
    alloc, used = ni.allocatable, ni.requested
    reasons = []
    if len(ni.pods) + 1 > alloc.get("pods", 0):
        reasons.append("Insufficient pods")
    req = pi.requests
    scalars = [k for k in req if is_scalar_resource(k)]
    if not scalars and not any(req.get(k, 0) for k in FIXED_RESOURCES):
        return (not reasons), reasons
    for k in FIXED_RESOURCES:
        if alloc.get(k, 0) < req.get(k, 0) + used.get(k, 0):
            reasons.append(f"Insufficient {k}")
    for k in scalars:
        if alloc.get(k, 0) < req[k] + used.get(k, 0):
            reasons.append(f"Insufficient {k}")
    return (not reasons), reasons


def pod_fits_host(pi, ni, ctx=None):
    nn = pi.spec.get("nodeName")
    if nn and nn != ni.name:
        return _fail(ERR_POD_NOT_MATCH_HOST_NAME)
    return OK


def ports_conflict(existing, wanted) -> bool:
    """portsConflict: same port and protocol, and the same host IP or either 0.0.0.0."""
    for hp in wanted:
        for used in existing:
            if used[2] == hp[2] and used[1] == hp[1] and (used[0] == hp[0] or "0.0.0.0" in (used[0], hp[0])):
                return True
    return False


def pod_fits_host_ports(pi, ni, ctx=None):
    if pi.ports and ports_conflict(ni.ports, pi.ports):
        return _fail(ERR_POD_NOT_FITS_HOST_PORTS)
    return OK


def pod_matches_node_labels(pi, labels) -> bool:
    """podMatchesNodeLabels (predicates.go:706-749): nodeSelector AND the required node
    affinity terms (ORed; none, or a term without requirements, matches no node)."""
    for k, v in pi.node_selector.items():
        if labels.get(k) != v:
            return False
    if pi.required_terms is None:
        return True
    for sel in pi.required_terms:
        if sel is None:
            return False            # a requirement that does not parse ends the search
        if sel is not _NOTHING and sel.matches(labels):
            return True
    return False


def pod_match_node_selector(pi, ni, ctx=None):
    return OK if pod_matches_node_labels(pi, ni.labels) else _fail(ERR_NODE_SELECTOR_NOT_MATCH)


def general_predicates(pi, ni, ctx=None):
    """GeneralPredicates = PodFitsResources + PodFitsHost + PodFitsHostPorts + PodMatchNodeSelector,
    every failure reported (predicates.go:965-1029)."""
    reasons = []
    for p in (pod_fits_resources, pod_fits_host, pod_fits_host_ports, pod_match_node_selector):
        ok, r = p(pi, ni, ctx)
        reasons += r
    return (not reasons), reasons


def pod_tolerates_node_taints(pi, ni, ctx=None):
    t = find_untolerated_taint(ni.taints, pi.tolerations, ("NoSchedule", "NoExecute"))
    if t:
        return _fail(ERR_TAINTS_TOLERATIONS_NOT_MATCH)
    return OK


def pod_tolerates_node_no_execute_taints(pi, ni, ctx=None):
    if find_untolerated_taint(ni.taints, pi.tolerations, ("NoExecute",)):
        return _fail(ERR_TAINTS_TOLERATIONS_NOT_MATCH)
    return OK


def check_node_condition(pi, ni, ctx=None):
    """CheckNodeConditionPredicate (predicates.go:1414-1441): every offending condition present
    is a reason (a node that reports no Ready condition is not excluded here)."""
    node = ni.node
    if node is None:
        return _fail(ERR_NODE_UNKNOWN_CONDITION)
    reasons = []
    for c in (node.get("status") or {}).get("conditions") or []:
        t, st = c.get("type"), c.get("status")
        if t == "Ready" and st != "True":
            reasons.append(ERR_NODE_NOT_READY)
        elif t == "OutOfDisk" and st != "False":
            reasons.append(ERR_NODE_OUT_OF_DISK)
        elif t == "NetworkUnavailable" and st != "False":
            reasons.append(ERR_NODE_NETWORK_UNAVAILABLE)
    if (node.get("spec") or {}).get("unschedulable"):
        reasons.append(ERR_NODE_UNSCHEDULABLE)
    return (not reasons), reasons


def check_node_memory_pressure(pi, ni, ctx=None):
    if not pi.best_effort:
        return OK
    c = get_condition(ni.node or {}, "MemoryPressure")
    if c is not None and c.get("status") == "True":
        return _fail(ERR_NODE_UNDER_MEMORY_PRESSURE)
    return OK


def check_node_disk_pressure(pi, ni, ctx=None):
    c = get_condition(ni.node or {}, "DiskPressure")
    if c is not None and c.get("status") == "True":
        return _fail(ERR_NODE_UNDER_DISK_PRESSURE)
    return OK


def is_volume_conflict(v: dict, other_pod: dict) -> bool:
    """isVolumeConflict (predicates.go:146-191): the same GCE PD, iSCSI IQN or RBD image (an
    overlapping Ceph monitor, same pool and image) may be shared only when every user mounts it
    read-only; an AWS EBS volume attaches to one instance, so never twice."""
    gce, ebs, iscsi, rbd = v.get("gcePersistentDisk"), v.get("awsElasticBlockStore"), v.get("iscsi"), v.get("rbd")
    if not (gce or ebs or iscsi or rbd):
        return False
    for ev in (other_pod.get("spec") or {}).get("volumes") or []:
        e = ev.get("gcePersistentDisk")
        if gce and e and gce.get("pdName") == e.get("pdName") and not (gce.get("readOnly") and e.get("readOnly")):
            return True
        e = ev.get("awsElasticBlockStore")
        if ebs and e and ebs.get("volumeID") == e.get("volumeID"):
            return True
        e = ev.get("iscsi")
        if iscsi and e and iscsi.get("iqn") == e.get("iqn") and not (iscsi.get("readOnly") and e.get("readOnly")):
            return True
        e = ev.get("rbd")
        if rbd and e and set(rbd.get("monitors") or []) & set(e.get("monitors") or []) and \
                rbd.get("pool", "rbd") == e.get("pool", "rbd") and rbd.get("image") == e.get("image") and \
                not (rbd.get("readOnly") and e.get("readOnly")):
            return True
    return False


def no_disk_conflict(pi, ni, ctx=None):
    vols = pi.spec.get("volumes") or []
    if not vols:
        return OK
    for v in vols:
        for p in ni.pods.values():
            if is_volume_conflict(v, p):
                return _fail(ERR_DISK_CONFLICT)
    return OK


def _topology_value(ni, key):
    return ni.labels.get(key) if key else None


def _same_topology(a, b, key) -> bool:
    """NodesHaveSameTopologyKey: both nodes carry the label, with the same value."""
    if not key:
        return False
    va, vb = a.labels.get(key), b.labels.get(key)
    return va is not None and vb is not None and va == vb


def _term_selector(term):
    return selector_from_label_selector(term.get("labelSelector"))


def _term_namespaces(term, pod):
    return set(term.get("namespaces") or [m.namespace_of(pod)])


def _term_matches(term, owner_pod, pod) -> bool:
    """PodMatchesTermsNamespaceAndSelector for `pod` against `owner_pod`'s term."""
    try:
        return m.namespace_of(pod) in _term_namespaces(term, owner_pod) and _term_selector(term).matches(m.labels_of(pod))
    except SelectorError:
        return False


def _all_pods(ni, ctx):
    """(pod, its NodeInfo) over the cluster the context describes (or just this node)."""
    for other in (ctx.nodes if ctx is not None else [ni]):
        for p in other.pods.values():
            yield p, other


def _existing_anti_affinity_ok(pi, ni, ctx) -> bool:
    """satisfiesExistingPodsAntiAffinity (:1238-1283): no placed pod's required anti-affinity
    term selects this pod within the topology it shares with the candidate node."""
    for p, other in _all_pods(ni, ctx):
        terms = (((p.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {}).get(
            "requiredDuringSchedulingIgnoredDuringExecution") or []
        for term in terms:
            if not _term_matches(term, p, pi.pod):
                continue
            if not term.get("topologyKey") or _same_topology(ni, other, term.get("topologyKey")):
                return False
    return True


def _any_pod_matches_term(pi, ni, ctx, term) -> tuple[bool, bool]:
    """anyPodMatchesPodAffinityTerm (:1080-1104): (a matching pod shares the topology, a
    matching pod exists anywhere)."""
    exists = False
    for p, other in _all_pods(ni, ctx):
        if _term_matches(term, pi.pod, p):
            exists = True
            if _same_topology(ni, other, term.get("topologyKey")):
                return True, True
    return False, exists


def match_inter_pod_affinity(pi, ni, ctx=None):
    """InterPodAffinityMatches (predicates.go:1047-1074): reasons are MatchInterPodAffinity plus
    the specific rule that failed."""
    if ctx is None and not (pi.pod_affinity or pi.pod_anti_affinity):
        return OK       # the context-free (fit index) path runs only while no placed pod has anti-affinity
    if ni.node is None:
        return _fail(ERR_POD_AFFINITY_NOT_MATCH, ERR_EXISTING_PODS_ANTI_AFFINITY_RULES_NOT_MATCH)
    if (ctx is None or ctx.any_anti_affinity) and not _existing_anti_affinity_ok(pi, ni, ctx):
        return _fail(ERR_POD_AFFINITY_NOT_MATCH, ERR_EXISTING_PODS_ANTI_AFFINITY_RULES_NOT_MATCH)
    if not (pi.pod_affinity or pi.pod_anti_affinity):
        return OK
    for term in pi.pod_affinity:
        if not term.get("topologyKey"):
            return _fail(ERR_POD_AFFINITY_NOT_MATCH, ERR_POD_AFFINITY_RULES_NOT_MATCH)
        matches, exists = _any_pod_matches_term(pi, ni, ctx, term)
        if not matches:
            # a term that selects the pod itself, with no such pod anywhere yet, is waived so the
            # first pod of a group can schedule (:1304-1326)
            if exists or not _term_matches(term, pi.pod, pi.pod):
                return _fail(ERR_POD_AFFINITY_NOT_MATCH, ERR_POD_AFFINITY_RULES_NOT_MATCH)
    for term in pi.pod_anti_affinity:
        if not term.get("topologyKey") or _any_pod_matches_term(pi, ni, ctx, term)[0]:
            return _fail(ERR_POD_AFFINITY_NOT_MATCH, ERR_POD_ANTI_AFFINITY_RULES_NOT_MATCH)
    return OK


def always_fit(pi, ni, ctx=None):
    return OK


def no_volume_zone_conflict(pi, ni, ctx=None):
    """VolumeZoneChecker (predicates.go:463-557): on a node with zone/region labels every bound
    PV's zone labels must admit the node's; a claim that is missing, or unbound without a
    WaitForFirstConsumer class, cannot be placed (the reference returns an error)."""
    vol = getattr(pi, "vol", None)
    if vol is None or not pi.spec.get("volumes"):
        return OK
    from .volumes import REGION, ZONE, no_volume_zone_conflict as zc
    if ZONE not in ni.labels and REGION not in ni.labels:
        return OK
    if vol.missing:
        return _fail(f'PersistentVolumeClaim was not found: "{vol.missing[0]}"')
    if vol.unbound:
        return _fail(f'PersistentVolumeClaim is not bound: "{vol.unbound[0]}"')
    return OK if zc(vol.bound, ni.labels) else _fail(ERR_VOLUME_ZONE_CONFLICT)


def pd_volume_ids(pod: dict, kind: str, lister) -> set:
    """MaxPDVolumeCountChecker.filterVolumes (predicates.go:286-338): the ids of `kind` disks a
    pod uses, inline or through a bound claim; a claim whose PVC or PV cannot be resolved, or
    that is unbound, counts as one disk under a placeholder id (it may still hold one)."""
    from .volumes import MAX_PD
    idk = MAX_PD[kind][0]
    ns = m.namespace_of(pod)
    out = set()
    for v in (pod.get("spec") or {}).get("volumes") or []:
        if kind in v:
            out.add(v[kind].get(idk))
            continue
        ref = v.get("persistentVolumeClaim")
        if ref is None:
            continue
        name = ref.get("claimName") or ""
        placeholder = f"\0pvc:{ns}/{name}"
        pvc = lister.pvc(ns, name) if lister is not None and name else None
        pv_name = ((pvc or {}).get("spec") or {}).get("volumeName")
        pv = lister.pv(pv_name) if pvc is not None and pv_name else None
        if pv is None:
            out.add(placeholder)
        elif kind in (pv.get("spec") or {}):
            out.add(pv["spec"][kind].get(idk))
    return out


def _max_pd(kind):
    def pred(pi, ni, ctx=None):
        from .volumes import max_pd_limit
        if not pi.spec.get("volumes"):
            return OK
        lister = getattr(pi, "lister", None)
        mine = pd_volume_ids(pi.pod, kind, lister)
        if not mine:
            return OK             # the pod adds no such disk
        have = set()
        for p in ni.pods.values():
            have |= pd_volume_ids(p, kind, lister)
        if len(have) + len(mine - have) > max_pd_limit(kind):
            return _fail(ERR_MAX_VOLUME_COUNT_EXCEEDED)
        return OK
    pred.__name__ = f"max_{kind}_count"
    return pred


def check_volume_binding(pi, ni, ctx=None):
    vol = getattr(pi, "vol", None)
    if vol is None or not getattr(pi, "volume_scheduling", False):
        return OK
    from .volumes import match_delayed, pv_node_affinity_ok
    if vol.missing:       # FindPodVolumes cannot read the claim: an error in the reference
        return _fail(f'persistentvolumeclaim "{vol.missing[0]}" not found')
    if vol.unbound:
        return _fail("pod has unbound PersistentVolumeClaims")
    reasons = []
    for pvc, pv in vol.bound:
        if not pv_node_affinity_ok(pv, ni.labels):
            reasons.append(ERR_VOLUME_NODE_CONFLICT)
            break
    if vol.delayed and match_delayed(vol.delayed, pi.lister, ni.labels) is None:
        reasons.append(ERR_VOLUME_BIND_CONFLICT)
    if reasons:
        return False, reasons
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
    "PodToleratesNodeNoExecuteTaints": pod_tolerates_node_no_execute_taints,
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
