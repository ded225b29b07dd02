"""Volume-aware scheduling (plugin/pkg/scheduler/algorithm/predicates/predicates.go
VolumeZoneChecker, MaxPDVolumeCountChecker, NewVolumeBindingPredicate; pkg/controller/volume/
persistentvolume/scheduler_binder.go — the alpha VolumeScheduling feature of the reference).

* NoVolumeZoneConflict: a bound PV labelled with a zone/region (failure-domain.beta.kubernetes
  .io/zone|region; `a__b` = several) only fits nodes in one of those zones.
* Max{EBS,GCEPD,AzureDisk}VolumeCount: distinct cloud disks per node (inline and through PVs,
  the pod's plus the node's pods') stay within 39 / 16 / 16 (KUBE_MAX_PD_VOLS overrides).
* CheckVolumeBinding (VolumeScheduling gate): a bound PV's node affinity
  (volume.alpha.kubernetes.io/node-affinity) must admit the node; a claim of a StorageClass
  with volumeBindingMode WaitForFirstConsumer is matched against the available PVs whose node
  affinity admits the node — the smallest that fits, as the PV controller would — and once a
  host is chosen the scheduler pre-binds those PVs (PV.spec.claimRef) before the pod, so the PV
  controller completes the binding on the node the pod runs on. Unbound claims of
  Immediate-mode classes are not schedulable yet.
"""
from __future__ import annotations

import json
import os

from ..api import meta as m
from ..api.labels import node_requirements_as_selector
from ..api.quantity import Quantity

ZONE = "failure-domain.beta.kubernetes.io/zone"
REGION = "failure-domain.beta.kubernetes.io/region"
NODE_AFFINITY_ANN = "volume.alpha.kubernetes.io/node-affinity"
MAX_PD = {"awsElasticBlockStore": ("volumeID", 39), "gcePersistentDisk": ("pdName", 16), "azureDisk": ("diskName", 16)}


class VolumeLister:
    """PVC / PV / StorageClass lookups over the scheduler's informers (or plain dicts in tests)."""

    def __init__(self, pvcs=None, pvs=None, classes=None):
        self._pvcs, self._pvs, self._classes = pvcs, pvs, classes
        self.assumed: dict[str, str] = {}     # PV name -> claim key pre-bound by this scheduler, not yet observed

    @staticmethod
    def _get(src, key):
        if src is None:
            return None
        return src.get(key) if isinstance(src, dict) else src.get(key)

    def pvc(self, ns, name):
        return self._get(self._pvcs, f"{ns}/{name}")

    def pv(self, name):
        return self._get(self._pvs, name)

    def storage_class(self, name):
        return self._get(self._classes, name) if name else None

    def pv_list(self):
        if self._pvs is None:
            return []
        return list(self._pvs.values()) if isinstance(self._pvs, dict) else self._pvs.list()


class PodVolumes:
    __slots__ = ("sources", "bound", "delayed", "unbound", "missing")

    def __init__(self):
        self.sources: list[tuple[str, dict]] = []     # (kind, source) inline and from bound PVs
        self.bound: list[tuple[dict, dict]] = []      # (pvc, pv)
        self.delayed: list[dict] = []                 # unbound claims waiting for the first consumer
        self.unbound: list[str] = []                  # unbound claims of Immediate classes
        self.missing: list[str] = []


def claim_class(pvc) -> str:
    return (pvc.get("spec") or {}).get("storageClassName") or \
        (m.annotations_of(pvc).get("volume.beta.kubernetes.io/storage-class") or "")


def pod_volumes(pod: dict, lister: VolumeLister | None) -> PodVolumes:
    out = PodVolumes()
    ns = m.namespace_of(pod)
    for v in (pod.get("spec") or {}).get("volumes") or []:
        ref = v.get("persistentVolumeClaim")
        if ref is None:
            for k in MAX_PD:
                if k in v:
                    out.sources.append((k, v[k]))
            continue
        if lister is None:
            continue
        pvc = lister.pvc(ns, ref.get("claimName", ""))
        if pvc is None:
            out.missing.append(ref.get("claimName", ""))
            continue
        pv_name = (pvc.get("spec") or {}).get("volumeName")
        pv = lister.pv(pv_name) if pv_name else None
        if pv is not None:
            out.bound.append((pvc, pv))
            for k in MAX_PD:
                if k in (pv.get("spec") or {}):
                    out.sources.append((k, pv["spec"][k]))
            continue
        sc = lister.storage_class(claim_class(pvc))
        if sc is not None and sc.get("volumeBindingMode") == "WaitForFirstConsumer":
            out.delayed.append(pvc)
        else:
            out.unbound.append(m.name_of(pvc))
    return out


def _zones(value: str) -> set[str]:
    return {z for z in (value or "").split("__") if z}


def no_volume_zone_conflict(pv_list, node_labels: dict) -> bool:
    if ZONE not in node_labels and REGION not in node_labels:
        return True
    for pvc, pv in pv_list:
        lab = m.labels_of(pv)
        for key in (ZONE, REGION):
            want = _zones(lab.get(key, ""))
            if want and node_labels.get(key) not in want:
                return False
    return True


def max_pd_limit(kind: str) -> int:
    """getMaxVols (predicates.go:272-284): KUBE_MAX_PD_VOLS when it is a positive integer."""
    env = os.environ.get("KUBE_MAX_PD_VOLS", "")
    try:
        n = int(env)
    except ValueError:
        n = 0
    return n if n > 0 else MAX_PD[kind][1]


def pv_node_affinity_ok(pv: dict, node_labels: dict) -> bool:
    raw = m.annotations_of(pv).get(NODE_AFFINITY_ANN)
    if not raw:
        return True
    try:
        aff = json.loads(raw)
    except ValueError:
        return False
    terms = ((aff.get("requiredDuringSchedulingIgnoredDuringExecution") or {}).get("nodeSelectorTerms")) or []
    if not terms:
        return True
    return any(node_requirements_as_selector(t.get("matchExpressions")).matches(node_labels) for t in terms)


def _size(q) -> int:
    return Quantity(q).value() if q is not None else 0


def match_delayed(claims: list[dict], lister: VolumeLister, node_labels: dict) -> list[tuple[dict, dict]] | None:
    """For each delayed claim the smallest available PV of its class whose access modes and
    capacity cover it and whose node affinity admits this node; None if any claim has none."""
    taken: set[str] = set()
    out = []
    pvs = lister.pv_list()
    for pvc in claims:
        spec = pvc.get("spec") or {}
        want = _size(((spec.get("resources") or {}).get("requests") or {}).get("storage"))
        modes = set(spec.get("accessModes") or [])
        cls = claim_class(pvc)
        best = None
        for pv in pvs:
            ps = pv.get("spec") or {}
            name = m.name_of(pv)
            if name in taken or (name in lister.assumed and lister.assumed[name] != m.key_of(pvc)):
                continue
            ref = ps.get("claimRef")
            if ref and not (ref.get("namespace") == m.namespace_of(pvc) and ref.get("name") == m.name_of(pvc)):
                continue
            if (pv.get("status") or {}).get("phase", "Available") not in ("Available", "Pending") and not ref:
                continue
            if (ps.get("storageClassName") or "") != cls or not modes <= set(ps.get("accessModes") or []):
                continue
            cap = _size((ps.get("capacity") or {}).get("storage"))
            if cap < want or not pv_node_affinity_ok(pv, node_labels):
                continue
            if best is None or cap < _size(((best.get("spec") or {}).get("capacity") or {}).get("storage")):
                best = pv
        if best is None:
            return None
        taken.add(m.name_of(best))
        out.append((pvc, best))
    return out
