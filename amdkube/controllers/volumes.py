"""Persistent volumes: binder + host-path provisioner, attach/detach, expansion, protection.

Reference:
  * pkg/controller/volume/persistentvolume/pv_controller.go — syncClaim: an unbound claim
    binds the smallest Available volume with the same storage class whose access modes
    cover the claim's, whose capacity covers the request and whose labels match the
    claim's selector (index.go findBestMatchForClaim); volume.spec.claimRef and
    claim.spec.volumeName are written (annotations pv.kubernetes.io/bind-completed,
    bound-by-controller) and both go Bound. With no match and a StorageClass, the class's
    provisioner creates `pvc-<claim uid>`. syncVolume: a volume whose claim is gone is
    Released, then reclaimed per persistentVolumeReclaimPolicy (Delete removes it and its
    provisioned data; Recycle scrubs it and makes it Available again; Retain keeps it).
  * pkg/controller/volume/attachdetach — desired vs actual attachments per node from the
    scheduled pods' volumes, reported in node.status.volumesAttached (VolumeAttachment
    objects, storage.k8s.io/v1beta1, as CSI does).
  * pkg/controller/volume/expand — a claim asking for more than its bound size on a class
    with allowVolumeExpansion grows the volume and then status.capacity.
  * pkg/controller/volume/pvcprotection, pvprotection — finalizers kubernetes.io/pvc-protection
    (kept while a non-terminal pod uses the claim) and kubernetes.io/pv-protection (kept
    while the volume is Bound).

The in-tree provisioner is a host-path one, `amdkube.io/host-path` (alias
kubernetes.io/host-path), which makes a directory per volume under its root. This is local
scratch or dataset storage for GPU pods on one MI355X node.
"""
from __future__ import annotations

import os
import shutil

from ..api import meta as m
from ..api.helpers import is_pod_terminal
from ..api.labels import selector_from_label_selector
from ..api.quantity import Quantity
from .base import Controller, split_key

HOSTPATH_PROVISIONERS = ("amdkube.io/host-path", "kubernetes.io/host-path")
DEFAULT_CLASS_ANN = "storageclass.kubernetes.io/is-default-class"
PVC_FINALIZER = "kubernetes.io/pvc-protection"
PV_FINALIZER = "kubernetes.io/pv-protection"


def _size(q) -> int:
    return Quantity(q).value() if q is not None else 0


def claim_class(pvc) -> str:
    return (pvc.get("spec") or {}).get("storageClassName") or \
        (m.annotations_of(pvc).get("volume.beta.kubernetes.io/storage-class") or "")


def volume_class(pv) -> str:
    return (pv.get("spec") or {}).get("storageClassName") or \
        (m.annotations_of(pv).get("volume.beta.kubernetes.io/storage-class") or "")


def find_best_match(pvc, volumes) -> dict | None:
    spec = pvc.get("spec") or {}
    want = _size(((spec.get("resources") or {}).get("requests") or {}).get("storage"))
    modes = set(spec.get("accessModes") or [])
    sel = selector_from_label_selector(spec["selector"]) if spec.get("selector") else None
    cls = claim_class(pvc)
    best = None
    for pv in volumes:
        ps = pv.get("spec") or {}
        ref = ps.get("claimRef")
        if ref and not (ref.get("namespace") == m.namespace_of(pvc) and ref.get("name") == m.name_of(pvc)
                        and (not ref.get("uid") or ref.get("uid") == m.uid_of(pvc))):
            continue
        if (pv.get("status") or {}).get("phase", "Available") not in ("Available", "Pending", "Bound" if ref else "Available"):
            continue
        if (pv.get("metadata") or {}).get("deletionTimestamp"):
            continue
        if volume_class(pv) != cls or not modes <= set(ps.get("accessModes") or []):
            continue
        cap = _size((ps.get("capacity") or {}).get("storage"))
        if cap < want or (sel and not sel.matches(m.labels_of(pv))):
            continue
        if ref:   # pre-bound to this claim wins outright
            return pv
        if best is None or cap < _size(((best.get("spec") or {}).get("capacity") or {}).get("storage")):
            best = pv
    return best


class PersistentVolumeBinderController(Controller):
    name = "persistentvolume-binder"
    workers = 1

    def __init__(self, mgr, hostpath_root: str = "/tmp/amdkube-hostpath-pv"):
        super().__init__(mgr)
        self.root = hostpath_root

    def setup(self):
        f = self.mgr.factory
        self.pvc_inf = f.informer("persistentvolumeclaims")
        self.pv_inf = f.informer("persistentvolumes")
        self.sc_inf = f.informer("storageclasses")
        self.pvc_inf.add_handler(on_add=self._claim, on_update=lambda o, n: self._claim(n), on_delete=self._claim_gone)
        self.pv_inf.add_handler(on_add=self._vol, on_update=lambda o, n: self._vol(n))

    def _claim(self, pvc):
        self.enqueue("claim:" + m.key_of(pvc))

    def _claim_gone(self, pvc):
        for pv in self.pv_inf.list():
            ref = (pv.get("spec") or {}).get("claimRef") or {}
            if ref.get("uid") == m.uid_of(pvc):
                self.enqueue("volume:" + m.name_of(pv))

    def _vol(self, pv):
        self.enqueue("volume:" + m.name_of(pv))
        for pvc in self.pvc_inf.list():   # a new volume may satisfy a pending claim
            if (pvc.get("status") or {}).get("phase", "Pending") == "Pending":
                self.enqueue("claim:" + m.key_of(pvc))

    def _class(self, name):
        if name:
            return self.sc_inf.get(name)
        for sc in self.sc_inf.list():
            if m.annotations_of(sc).get(DEFAULT_CLASS_ANN) == "true":
                return sc
        return None

    async def sync(self, key):
        kind, _, k = key.partition(":")
        if kind == "claim":
            await self._sync_claim(k)
        else:
            await self._sync_volume(k)

    async def _sync_claim(self, key):
        pvc = self.pvc_inf.get(key)
        if pvc is None or (pvc.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec = pvc.get("spec") or {}
        if spec.get("volumeName"):
            pv = self.pv_inf.get(spec["volumeName"])
            if pv is None:
                if (pvc.get("status") or {}).get("phase") != "Lost":
                    await self.client.patch("persistentvolumeclaims", name, {"status": {"phase": "Lost"}}, ns, sub="status")
                return
            await self._finish_bind(pvc, pv)
            return
        pv = find_best_match(pvc, self.pv_inf.list())
        if pv is None:
            sc = self._class(claim_class(pvc))
            if sc is not None and sc.get("provisioner") in HOSTPATH_PROVISIONERS:
                pv = await self._provision(pvc, sc)
            else:
                if (pvc.get("status") or {}).get("phase") != "Pending":
                    await self.client.patch("persistentvolumeclaims", name, {"status": {"phase": "Pending"}}, ns, sub="status")
                return
        ref = {"kind": "PersistentVolumeClaim", "namespace": ns, "name": name, "uid": m.uid_of(pvc), "apiVersion": "v1"}
        pv = await self.client.patch("persistentvolumes", m.name_of(pv), {"spec": {"claimRef": ref}})
        await self._finish_bind(pvc, pv)

    async def _finish_bind(self, pvc, pv):
        ns, name = m.namespace_of(pvc), m.name_of(pvc)
        if (pv.get("status") or {}).get("phase") != "Bound":
            await self.client.patch("persistentvolumes", m.name_of(pv), {"status": {"phase": "Bound"}}, sub="status")
        ann = {"pv.kubernetes.io/bind-completed": "yes", "pv.kubernetes.io/bound-by-controller": "yes"}
        if (pvc.get("spec") or {}).get("volumeName") != m.name_of(pv) or any(m.annotations_of(pvc).get(k) != v for k, v in ann.items()):
            pvc = await self.client.patch("persistentvolumeclaims", name,
                                          {"metadata": {"annotations": ann}, "spec": {"volumeName": m.name_of(pv)}}, ns)
        ps = pv.get("spec") or {}
        st = {"phase": "Bound", "accessModes": ps.get("accessModes") or [], "capacity": dict(ps.get("capacity") or {})}
        if {k: (pvc.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch("persistentvolumeclaims", name, {"status": st}, ns, sub="status")

    async def _provision(self, pvc, sc):
        size = ((pvc.get("spec") or {}).get("resources") or {}).get("requests", {}).get("storage", "1Gi")
        name = f"pvc-{m.uid_of(pvc)}"
        path = os.path.join((sc.get("parameters") or {}).get("root") or self.root, name)
        os.makedirs(path, exist_ok=True)
        pv = {"apiVersion": "v1", "kind": "PersistentVolume",
              "metadata": {"name": name, "annotations": {"pv.kubernetes.io/provisioned-by": sc["provisioner"]}},
              "spec": {"capacity": {"storage": size}, "accessModes": (pvc.get("spec") or {}).get("accessModes") or ["ReadWriteOnce"],
                       "persistentVolumeReclaimPolicy": sc.get("reclaimPolicy", "Delete"),
                       "storageClassName": m.name_of(sc), "hostPath": {"path": path},
                       "claimRef": {"kind": "PersistentVolumeClaim", "namespace": m.namespace_of(pvc), "name": m.name_of(pvc),
                                    "uid": m.uid_of(pvc), "apiVersion": "v1"}}}
        try:
            return await self.client.create(pv)
        except m.StatusError as e:
            if m.is_already_exists(e):
                return await self.client.get("persistentvolumes", name)
            raise

    async def _sync_volume(self, name):
        pv = self.pv_inf.get(name)
        if pv is None:
            return
        ps, phase = pv.get("spec") or {}, (pv.get("status") or {}).get("phase")
        ref = ps.get("claimRef")
        if not ref:
            if phase not in ("Available",):
                await self.client.patch("persistentvolumes", name, {"status": {"phase": "Available"}}, sub="status")
            return
        claim = self.pvc_inf.get(f"{ref.get('namespace')}/{ref.get('name')}")
        if claim is not None and (not ref.get("uid") or m.uid_of(claim) == ref.get("uid")):
            return
        if claim is None and not ref.get("uid"):
            return   # pre-bound by the user to a claim that does not exist yet
        policy = ps.get("persistentVolumeReclaimPolicy", "Retain")
        if phase != "Released":
            await self.client.patch("persistentvolumes", name, {"status": {"phase": "Released"}}, sub="status")
        if policy == "Delete":
            if m.annotations_of(pv).get("pv.kubernetes.io/provisioned-by") in HOSTPATH_PROVISIONERS:
                shutil.rmtree((ps.get("hostPath") or {}).get("path", "") or "/nonexistent", ignore_errors=True)
            try:
                await self.client.delete("persistentvolumes", name)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise
        elif policy == "Recycle":
            p = (ps.get("hostPath") or {}).get("path")
            if p and os.path.isdir(p):
                for e in os.listdir(p):
                    q = os.path.join(p, e)
                    shutil.rmtree(q, ignore_errors=True) if os.path.isdir(q) else os.unlink(q)
            await self.client.patch("persistentvolumes", name, {"spec": {"claimRef": None}})
            await self.client.patch("persistentvolumes", name, {"status": {"phase": "Available"}}, sub="status")


def pod_claims(pod) -> list[str]:
    return [v["persistentVolumeClaim"]["claimName"] for v in (pod.get("spec") or {}).get("volumes") or []
            if (v.get("persistentVolumeClaim") or {}).get("claimName")]


class AttachDetachController(Controller):
    name = "attachdetach"
    workers = 1
    attacher = "amdkube.io/host-path"

    def setup(self):
        f = self.mgr.factory
        self.pod_inf = self.mgr.pods
        self.pvc_inf = f.informer("persistentvolumeclaims")
        self.va_inf = f.informer("volumeattachments")
        self.node_inf = self.mgr.nodes
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _pod(self, pod):
        node = (pod.get("spec") or {}).get("nodeName")
        if node:
            self.enqueue(node)

    async def sync(self, key):
        _, node = split_key(key)
        desired = {}
        for p in self.pod_inf.list():
            if (p.get("spec") or {}).get("nodeName") != node or is_pod_terminal(p):
                continue
            for c in pod_claims(p):
                pvc = self.pvc_inf.get(f"{m.namespace_of(p)}/{c}")
                pv = ((pvc or {}).get("spec") or {}).get("volumeName")
                if pv:
                    desired[f"{self.attacher.replace('/', '-').replace('.', '-')}-{pv}-{node}"] = pv
        actual = {m.name_of(v): v for v in self.va_inf.list() if (v.get("spec") or {}).get("nodeName") == node}
        for name, pv in desired.items():
            if name not in actual:
                try:
                    await self.client.create({"apiVersion": "storage.k8s.io/v1beta1", "kind": "VolumeAttachment",
                                              "metadata": {"name": name},
                                              "spec": {"attacher": self.attacher, "nodeName": node,
                                                       "source": {"persistentVolumeName": pv}}})
                except m.StatusError as e:
                    if not m.is_already_exists(e):   # the informer has not seen our own create yet
                        raise
                await self.client.patch("volumeattachments", name, {"status": {"attached": True}}, sub="status")
        for name, va in actual.items():
            if name not in desired:
                try:
                    await self.client.delete("volumeattachments", name)
                except m.StatusError as e:
                    if not m.is_not_found(e):
                        raise
        want = [{"name": f"kubernetes.io/{self.attacher}/{pv}", "devicePath": ""} for pv in sorted(set(desired.values()))]
        n = self.node_inf.get(node)
        if n is not None and ((n.get("status") or {}).get("volumesAttached") or []) != want:
            await self.client.patch("nodes", node, {"status": {"volumesAttached": want}}, sub="status")


class VolumeExpandController(Controller):
    name = "persistentvolume-expander"
    workers = 1

    def setup(self):
        f = self.mgr.factory
        self.pvc_inf = f.informer("persistentvolumeclaims")
        self.pv_inf = f.informer("persistentvolumes")
        self.sc_inf = f.informer("storageclasses")
        self.pvc_inf.add_handler(on_update=lambda o, n: self.enqueue(n))

    async def sync(self, key):
        pvc = self.pvc_inf.get(key)
        if pvc is None or (pvc.get("status") or {}).get("phase") != "Bound":
            return
        ns, name = split_key(key)
        want = ((pvc.get("spec") or {}).get("resources") or {}).get("requests", {}).get("storage")
        have = ((pvc.get("status") or {}).get("capacity") or {}).get("storage")
        if want is None or _size(want) <= _size(have):
            return
        sc = self.sc_inf.get(claim_class(pvc)) if claim_class(pvc) else None
        if sc is None or not sc.get("allowVolumeExpansion"):
            return
        pv = self.pv_inf.get((pvc.get("spec") or {}).get("volumeName", ""))
        if pv is None:
            return
        if _size(((pv.get("spec") or {}).get("capacity") or {}).get("storage")) < _size(want):
            await self.client.patch("persistentvolumes", m.name_of(pv), {"spec": {"capacity": {"storage": want}}})
        await self.client.patch("persistentvolumeclaims", name, {"status": {"capacity": {"storage": want}, "conditions": None}},
                                ns, sub="status")


class PVCProtectionController(Controller):
    name = "pvc-protection"
    workers = 1

    def setup(self):
        self.pvc_inf = self.mgr.factory.informer("persistentvolumeclaims")
        self.pod_inf = self.mgr.pods
        self.pvc_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))
        self.pod_inf.add_handler(on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _pod(self, pod):
        for c in pod_claims(pod):
            self.enqueue(f"{m.namespace_of(pod)}/{c}")

    def in_use(self, ns, name) -> bool:
        return any(m.namespace_of(p) == ns and name in pod_claims(p) and not is_pod_terminal(p) for p in self.pod_inf.list())

    async def sync(self, key):
        pvc = self.pvc_inf.get(key)
        if pvc is None:
            return
        ns, name = split_key(key)
        md = pvc.get("metadata") or {}
        fin = list(md.get("finalizers") or [])
        if not md.get("deletionTimestamp"):
            if PVC_FINALIZER not in fin:
                await self.client.patch("persistentvolumeclaims", name, {"metadata": {"finalizers": fin + [PVC_FINALIZER]}}, ns)
            return
        if PVC_FINALIZER in fin and not self.in_use(ns, name):
            await self.client.patch("persistentvolumeclaims", name,
                                    {"metadata": {"finalizers": [f for f in fin if f != PVC_FINALIZER]}}, ns)


class PVProtectionController(Controller):
    name = "pv-protection"
    workers = 1

    def setup(self):
        self.pv_inf = self.mgr.factory.informer("persistentvolumes")
        self.pv_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))

    async def sync(self, key):
        _, name = split_key(key)
        pv = self.pv_inf.get(name)
        if pv is None:
            return
        md = pv.get("metadata") or {}
        fin = list(md.get("finalizers") or [])
        if not md.get("deletionTimestamp"):
            if PV_FINALIZER not in fin:
                await self.client.patch("persistentvolumes", name, {"metadata": {"finalizers": fin + [PV_FINALIZER]}})
            return
        if PV_FINALIZER in fin and (pv.get("status") or {}).get("phase") != "Bound":
            await self.client.patch("persistentvolumes", name, {"metadata": {"finalizers": [f for f in fin if f != PV_FINALIZER]}})
