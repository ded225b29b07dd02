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
  * pkg/controller/volume/attachdetach — desired vs actual attachments of attachable volumes
    per node, attached/detached through the volume plugins (amdkube/volume) and reported in
    node.status.volumesAttached; safe detach waits for node.status.volumesInUse to drop it.
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

import asyncio
import logging
import os
import shutil
import time

from ..api import meta as m
from ..api.helpers import is_pod_terminal
from ..api.labels import selector_from_label_selector
from ..api.quantity import Quantity
from .base import Controller, split_key

log = logging.getLogger("amdkube.controllers.volumes")

HOSTPATH_PROVISIONERS = ("amdkube.io/host-path", "kubernetes.io/host-path")
CINDER_PROVISIONER = "kubernetes.io/cinder"
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
        sc0 = self._class(claim_class(pvc))
        if sc0 is not None and sc0.get("volumeBindingMode") == "WaitForFirstConsumer":
            # delayed binding (VolumeScheduling): the scheduler picks the volume together with
            # the pod's node and pre-binds it (claimRef); only such a volume completes the claim
            ref = ((pv or {}).get("spec") or {}).get("claimRef") or {}
            if pv is None or ref.get("name") != name or ref.get("namespace") != ns:
                if (pvc.get("status") or {}).get("phase") != "Pending":
                    await self.client.patch("persistentvolumeclaims", name, {"status": {"phase": "Pending"}}, ns, sub="status")
                return
        if pv is None:
            sc = self._class(claim_class(pvc))
            if sc is not None and sc.get("provisioner") in HOSTPATH_PROVISIONERS:
                pv = await self._provision(pvc, sc)
            elif sc is not None and sc.get("provisioner") in self._provisioners():
                pv = await self._provision_cloud(pvc, sc, self._provisioners()[sc["provisioner"]])
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

    def _cloud_disks(self):
        """The cloud provider's block-disk service (Cinder, EBS, GCE PD, Azure disks), if any."""
        cloud = getattr(getattr(self.mgr, "opts", None), "cloud", None)
        return cloud.volumes() if cloud is not None and hasattr(cloud, "volumes") else None

    def _provisioners(self) -> dict:
        """Dynamic provisioners by StorageClass provisioner name: the cloud's disks and the
        vendor storage backends (volume/vendor.py)."""
        from ..volume.vendor import provisioners
        out = {p.provisioner: p for p in provisioners()}
        d = self._cloud_disks()
        if d is not None:
            out[d.provisioner] = d
        return out

    async def _provision_cloud(self, pvc, sc, disks):
        """The in-tree cloud provisioners (cinder_util.go, aws_util.go, gce_util.go,
        azure_provision.go CreateVolume): a disk of the claim's size in GiB, rounded up, with the
        class's parameters, tagged with the claim; the PV carries the disk's zone/region labels."""
        from ..api.quantity import parse_quantity
        size = ((pvc.get("spec") or {}).get("resources") or {}).get("requests", {}).get("storage", "1Gi")
        gib = max(1, -(-int(parse_quantity(size).value()) // (1 << 30)))
        params = sc.get("parameters") or {}
        name = f"pvc-{m.uid_of(pvc)}"
        tags = {"kubernetes.io/created-for/pvc/namespace": m.namespace_of(pvc),
                "kubernetes.io/created-for/pvc/name": m.name_of(pvc), "kubernetes.io/created-for/pv/name": name}
        if hasattr(disks, "aprovision"):
            source, labels = await disks.aprovision(self.client, name, gib, params, tags, m.name_of(pvc))
        else:
            source, labels = await asyncio.to_thread(disks.provision, name, gib, params, tags, m.name_of(pvc))
        pv = {"apiVersion": "v1", "kind": "PersistentVolume",
              "metadata": {"name": name, "labels": {k: v for k, v in labels.items() if v},
                           "annotations": {"pv.kubernetes.io/provisioned-by": disks.provisioner}},
              "spec": {"capacity": {"storage": f"{gib}Gi"},
                       "accessModes": (pvc.get("spec") or {}).get("accessModes") or ["ReadWriteOnce"],
                       "persistentVolumeReclaimPolicy": sc.get("reclaimPolicy", "Delete"),
                       "storageClassName": m.name_of(sc), disks.source_key: source,
                       "claimRef": {"kind": "PersistentVolumeClaim", "namespace": m.namespace_of(pvc), "name": m.name_of(pvc),
                                    "uid": m.uid_of(pvc), "apiVersion": "v1"}}}
        try:
            return await self.client.create(pv)
        except m.StatusError as e:
            if m.is_already_exists(e):
                return await self.client.get("persistentvolumes", name)
            raise

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
            elif (disks := self._provisioners().get(m.annotations_of(pv).get("pv.kubernetes.io/provisioned-by"))) is not None \
                    and ps.get(disks.source_key):
                if hasattr(disks, "adelete"):
                    await disks.adelete(self.client, ps[disks.source_key])
                else:
                    await asyncio.to_thread(disks.delete_source, ps[disks.source_key])   # fails while attached: retried
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
    """pkg/controller/volume/attachdetach: for every node, the attachable volumes of its
    scheduled, non-terminal pods (desired) against what is attached (actual, seeded from
    node.status.volumesAttached at start). Attach/detach run through the volume plugins (CSI:
    a VolumeAttachment the driver's attacher fulfils; FlexVolume: the driver's attach/detach;
    iSCSI/FC/RBD: no-op attach, the node logs in) as background operations, one per volume.
    A volume still in node.status.volumesInUse is not detached until the kubelet unmounted it
    or `max_wait_unmount` (6 min) passed. node.status.volumesAttached lists {name: unique
    volume name, devicePath}; non-attachable volumes (hostPath, nfs, ...) never appear."""
    name = "attachdetach"
    workers = 1

    def __init__(self, mgr, plugins=None, max_wait_unmount: float = 360.0):
        super().__init__(mgr)
        self._plugins = plugins
        self.max_wait_unmount = max_wait_unmount
        self.attached: dict[str, dict[str, str]] = {}        # node -> unique -> devicePath
        self._pending: set[tuple[str, str]] = set()
        self._detach_wait: dict[tuple[str, str], float] = {}
        self._ops: set[asyncio.Task] = set()
        self._seeded = False

    @property
    def plugins(self):
        if self._plugins is None:
            from ..volume import NoopMounter, PluginMgr, VolumeHost, default_plugins
            self._plugins = PluginMgr(default_plugins(), VolumeHost("/var/lib/kubelet", client=self.client, mounter=NoopMounter()))
            self._plugins.host.cloud = getattr(getattr(self.mgr, "opts", None), "cloud", None)
        return self._plugins

    def setup(self):
        f = self.mgr.factory
        self.pod_inf = self.mgr.pods
        self.pvc_inf = f.informer("persistentvolumeclaims")
        self.pv_inf = f.informer("persistentvolumes")
        self.node_inf = self.mgr.nodes
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)
        self.node_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))

    def _pod(self, pod):
        node = (pod.get("spec") or {}).get("nodeName")
        if node:
            self.enqueue(node)

    def _desired(self, node: str) -> dict:
        from ..volume import Spec, VolumeError
        out = {}
        for p in self.pod_inf.list():
            if (p.get("spec") or {}).get("nodeName") != node or is_pod_terminal(p):
                continue
            for v in (p.get("spec") or {}).get("volumes") or []:
                if "persistentVolumeClaim" in v:
                    pvc = self.pvc_inf.get(f"{m.namespace_of(p)}/{v['persistentVolumeClaim'].get('claimName', '')}")
                    pv = self.pv_inf.get(((pvc or {}).get("spec") or {}).get("volumeName") or "")
                    if pv is None:
                        continue
                    spec = Spec(pv=pv, read_only=bool(v["persistentVolumeClaim"].get("readOnly")))
                else:
                    spec = Spec(volume=v)
                try:
                    plugin = self.plugins.find_by_spec(spec)
                except VolumeError:
                    continue
                if plugin.attachable:
                    out[plugin.unique_name(spec, m.uid_of(p))] = (plugin, spec)
        return out

    def _seed(self):
        """populateActualStateOfWorld: what the nodes say is attached."""
        for n in self.node_inf.list():
            att = {a.get("name", ""): a.get("devicePath", "") for a in (n.get("status") or {}).get("volumesAttached") or []}
            if att:
                self.attached.setdefault(m.name_of(n), {}).update(att)
        self._seeded = True

    def _op(self, node, unique, coro):
        self._pending.add((node, unique))

        async def run():
            try:
                await coro
            except Exception as e:
                log.warning("attachdetach: %s on %s: %r", unique, node, e)
                self.queue.add_after(node, 2.0)
            finally:
                self._pending.discard((node, unique))
                self.enqueue(node)
        t = asyncio.create_task(run(), name=f"attachdetach-{unique}")
        self._ops.add(t)
        t.add_done_callback(self._ops.discard)

    async def _attach(self, node, unique, plugin, spec):
        device = await plugin.attach(spec, node)
        self.attached.setdefault(node, {})[unique] = device or ""

    async def _detach(self, node, unique):
        from ..volume import VolumeError
        plugin_name, _, vol = unique.rpartition("/")
        try:
            plugin = self.plugins.find_by_name(plugin_name)
        except VolumeError:
            plugin = None
        if plugin is not None:
            await plugin.detach(vol, node)
        self.attached.get(node, {}).pop(unique, None)
        self._detach_wait.pop((node, unique), None)

    async def sync(self, key):
        _, node = split_key(key)
        if not self._seeded:
            self._seed()
        n = self.node_inf.get(node)
        desired = self._desired(node) if n is not None else {}
        actual = self.attached.setdefault(node, {})
        for unique, (plugin, spec) in desired.items():
            if unique not in actual and (node, unique) not in self._pending:
                self._op(node, unique, self._attach(node, unique, plugin, spec))
        in_use = set(((n or {}).get("status") or {}).get("volumesInUse") or [])
        now = time.monotonic()
        for unique in list(actual):
            if unique in desired or (node, unique) in self._pending:
                continue
            if unique in in_use:
                first = self._detach_wait.setdefault((node, unique), now)
                if now - first < self.max_wait_unmount:
                    self.queue.add_after(node, 1.0)    # the kubelet has not unmounted it yet
                    continue
            self._op(node, unique, self._detach(node, unique))
        if n is None:
            return
        want = [{"name": u, "devicePath": d} for u, d in sorted(actual.items())]
        if ((n.get("status") or {}).get("volumesAttached") or []) != want:
            await self.client.patch("nodes", node, {"status": {"volumesAttached": want or None}}, sub="status")

    async def stop(self):
        for t in list(self._ops):
            t.cancel()
        await super().stop()


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
