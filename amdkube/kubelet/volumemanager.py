"""Kubelet volume manager (pkg/kubelet/volumemanager: desired/actual state of world,
populator, reconciler, WaitForAttachAndMount, reconstruction).

* Desired state: every admitted, non-terminal pod's volumes resolved to volume.Spec (a
  persistentVolumeClaim becomes its bound PersistentVolume, with the claim's readOnly), each
  with its plugin and unique volume name (attachable volumes are shared node-wide).
* Actual state: attached/device-mounted volumes and per-pod mounts.
* Reconciler (woken by pod changes, else every `period`): (1) tears down pod mounts that are no
  longer desired; (2) for desired volumes — attachable ones must first be attached: by the
  attach/detach controller (the volume appears in node.status.volumesAttached; default, as
  --enable-controller-attach-detach) or by the kubelet itself — then WaitForAttach, MountDevice
  at the plugin's global path once, then SetUp per pod; volumes whose plugin requires remount
  (secret, configMap, downwardAPI, projected) are set up again once their content is older than
  `remount_period` (the reference re-renders on its periodic pod sync) so it follows the API
  objects; (3) unmounts the device and (kubelet-managed attach) detaches volumes no pod
  wants any more.
* `wait_for_attach_and_mount(pod)` blocks the pod's sync until all its volumes are mounted or
  the timeout expires (then: "timeout expired waiting for volumes to attach or mount for pod
  ...: unmounted volumes=[...]", surfaced as a FailedMount event).
* Reconstruction: on start, volume directories found under pods/<uid>/volumes/<plugin>/<name>
  are entered as mounted so the reconciler tears down those of pods that no longer exist
  (reconciler.go sync / reconstructVolume).
* `volumes_in_use()` feeds node.status.volumesInUse, which the attach/detach controller
  consults before detaching (safe detach).

A pod without volumes costs nothing: no state, no reconcile work, no wait.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time
from dataclasses import dataclass, field

from ..api import meta as m
from ..volume import PluginMgr, Spec, VolumeError, unescape_plugin_name
from ..utils import wait_event

log = logging.getLogger("amdkube.kubelet.volumemanager")


@dataclass
class DesiredVolume:
    outer: str              # the pod's volume name
    unique: str
    plugin: object
    spec: Spec


@dataclass
class MountedVolume:
    uid: str
    outer: str
    unique: str
    plugin: object
    dir: str                # pods/<uid>/volumes/<plugin>/<outer>
    path: str               # what containers bind (set_up's answer)
    spec: Spec | None = None
    reconstructed: bool = False
    at: float = 0.0         # monotonic time of the last set-up


@dataclass
class AttachedVolume:
    unique: str
    plugin: object
    spec: Spec
    device: str = ""
    device_mount: str = ""
    globally_mounted: bool = False
    pods: set = field(default_factory=set)


def subpath(volume_path: str, sub: str, what: str) -> str:
    """volumeMounts[].subPath: relative, no '..' escape, created if missing, and (after symlink
    resolution) still inside the volume — the 1.9.4 subPath hardening."""
    if not sub:
        return volume_path
    if os.path.isabs(sub) or any(p == ".." for p in sub.split("/")):
        raise VolumeError(f"{what}: subPath {sub!r} must be a relative path without '..'")
    full = os.path.join(volume_path, sub)
    if not os.path.lexists(full):
        os.makedirs(full, mode=0o750, exist_ok=True)
    root = os.path.realpath(volume_path)
    real = os.path.realpath(full)
    if real != root and not real.startswith(root.rstrip("/") + "/"):
        raise VolumeError(f"{what}: subPath {sub!r} resolves outside the volume")
    return full


class VolumeManager:
    def __init__(self, kubelet, plugins: PluginMgr, controller_attach_detach: bool = True, period: float = 2.0,
                 wait_timeout: float = 120.0, remount_period: float = 60.0):
        self.k = kubelet
        self.mgr = plugins
        self.controller_attach_detach = controller_attach_detach
        self.period = period
        self.wait_timeout = wait_timeout
        self.remount_period = remount_period     # how stale rendered content (secret, configMap, ...) may get
        self.desired: dict[str, dict[str, DesiredVolume]] = {}
        self.pods: dict[str, dict] = {}
        self.mounted: dict[tuple[str, str], MountedVolume] = {}
        self.attached: dict[str, AttachedVolume] = {}
        self.errors: dict[tuple[str, str], str] = {}
        self._reported: dict[tuple[str, str], str] = {}
        self._wake = asyncio.Event()
        self._changed = asyncio.Condition()
        self._task = None
        self._lock = asyncio.Lock()
        self.passes = 0

    # ------------------------------------------------------------ populator
    async def _resolve(self, pod: dict) -> dict[str, DesiredVolume]:
        ns, uid = m.namespace_of(pod), m.uid_of(pod)
        out = {}
        for v in (pod.get("spec") or {}).get("volumes") or []:
            if "persistentVolumeClaim" in v:
                ref = v["persistentVolumeClaim"]
                claim = ref.get("claimName", "")
                pvc = await self.k.client.get_or_none("persistentvolumeclaims", claim, ns)
                if pvc is None:
                    raise VolumeError(f"volume {v['name']}: PersistentVolumeClaim {claim!r} not found")
                pv_name = (pvc.get("spec") or {}).get("volumeName")
                if not pv_name or (pvc.get("status") or {}).get("phase") != "Bound":
                    raise VolumeError(f"volume {v['name']}: PersistentVolumeClaim {claim} is not bound")
                pv = await self.k.client.get_or_none("persistentvolumes", pv_name)
                if pv is None:
                    raise VolumeError(f"volume {v['name']}: PersistentVolume {pv_name} not found")
                if (((pv.get("spec") or {}).get("claimRef")) or {}).get("uid") not in (None, m.uid_of(pvc)):
                    raise VolumeError(f"volume {v['name']}: PersistentVolume {pv_name} is bound to another claim")
                spec = Spec(pv=pv, read_only=bool(ref.get("readOnly")))
            else:
                spec = Spec(volume=v)
            plugin = self.mgr.find_by_spec(spec)
            out[v["name"]] = DesiredVolume(v["name"], plugin.unique_name(spec, uid), plugin, spec)
        return out

    async def add_pod(self, pod: dict):
        uid = m.uid_of(pod)
        self.pods[uid] = pod
        if not (pod.get("spec") or {}).get("volumes"):
            self.desired[uid] = {}
            return
        if uid in self.desired and all(k in self.desired[uid] for k in (v["name"] for v in pod["spec"]["volumes"])):
            return
        self.desired[uid] = await self._resolve(pod)
        self._wake.set()
        if any(dv.plugin.attachable for dv in self.desired[uid].values()):
            dirty = getattr(self.k, "_node_dirty", None)
            if dirty is not None:
                dirty.set()          # publish volumesInUse

    def remove_pod(self, uid: str):
        gone = self.desired.pop(uid, None)
        self.pods.pop(uid, None)
        if gone or any(k[0] == uid for k in self.mounted):
            self._wake.set()
        if gone and any(dv.plugin.attachable for dv in gone.values()):
            dirty = getattr(self.k, "_node_dirty", None)
            if dirty is not None:
                dirty.set()

    # ---------------------------------------------------------------- queries
    def mounted_volumes(self, uid: str) -> dict[str, str]:
        return {mv.outer: mv.path for k, mv in self.mounted.items() if k[0] == uid and not mv.reconstructed}

    def volumes_in_use(self) -> list[str]:
        return sorted({dv.unique for vols in self.desired.values() for dv in vols.values() if dv.plugin.attachable})

    def has_mounts(self, uid: str) -> bool:
        """Anything of the pod still set up (or found on disk and not yet torn down)."""
        return any(k[0] == uid for k in self.mounted)

    async def wait_for_attach_and_mount(self, pod: dict, timeout: float | None = None) -> dict[str, str]:
        await self.add_pod(pod)
        uid = m.uid_of(pod)
        want = self.desired.get(uid) or {}
        if not want:
            return {}
        self._wake.set()
        deadline = time.monotonic() + (self.wait_timeout if timeout is None else timeout)
        async with self._changed:
            while True:
                missing = [o for o in want if (uid, o) not in self.mounted]
                if not missing:
                    return self.mounted_volumes(uid)
                rem = deadline - time.monotonic()
                if rem <= 0:
                    errs = "; ".join(f"{o}: {self.errors[(uid, o)]}" for o in missing if (uid, o) in self.errors)
                    raise VolumeError(f"timeout expired waiting for volumes to attach or mount for pod "
                                      f"{m.namespace_of(pod)}/{m.name_of(pod)}. list of unmounted volumes={sorted(missing)}"
                                      + (f": {errs}" if errs else ""))
                try:
                    await asyncio.wait_for(self._changed.wait(), rem)
                except asyncio.TimeoutError:
                    pass

    # -------------------------------------------------------------- reconciler
    async def _node_attached(self) -> set[str]:
        """node.status.volumesAttached as the attach/detach controller last wrote it (a fresh
        read: the controller patches the node behind the kubelet's back)."""
        node = None
        try:
            node = await self.k.client.get_or_none("nodes", self.k.node_name)
        except Exception as e:
            log.debug("node read failed: %r", e)
        node = node or self.k.node or {}
        return {a.get("name", "") for a in (node.get("status") or {}).get("volumesAttached") or []}

    def _dir(self, uid, dv: DesiredVolume):
        """pods/<uid>/volumes/<plugin>/<spec name>: the PV's name for claims (GetPodVolumeDir
        with volumeSpec.Name()), the pod's volume name otherwise."""
        return self.mgr.host.pod_volume_dir(uid, dv.plugin.name, dv.spec.name())

    async def _notify(self):
        async with self._changed:
            self._changed.notify_all()

    def _error(self, key, msg):
        self.errors[key] = msg
        if self._reported.get(key) != msg:
            self._reported[key] = msg
            pod = self.pods.get(key[0])
            log.warning("volume %s of pod %s: %s", key[1], key[0], msg)
            if pod is not None and getattr(self.k, "recorder", None) is not None:
                self.k.recorder.event(pod, "Warning", "FailedMount", f"MountVolume.SetUp failed for volume \"{key[1]}\" : {msg}")

    async def reconcile(self):
        async with self._lock:
            await self._reconcile()
        self.passes += 1
        await self._notify()

    async def _reconcile(self):
        # (1) unmount what is no longer desired
        for key, mv in list(self.mounted.items()):
            uid, outer = key
            want = self.desired.get(uid) or {}
            if not mv.reconstructed and outer in want:
                continue
            if mv.reconstructed and any(self._dir(uid, dv) == mv.dir for dv in want.values()):
                del self.mounted[key]        # re-adopt: the set-up below re-establishes it
                continue
            try:
                await mv.plugin.tear_down(mv.dir)
            except VolumeError as e:
                self._error(key, f"UnmountVolume.TearDown failed: {e}")
                continue
            except Exception as e:      # a broken plugin must not wedge the loop
                self._error(key, f"UnmountVolume.TearDown failed: {e!r}")
                continue
            del self.mounted[key]
            self.errors.pop(key, None)
            self._reported.pop(key, None)
            if mv.unique in self.attached:
                self.attached[mv.unique].pods.discard(uid)
        # (2) attach / mount device / set up
        node_attached = None
        for uid, vols in list(self.desired.items()):
            pod = self.pods.get(uid)
            if pod is None:
                continue
            for outer, dv in vols.items():
                key = (uid, outer)
                mv = self.mounted.get(key)
                if mv is not None and not (dv.plugin.requires_remount and time.monotonic() - mv.at >= self.remount_period):
                    continue
                try:
                    dev_mount = None
                    if dv.plugin.attachable:
                        av = self.attached.get(dv.unique)
                        if av is None or not av.globally_mounted:
                            if self.controller_attach_detach:
                                if node_attached is None:
                                    node_attached = await self._node_attached()
                                if dv.unique not in node_attached:
                                    raise VolumeError(f"Volume {dv.unique} not attached to node {self.k.node_name} yet "
                                                      "(waiting for the attach/detach controller)")
                                device = ""
                            else:
                                device = await dv.plugin.attach(dv.spec, self.k.node_name)
                            device = await dv.plugin.wait_for_attach(dv.spec, device, pod, self.wait_timeout)
                            dmp = dv.plugin.device_mount_path(dv.spec)
                            if dmp:
                                await dv.plugin.mount_device(dv.spec, device, dmp)
                            av = self.attached[dv.unique] = AttachedVolume(dv.unique, dv.plugin, dv.spec, device, dmp, True)
                        dev_mount = av.device_mount or None
                        av.pods.add(uid)
                    d = self._dir(uid, dv)
                    path = await dv.plugin.set_up(dv.spec, pod, d, dev_mount,
                                                  ((pod.get("spec") or {}).get("securityContext") or {}).get("fsGroup"))
                    self.mounted[key] = MountedVolume(uid, outer, dv.unique, dv.plugin, d, path or d, dv.spec,
                                                      at=time.monotonic())
                    self.errors.pop(key, None)
                    self._reported.pop(key, None)
                except VolumeError as e:
                    self._error(key, str(e))
                except Exception as e:
                    self._error(key, repr(e))
        # (3) unmount devices / detach volumes nobody wants
        wanted = {dv.unique for vols in self.desired.values() for dv in vols.values()}
        for unique, av in list(self.attached.items()):
            if unique in wanted or any(mv.unique == unique for mv in self.mounted.values()):
                continue
            try:
                if av.globally_mounted and av.device_mount:
                    await av.plugin.unmount_device(av.device_mount)
                if not self.controller_attach_detach:
                    await av.plugin.detach(av.plugin.volume_name(av.spec), self.k.node_name)
            except Exception as e:
                log.warning("unmount device / detach of %s failed: %r", unique, e)
                continue
            del self.attached[unique]

    # ------------------------------------------------------------ lifecycle
    def reconstruct(self):
        """Volume dirs left by a previous kubelet: entered as mounted (to be torn down unless a
        pod still wants them)."""
        base = os.path.join(self.mgr.host.root_dir, "pods")
        if not os.path.isdir(base):
            return
        for uid in os.listdir(base):
            vdir = os.path.join(base, uid, "volumes")
            if not os.path.isdir(vdir):
                continue
            for pdir in os.listdir(vdir):
                try:
                    plugin = self.mgr.find_by_name(unescape_plugin_name(pdir))
                except VolumeError:
                    continue
                for outer in os.listdir(os.path.join(vdir, pdir)):
                    if ".deleting~" in outer:
                        continue
                    d = os.path.join(vdir, pdir, outer)
                    if not any(mv.dir == d for mv in self.mounted.values()):
                        self.mounted[(uid, "\0" + d)] = MountedVolume(uid, outer, f"{plugin.name}/{uid}-{outer}", plugin, d, d,
                                                                        reconstructed=True)

    async def run(self):
        while True:
            await wait_event(self._wake, self.period)
            self._wake.clear()
            if not self.desired and not self.mounted and not self.attached:
                continue
            try:
                await self.reconcile()
            except Exception as e:
                log.warning("volume reconcile failed: %r", e)

    def start(self):
        self.reconstruct()
        self._task = asyncio.create_task(self.run(), name="volume-reconciler")
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass

