"""CSI volume plugin (pkg/volume/csi, alpha in the reference release) and an external attacher.

Kubelet side (`CSIPlugin`, PersistentVolumes with spec.csi {driver, volumeHandle, readOnly}):
  * attach = a storage.k8s.io VolumeAttachment named csi-<sha256(handle + driver + node)>
    (attacher = driver, source.persistentVolumeName) created by the attach/detach controller;
    the kubelet's WaitForAttach waits for status.attached (attachError fails the mount);
  * SetUp at pods/<uid>/volumes/kubernetes.io~csi/<pv>/mount: GetSupportedVersions must list
    0.1.0, NodeProbe, then NodePublishVolume(volume_id = handle, publish_volume_info =
    the attachment's status.attachmentMetadata, target_path, capability mount/ext4 + access
    mode from the PV, readonly, volume_attributes from the PV annotation
    csi.volume.kubernetes.io/volume-attributes); vol_data.json next to the mount keeps what
    TearDown needs (NodeUnpublishVolume) after a kubelet restart.
  * The driver listens on <kubelet root>/plugins/<driver>/csi.sock.

Controller side (`ExternalAttacher`, the csi-attacher sidecar the reference relies on): watches
VolumeAttachments of its driver, calls ControllerPublishVolume (node id from the node's
csi.volume.kubernetes.io/nodeid annotation, else the node name) and records attached /
attachmentMetadata or attachError; on deletion ControllerUnpublishVolume, then drops its
finalizer external-attacher/<driver>.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time

import grpc

from ..api import meta as m
from ..grpcdesc.csi import CSI, VERSION
from . import VolumeError, VolumePlugin, sha256_name

log = logging.getLogger("amdkube.volume.csi")
PLUGIN = "kubernetes.io/csi"
ATTRIBS_ANN = "csi.volume.kubernetes.io/volume-attributes"
NODEID_ANN = "csi.volume.kubernetes.io/nodeid"
TIMEOUT = 15.0
_MODES = {"ReadWriteOnce": CSI.SINGLE_NODE_WRITER, "ReadOnlyMany": CSI.MULTI_NODE_READER_ONLY,
          "ReadWriteMany": CSI.MULTI_NODE_MULTI_WRITER}


def attachment_name(handle: str, driver: str, node: str) -> str:
    return "csi-" + sha256_name(handle, driver, node)


def _version():
    return CSI.Version(major=VERSION[0], minor=VERSION[1], patch=VERSION[2])


class CSIClient:
    """One driver's gRPC endpoint over its unix socket."""

    def __init__(self, socket: str):
        self.socket = socket
        self._ch = None
        self._version_ok = None

    def _channel(self):
        if self._ch is None:
            self._ch = grpc.aio.insecure_channel("unix://" + self.socket)
        return self._ch

    async def assert_version(self):
        if self._version_ok is None:
            rsp = await CSI.Identity.stub(self._channel()).GetSupportedVersions(CSI.GetSupportedVersionsRequest(),
                                                                               timeout=TIMEOUT)
            self._version_ok = any((v.major, v.minor, v.patch) == VERSION for v in rsp.supported_versions)
        if not self._version_ok:
            raise VolumeError(f"CSI driver at {self.socket} does not support version {'.'.join(map(str, VERSION))}")

    async def node_probe(self):
        await CSI.Node.stub(self._channel()).NodeProbe(CSI.NodeProbeRequest(version=_version()), timeout=TIMEOUT)

    async def node_publish(self, vol_id, target, read_only, access_mode, info, attribs, fs_type="ext4"):
        cap = CSI.VolumeCapability(mount=CSI.MountVolume(fs_type=fs_type),
                                   access_mode=CSI.AccessMode(mode=_MODES.get(access_mode, CSI.UNKNOWN)))
        await CSI.Node.stub(self._channel()).NodePublishVolume(CSI.NodePublishVolumeRequest(
            version=_version(), volume_id=vol_id, publish_volume_info=info or {}, target_path=target,
            volume_capability=cap, readonly=read_only, volume_attributes=attribs or {}), timeout=TIMEOUT)

    async def node_unpublish(self, vol_id, target):
        await CSI.Node.stub(self._channel()).NodeUnpublishVolume(CSI.NodeUnpublishVolumeRequest(
            version=_version(), volume_id=vol_id, target_path=target), timeout=TIMEOUT)

    async def controller_publish(self, vol_id, node_id, read_only, access_mode, attribs) -> dict:
        cap = CSI.VolumeCapability(mount=CSI.MountVolume(fs_type="ext4"),
                                   access_mode=CSI.AccessMode(mode=_MODES.get(access_mode, CSI.UNKNOWN)))
        rsp = await CSI.Controller.stub(self._channel()).ControllerPublishVolume(CSI.ControllerPublishVolumeRequest(
            version=_version(), volume_id=vol_id, node_id=node_id, volume_capability=cap, readonly=read_only,
            volume_attributes=attribs or {}), timeout=TIMEOUT)
        return dict(rsp.publish_volume_info)

    async def controller_unpublish(self, vol_id, node_id):
        await CSI.Controller.stub(self._channel()).ControllerUnpublishVolume(CSI.ControllerUnpublishVolumeRequest(
            version=_version(), volume_id=vol_id, node_id=node_id), timeout=TIMEOUT)

    async def close(self):
        if self._ch is not None:
            await self._ch.close()
            self._ch = None


def _attribs(pv: dict) -> dict:
    raw = ((pv.get("metadata") or {}).get("annotations") or {}).get(ATTRIBS_ANN)
    if not raw:
        return {}
    try:
        return {str(k): str(v) for k, v in json.loads(raw).items()}
    except (ValueError, AttributeError):
        raise VolumeError(f"bad {ATTRIBS_ANN} annotation on {m.name_of(pv)}")


class CSIPlugin(VolumePlugin):
    name = PLUGIN
    source_key = "csi"
    attachable = True
    supports_inline = False

    def __init__(self):
        self.clients: dict[str, CSIClient] = {}

    def socket(self, driver: str) -> str:
        return os.path.join(self.host.root_dir, "plugins", driver, "csi.sock")

    def client(self, driver: str) -> CSIClient:
        c = self.clients.get(driver)
        if c is None:
            c = self.clients[driver] = CSIClient(self.socket(driver))
        return c

    def volume_name(self, spec):
        src = spec.source("csi")
        return f"{src.get('driver', '')}^{src.get('volumeHandle', '')}"

    def device_mount_path(self, spec):
        return ""        # CSI 0.1 has no node-global staging step

    async def _attachment(self, name: str) -> dict | None:
        return await self.host.client.get_or_none("volumeattachments", name) if self.host.client else None

    async def attach(self, spec, node):
        """csi_attacher.go Attach: create the VolumeAttachment and wait for the attacher."""
        src = spec.source("csi")
        name = attachment_name(src.get("volumeHandle", ""), src.get("driver", ""), node)
        try:
            await self.host.client.create({"apiVersion": "storage.k8s.io/v1beta1", "kind": "VolumeAttachment",
                                           "metadata": {"name": name},
                                           "spec": {"attacher": src.get("driver", ""), "nodeName": node,
                                                    "source": {"persistentVolumeName": spec.name()}}})
        except m.StatusError as e:
            if not m.is_already_exists(e):
                raise
        return await self.wait_for_attach(spec, name, None, TIMEOUT, node=node)

    async def wait_for_attach(self, spec, device_path, pod, timeout, node=None):
        src = spec.source("csi")
        name = attachment_name(src.get("volumeHandle", ""), src.get("driver", ""), node or self.host.node_name)
        deadline = time.monotonic() + timeout
        while True:
            va = await self._attachment(name)
            st = (va or {}).get("status") or {}
            if st.get("attached"):
                return name
            if st.get("attachError"):
                raise VolumeError(f"attachment {name} failed: {st['attachError'].get('message', '')}")
            if time.monotonic() >= deadline:
                raise VolumeError(f"attachment {name} timed out" if va else f"volume attachment {name} not found")
            await asyncio.sleep(min(0.2, max(0.01, deadline - time.monotonic())))

    async def mount_device(self, spec, device_path, device_mount_path):
        pass

    async def unmount_device(self, device_mount_path):
        pass

    async def detach(self, volume_name, node):
        driver, _, handle = volume_name.partition("^")
        name = attachment_name(handle, driver, node)
        try:
            await self.host.client.delete("volumeattachments", name)
        except m.StatusError as e:
            if not m.is_not_found(e):
                raise

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("csi")
        driver, handle = src.get("driver", ""), src.get("volumeHandle", "")
        target = os.path.join(dir, "mount")
        data_file = os.path.join(dir, "vol_data.json")
        if os.path.exists(data_file) and self.host.mounter.is_mount_point(target):
            return target
        c = self.client(driver)
        try:
            await c.assert_version()
            await c.node_probe()
            aid = attachment_name(handle, driver, self.host.node_name)
            va = await self._attachment(aid)
            if va is None:
                raise VolumeError(f"no existing VolumeAttachment {aid} found")
            info = ((va.get("status") or {}).get("attachmentMetadata")) or {}
            os.makedirs(target, mode=0o750, exist_ok=True)
            with open(data_file, "w") as f:
                json.dump({"specVolID": spec.name(), "volumeHandle": handle, "driverName": driver,
                           "nodeName": self.host.node_name, "attachmentID": aid}, f)
            modes = spec.access_modes()
            await c.node_publish(handle, target, spec.source_read_only("csi"), modes[0] if modes else "ReadWriteOnce", info,
                                 _attribs(spec.pv or {}))
        except grpc.aio.AioRpcError as e:
            self._cleanup(dir)
            raise VolumeError(f"CSI {driver}: {e.code().name}: {e.details()}")
        except VolumeError:
            self._cleanup(dir)
            raise
        return target

    @staticmethod
    def _cleanup(dir):
        for p in (os.path.join(dir, "mount"), os.path.join(dir, "vol_data.json"), dir):
            try:
                os.rmdir(p) if not p.endswith(".json") else os.unlink(p)
            except OSError:
                pass

    async def tear_down(self, dir):
        if dir.rstrip("/").endswith("/mount"):
            dir = os.path.dirname(dir.rstrip("/"))
        data_file = os.path.join(dir, "vol_data.json")
        if not os.path.exists(data_file):
            self._cleanup(dir)
            return
        with open(data_file) as f:
            data = json.load(f)
        c = self.client(data["driverName"])
        try:
            await c.assert_version()
            await c.node_unpublish(data["volumeHandle"], os.path.join(dir, "mount"))
        except grpc.aio.AioRpcError as e:
            raise VolumeError(f"CSI {data['driverName']}: {e.code().name}: {e.details()}")
        self._cleanup(dir)


class ExternalAttacher:
    """csi-attacher sidecar: VolumeAttachment → ControllerPublishVolume."""

    def __init__(self, client, driver: str, socket: str, resync: float = 1.0):
        self.client, self.driver, self.resync = client, driver, resync
        self.csi = CSIClient(socket)
        self.finalizer = "external-attacher/" + driver.replace("/", "-")
        self._task = None

    async def _node_id(self, node: str) -> str:
        n = await self.client.get_or_none("nodes", node)
        raw = ((n or {}).get("metadata") or {}).get("annotations", {}).get(NODEID_ANN)
        if raw:
            try:
                return json.loads(raw).get(self.driver) or node
            except ValueError:
                pass
        return node

    async def sync(self, va: dict):
        spec = va.get("spec") or {}
        if spec.get("attacher") != self.driver:
            return
        name = m.name_of(va)
        md = va.get("metadata") or {}
        fins = list(md.get("finalizers") or [])
        pv_name = (spec.get("source") or {}).get("persistentVolumeName", "")
        pv = await self.client.get_or_none("persistentvolumes", pv_name) if pv_name else None
        handle = (((pv or {}).get("spec") or {}).get("csi") or {}).get("volumeHandle", "")
        node_id = await self._node_id(spec.get("nodeName", ""))
        if md.get("deletionTimestamp"):
            if self.finalizer in fins:
                try:
                    await self.csi.controller_unpublish(handle, node_id)
                except grpc.aio.AioRpcError as e:
                    await self._status(name, {"detachError": {"time": m.now_rfc3339(), "message": e.details() or e.code().name}})
                    return
                await self.client.patch("volumeattachments", name,
                                        {"metadata": {"finalizers": [f for f in fins if f != self.finalizer]}})
            return
        if (va.get("status") or {}).get("attached"):
            return
        if self.finalizer not in fins:
            await self.client.patch("volumeattachments", name, {"metadata": {"finalizers": fins + [self.finalizer]}})
        if pv is None:
            await self._status(name, {"attached": False, "attachError": {"time": m.now_rfc3339(),
                                                                         "message": f"persistentvolume {pv_name} not found"}})
            return
        ps = pv.get("spec") or {}
        modes = ps.get("accessModes") or ["ReadWriteOnce"]
        try:
            info = await self.csi.controller_publish(handle, node_id, bool((ps.get("csi") or {}).get("readOnly")), modes[0],
                                                     _attribs(pv))
        except grpc.aio.AioRpcError as e:
            await self._status(name, {"attached": False, "attachError": {"time": m.now_rfc3339(),
                                                                         "message": e.details() or e.code().name}})
            return
        await self._status(name, {"attached": True, "attachmentMetadata": info, "attachError": None})

    async def _status(self, name, st):
        try:
            await self.client.patch("volumeattachments", name, {"status": st}, sub="status")
        except m.StatusError as e:
            if not m.is_not_found(e):
                raise

    async def run(self):
        while True:
            try:
                vas, _ = await self.client.list("volumeattachments")
                for va in vas:
                    try:
                        await self.sync(va)
                    except Exception as e:      # one bad attachment never stops the others
                        log.warning("attacher: %s: %r", m.name_of(va), e)
            except Exception as e:
                log.debug("attacher list failed: %r", e)
            await asyncio.sleep(self.resync)

    def start(self):
        self._task = asyncio.create_task(self.run(), name=f"csi-attacher-{self.driver}")
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
        await self.csi.close()
