"""OpenStack Cinder volumes (pkg/volume/cinder: attacher.go, cinder.go, cinder_util.go).

Attachable block volumes: the attach/detach controller attaches the volume to the node's Nova
server through the cloud provider (`--cloud-provider=openstack`, cloudprovider/openstack.py),
the kubelet waits for the disk to appear by its serial (/dev/disk/by-id/virtio-<id[:20]>,
the device Nova reported only with [BlockStorage] trust-device-path), formats it if blank,
mounts it once per node and bind-mounts it into pods (the shared _Block machinery).
"""
from __future__ import annotations

import asyncio

from . import VolumeError
from .network import _Block


class CinderPlugin(_Block):
    name = "kubernetes.io/cinder"
    source_key = "cinder"

    def volume_name(self, spec) -> str:
        return spec.source("cinder").get("volumeID", "")

    def _volumes(self):
        cloud = getattr(self.host, "cloud", None)
        vols = cloud.volumes() if cloud is not None and hasattr(cloud, "volumes") else None
        if vols is None:
            raise VolumeError("cinder volumes need the OpenStack cloud provider (--cloud-provider=openstack)")
        return vols

    async def attach(self, spec, node: str) -> str:
        vid = self.volume_name(spec)
        if not vid:
            raise VolumeError(f"cinder volume {spec.name()!r} has no volumeID")
        return await asyncio.to_thread(self._volumes().attach, node, vid)

    async def wait_for_attach(self, spec, device_path, pod, timeout):
        from ..cloudprovider.openstack import device_candidates
        vid = self.volume_name(spec)
        pats = device_candidates(vid)
        cloud = getattr(self.host, "cloud", None)
        trust = str(((getattr(cloud, "cfg", None) or {}).get("blockstorage") or {}).get("trust-device-path", "false")).lower()
        if device_path and trust == "true":
            pats = [device_path] + pats
        return await self._wait_device(pats, timeout, f"cinder volume {vid}")

    async def detach(self, volume_name: str, node: str):
        await asyncio.to_thread(self._volumes().detach, node, volume_name)


def plugins():
    return [CinderPlugin()]
