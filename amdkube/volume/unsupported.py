"""Volume types recognised without a backend: a pod using one gets a precise FailedMount event
instead of "no volume plugin matched". Every in-tree type of the reference now has a real
plugin (volume/cinder.py for the cloud disks, volume/vendor.py for Flocker, StorageOS,
Portworx and ScaleIO) — this table is kept for types a build
leaves out.
"""
from __future__ import annotations

from . import VolumeError, VolumePlugin

_TYPES: dict[str, tuple[str, str]] = {}


class UnavailableBackendPlugin(VolumePlugin):
    def __init__(self, key: str, name: str, needs: str):
        self.source_key, self.name, self.needs = key, name, needs

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        raise VolumeError(f"{self.source_key} volume {spec.name()!r} needs {self.needs}, which this node cannot reach "
                          f"(use csi, flexVolume, iscsi, rbd, nfs or local volumes on MI355X hosts)")


def plugins() -> list[VolumePlugin]:
    return [UnavailableBackendPlugin(k, n, why) for k, (n, why) in _TYPES.items()]
