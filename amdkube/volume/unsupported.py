"""Volume types whose backends are vendor services this build cannot reach (pkg/volume/
vsphere_volume, photon_pd, portworx, scaleio, storageos, flocker). Cinder, AWS EBS, GCE PD and
Azure managed disks are real plugins (volume/cinder.py) over the OpenStack, AWS, GCE and Azure
providers. These are recognised — so a pod using one gets a precise FailedMount event instead
of "no volume plugin matched" — but their set-up fails: attaching them needs the vendor's API
or client library (vCenter, Photon controller, Portworx, ScaleIO gateway + drv_cfg, StorageOS,
Flocker control service), none of which an MI355X host has.
"""
from __future__ import annotations

from . import VolumeError, VolumePlugin

_TYPES = {
    "vsphereVolume": ("kubernetes.io/vsphere-volume", "the vSphere API"),
    "photonPersistentDisk": ("kubernetes.io/photon-pd", "the Photon controller API"),
    "portworxVolume": ("kubernetes.io/portworx-volume", "the Portworx REST API"),
    "scaleIO": ("kubernetes.io/scaleio", "the ScaleIO gateway and drv_cfg"),
    "storageos": ("kubernetes.io/storageos", "the StorageOS API"),
    "flocker": ("kubernetes.io/flocker", "the Flocker control service"),
}


class UnavailableBackendPlugin(VolumePlugin):
    def __init__(self, key: str, name: str, needs: str):
        self.source_key, self.name, self.needs = key, name, needs

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        raise VolumeError(f"{self.source_key} volume {spec.name()!r} needs {self.needs}, which this node cannot reach "
                          f"(use csi, flexVolume, iscsi, rbd, nfs or local volumes on MI355X hosts)")


def plugins() -> list[VolumePlugin]:
    return [UnavailableBackendPlugin(k, n, why) for k, (n, why) in _TYPES.items()]
