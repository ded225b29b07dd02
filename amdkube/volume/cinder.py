"""Cloud block disks attached through the cloud provider: OpenStack Cinder (pkg/volume/cinder:
attacher.go, cinder.go, cinder_util.go), AWS EBS (pkg/volume/aws_ebs: attacher.go, aws_ebs.go,
aws_util.go), GCE persistent disks (pkg/volume/gce_pd) and Azure managed disks
(pkg/volume/azure_dd) Photon persistent disks (pkg/volume/photon_pd) and vSphere
VMDKs (pkg/volume/vsphere_volume).

One flow for all of them: the attach/detach controller attaches the disk to the node's
instance through `--cloud-provider`'s volumes() (cloudprovider/{openstack,aws,gce,azure}.py),
the kubelet waits for the disk to appear under one of the provider's device paths (by serial /
by-id first, the device the cloud reported last), formats it if blank, mounts it once per node
and bind-mounts it into pods (the shared _Block machinery).
"""
from __future__ import annotations

import asyncio

from . import VolumeError
from .network import _Block


class CloudDiskPlugin(_Block):
    """A block disk whose attach/detach go through the cloud provider's volumes()."""
    provider = ""         # cloud provider name that serves this volume type
    id_field = ""         # the source field naming the disk

    def volume_name(self, spec) -> str:
        return spec.source(self.source_key).get(self.id_field, "")

    def _volumes(self):
        cloud = getattr(self.host, "cloud", None)
        vols = cloud.volumes() if cloud is not None and hasattr(cloud, "volumes") else None
        if vols is None or getattr(vols, "source_key", self.source_key) != self.source_key:
            raise VolumeError(f"{self.source_key} volumes need the {self.provider} cloud provider (--cloud-provider={self.provider})")
        return vols

    async def attach(self, spec, node: str) -> str:
        vid = self.volume_name(spec)
        if not vid:
            raise VolumeError(f"{self.source_key} volume {spec.name()!r} has no {self.id_field}")
        return await asyncio.to_thread(self._volumes().attach, node, vid)

    async def wait_for_attach(self, spec, device_path, pod, timeout):
        vid = self.volume_name(spec)
        pats = self._volumes().device_candidates(vid, device_path)
        return await self._wait_device(pats, timeout, f"{self.source_key} volume {vid}")

    async def detach(self, volume_name: str, node: str):
        await asyncio.to_thread(self._volumes().detach, node, volume_name)


class CinderPlugin(CloudDiskPlugin):
    name = "kubernetes.io/cinder"
    source_key = "cinder"
    provider = "openstack"
    id_field = "volumeID"


class AWSEBSPlugin(CloudDiskPlugin):
    """aws_ebs: volumeID `aws://<zone>/vol-…`; partition and readOnly from the source."""
    name = "kubernetes.io/aws-ebs"
    source_key = "awsElasticBlockStore"
    provider = "aws"
    id_field = "volumeID"


class GCEPDPlugin(CloudDiskPlugin):
    """gce_pd: pdName names a zonal persistent disk, attached with deviceName = pdName."""
    name = "kubernetes.io/gce-pd"
    source_key = "gcePersistentDisk"
    provider = "gce"
    id_field = "pdName"

    async def attach(self, spec, node: str) -> str:
        vid = self.volume_name(spec)
        if not vid:
            raise VolumeError(f"gcePersistentDisk volume {spec.name()!r} has no pdName")
        ro = spec.source_read_only(self.source_key)
        return await asyncio.to_thread(self._volumes().attach, node, vid, ro)


class AzureDiskPlugin(CloudDiskPlugin):
    """azure_dd (kind Managed): diskURI names the managed disk; attach answers the LUN and the
    kubelet finds the disk by it (azure_common_linux.go findDiskByLun)."""
    name = "kubernetes.io/azure-disk"
    source_key = "azureDisk"
    provider = "azure"
    id_field = "diskURI"

    async def attach(self, spec, node: str) -> str:
        src = spec.source(self.source_key)
        if (src.get("kind") or "Shared") != "Managed":
            raise VolumeError(f"azureDisk volume {spec.name()!r}: kind {src.get('kind') or 'Shared'} (blob disks) is not "
                              "supported; use kind: Managed")
        uri = self.volume_name(spec)
        if not uri:
            raise VolumeError(f"azureDisk volume {spec.name()!r} has no diskURI")
        caching = src.get("cachingMode") or "ReadOnly"
        return await asyncio.to_thread(self._volumes().attach, node, uri, caching)


class PhotonPDPlugin(CloudDiskPlugin):
    """photon_pd: pdID names a Photon persistent disk; it shows up by its WWN."""
    name = "kubernetes.io/photon-pd"
    source_key = "photonPersistentDisk"
    provider = "photon"
    id_field = "pdID"


class VSphereVolumePlugin(CloudDiskPlugin):
    """vsphere_volume: volumePath `[datastore] kubevols/<disk>.vmdk`, attached to the node VM's
    SCSI controller and found by the disk's WWN."""
    name = "kubernetes.io/vsphere-volume"
    source_key = "vsphereVolume"
    provider = "vsphere"
    id_field = "volumePath"


def plugins():
    return [CinderPlugin(), AWSEBSPlugin(), GCEPDPlugin(), AzureDiskPlugin(), PhotonPDPlugin(), VSphereVolumePlugin()]
