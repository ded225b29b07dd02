"""vSphere cloud provider and vsphereVolume disks (reference: pkg/cloudprovider/providers/vsphere
vsphere_test.go — TestInstances / TestVolumes, vclib/virtualmachine.go AttachDisk/DetachDisk,
diskmanagers/virtualdisk.go; pkg/volume/vsphere_volume attacher_test.go), against the in-repo
fake vCenter (tests/fake_vsphere.py). No vCenter exists offline: parity with the real vim25
service is unpinned; the SOAP shapes follow the public vSphere Web Services API."""
import asyncio

import pytest

from amdkube.cloudprovider import get_cloud_provider
from amdkube.cloudprovider.vsphere import MoRef, VSphereError, _xml, envelope, parse, parse_config
from amdkube.volume import FakeExec, FakeMounter, PluginMgr, Spec, VolumeHost, default_plugins
from tests.conftest import run
from tests.fake_vsphere import FakeVCenter
from tests.test_volumes import FakeClient


@pytest.fixture()
def vc():
    f = FakeVCenter().start()
    yield f
    f.stop()


def test_soap_codec_round_trip():
    body = envelope("ReconfigVM_Task", MoRef("VirtualMachine", "vm-7"), {"spec": {
        "@type": "VirtualMachineConfigSpec", "deviceChange": [{"operation": "add"}, {"operation": "remove"}]}})
    assert '<_this type="VirtualMachine">vm-7</_this>' in body and 'xsi:type="VirtualMachineConfigSpec"' in body
    import xml.etree.ElementTree as ET
    op = ET.fromstring(body)[0][0]
    spec = parse(op[1])
    assert parse(op[0]) == MoRef("VirtualMachine", "vm-7")
    assert spec == {"@type": "VirtualMachineConfigSpec", "deviceChange": [{"operation": "add"}, {"operation": "remove"}]}
    assert _xml("x", "a<b") == "<x>a&lt;b</x>" and _xml("b", True) == "<b>true</b>"
    cfg = parse_config('[Global]\nuser = u\n[VirtualCenter "10.0.0.1"]\nport = 8443\n[Workspace]\ndatacenter = d\n')
    assert cfg["vcenters"] == {"10.0.0.1": {"port": "8443"}} and cfg["workspace"]["datacenter"] == "d"


def test_instances(vc):
    a = vc.add_vm("gpu-a", [("VM Network", ["10.4.0.5", "fe80::1"]), ("storage", ["192.168.9.5"])])
    vc.add_vm("gpu-off", [("VM Network", ["10.4.0.9"])], power="poweredOff")
    cloud = get_cloud_provider("vsphere", vc.config(Network={"public-network": "VM Network"}))
    ins = cloud.instances()

    async def go():
        assert await ins.node_addresses("gpu-a") == [{"type": "ExternalIP", "address": "10.4.0.5"},
                                                     {"type": "InternalIP", "address": "10.4.0.5"}]
        uid = await ins.instance_id("gpu-a")
        assert uid == vc.vms[a]["uuid"].lower()
        assert await ins.instance_exists("gpu-a")
        assert not await ins.instance_exists("gpu-off") and not await ins.instance_exists("nope")
        assert await ins.instance_exists_by_provider_id(f"vsphere://{uid}")
        assert not await ins.instance_exists_by_provider_id("vsphere://4210c5d9-0000-0000-0000-000000000000")
    asyncio.run(go())
    assert vc.logins == 1
    # an expired session: one re-login, then the call succeeds
    vc.sessions.clear()
    assert asyncio.run(ins.instance_exists("gpu-a")) and vc.logins == 2
    # every network without public-network
    every = get_cloud_provider("vsphere", vc.config()).instances()
    assert {x["address"] for x in asyncio.run(every.node_addresses("gpu-a"))} == {"10.4.0.5", "192.168.9.5"}
    bad = get_cloud_provider("vsphere", vc.config().replace(vc.PASSWORD, "wrong"))
    with pytest.raises(VSphereError) as e:
        asyncio.run(bad.instances().instance_exists("gpu-a"))
    assert e.value.fault == "InvalidLogin"


def test_disks_create_attach_detach_delete(vc):
    a = vc.add_vm("gpu-a", [("VM Network", ["10.4.0.5"])])
    cloud = get_cloud_provider("vsphere", vc.config())
    vols = cloud.volumes()
    src, labels = vols.provision("pvc-1", 10, {"diskformat": "zeroedthick", "fstype": "xfs"}, {}, "claim")
    path = src["volumePath"]
    assert path == "[ds1] kubevols/kubernetes-dynamic-pvc-1.vmdk" and src["fsType"] == "xfs" and labels == {}
    assert vc.last_spec["capacityKb"] == str(10 << 20) and vc.last_spec["diskType"] == "zeroedthick"
    vols.create("second", 1)                                   # kubevols exists: MakeDirectory's fault is fine
    dev = vols.attach("gpu-a", path)
    wwn = vc.disks[path].replace(" ", "").lower()
    assert dev == f"/dev/disk/by-id/wwn-0x{wwn}"
    added = [d for d in vc.vms[a]["devices"] if d.get("backing", {}).get("fileName") == path]
    assert added and added[0]["unitNumber"] == "1" and added[0]["controllerKey"] == "1000"
    assert added[0]["backing"]["diskMode"] == "independent_persistent"
    assert vols.attach("gpu-a", path) == dev and len(vc.vms[a]["devices"]) == 3      # idempotent
    assert vols.is_attached("gpu-a", path) and vols.device_candidates(path, dev) == [dev]
    assert vols.device_candidates(path) == [dev]
    with pytest.raises(VSphereError):
        vols.delete_source(src)                                # attached: the task fails
    vols.detach("gpu-a", path)
    assert not vols.is_attached("gpu-a", path)
    vols.detach("gpu-a", path)
    vols.delete_source(src)
    assert path not in vc.disks
    vols.delete_source(src)                                    # already gone
    with pytest.raises(ValueError):
        vols.create("bad", 1, "sparse")


def test_vsphere_volume_plugin_attaches_through_the_provider(tmp_path, vc):
    vc.add_vm("node-a", [("VM Network", ["10.4.0.5"])])
    cloud = get_cloud_provider("vsphere", vc.config())
    path = cloud.volumes().create("ckpt", 2)
    h = VolumeHost(str(tmp_path / "kubelet"), "node-a", FakeClient(), FakeMounter(), FakeExec())
    h.dev_root, h.attach_poll, h.cloud = str(tmp_path / "root"), 0.01, cloud
    p = PluginMgr(default_plugins(), h).find_by_spec(Spec({"name": "v", "vsphereVolume": {"volumePath": path}}))
    assert p.name == "kubernetes.io/vsphere-volume" and p.attachable
    spec = Spec({"name": "v", "vsphereVolume": {"volumePath": path, "fsType": "ext4"}})
    dev = run(p.attach(spec, "node-a"))
    (tmp_path / "root" / "dev/disk/by-id").mkdir(parents=True)
    (tmp_path / "root" / dev.lstrip("/")).touch()
    assert run(p.wait_for_attach(spec, dev, None, 2)) == str(tmp_path / "root" / dev.lstrip("/"))
    run(p.detach(path, "node-a"))
    assert not cloud.volumes().is_attached("node-a", path)
