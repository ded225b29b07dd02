"""Flocker, StorageOS, Portworx and ScaleIO volumes (reference: pkg/volume/flocker
flocker_test.go / flocker_util_test.go, pkg/volume/storageos storageos_test.go /
storageos_util_test.go, pkg/volume/portworx portworx_test.go, pkg/volume/scaleio sio_volume_test.go
/ sio_mgr_test.go) through the kubelet's plugin manager, against the in-repo fakes in
tests/fake_storage.py. No vendor backend exists offline: parity with the real services is
unpinned."""
import asyncio
import base64
import os

import pytest

from amdkube.volume import FakeExec, FakeMounter, PluginMgr, Spec, VolumeError, VolumeHost, default_plugins
from amdkube.volume import vendor
from tests.conftest import run
from tests.fake_storage import FakeFlocker, FakePortworx, FakeScaleIO, FakeStorageOS
from tests.test_volumes import FakeClient


def _host(tmp_path, client=None, executor=None, node_ip="10.0.0.5"):
    h = VolumeHost(str(tmp_path / "kubelet"), "node-a", client or FakeClient(), FakeMounter(), executor or FakeExec(),
                   node_ip=node_ip)
    h.dev_root = str(tmp_path / "root")
    h.attach_poll = 0.01
    return h


def _secret(**kv):
    return {"data": {k: base64.b64encode(v.encode()).decode() for k, v in kv.items()}}


POD = {"metadata": {"name": "p", "namespace": "default", "uid": "u1"}}


def _dir(h, plugin, name, uid="u1"):
    return h.pod_volume_dir(uid, plugin, name)


@pytest.fixture()
def flocker(monkeypatch):
    f = FakeFlocker({"uuid-a": "10.0.0.5", "uuid-b": "10.0.0.6"}).start()
    monkeypatch.setenv("FLOCKER_CONTROL_SERVICE_PROTOCOL", "http")
    monkeypatch.setenv("FLOCKER_CONTROL_SERVICE_HOST", "127.0.0.1")
    monkeypatch.setenv("FLOCKER_CONTROL_SERVICE_PORT", f.url.rsplit(":", 1)[1])
    yield f
    f.stop()


def test_flocker_moves_the_dataset_here_and_binds_its_path(tmp_path, flocker):
    ds = flocker.add_dataset("gpu-ckpt", primary="uuid-b")
    h = _host(tmp_path)
    mgr = PluginMgr(default_plugins(), h)
    spec = Spec({"name": "data", "flocker": {"datasetName": "gpu-ckpt"}})
    p = mgr.find_by_spec(spec)
    assert p.name == "kubernetes.io/flocker" and p.volume_name(spec) == "gpu-ckpt"
    p.wait_tick = 0.01
    d = _dir(h, p.name, "data")
    run(p.set_up(spec, POD, d))
    assert flocker.moves == [(ds, "uuid-a")] and flocker.config[ds]["primary"] == "uuid-a"
    assert h.mounter.actions("mount")[-1][1:3] == (d, os.path.join(h.dev_root, f"flocker/{ds}"))
    # already primary here: no move, by UUID
    run(p.set_up(Spec({"name": "d2", "flocker": {"datasetUUID": ds}}), POD, _dir(h, p.name, "d2")))
    assert len(flocker.moves) == 1
    run(p.tear_down(d))
    assert not h.mounter.is_mount_point(d)
    with pytest.raises(VolumeError):
        run(p.set_up(Spec({"name": "x", "flocker": {"datasetName": "missing"}}), POD, _dir(h, p.name, "x")))
    # provisioning: a dataset of the claim's size, deleted on reclaim
    src, labels = run(vendor.FlockerProvisioner().aprovision(None, "pvc-1", 2, {}, {}, "claim"))
    assert flocker.config[src["datasetUUID"]]["maximum_size"] == 2 << 30 and labels == {}
    run(vendor.FlockerProvisioner().adelete(None, src))
    assert src["datasetUUID"] not in flocker.config


def test_storageos_loop_device_global_mount_and_release(tmp_path):
    devdir = str(tmp_path / "root" / "var/lib/storageos/volumes")
    f = FakeStorageOS(devdir, password="s3cret").start()
    try:
        vid = f.add_volume("default", "vol-1")
        client = FakeClient({("secrets", "default", "sos"): _secret(apiAddress=f.url.replace("http://", "tcp://"),
                                                                      apiUsername="storageos", apiPassword="s3cret")})
        ex = FakeExec({("losetup", "--find", "--show"): (0, "/dev/loop7\n"), ("losetup", "-j"): (0, "")})
        h = _host(tmp_path, client, ex)
        mgr = PluginMgr(default_plugins(), h)
        spec = Spec({"name": "v", "storageos": {"volumeName": "vol-1", "secretRef": {"name": "sos"}, "fsType": "ext4"}})
        p = mgr.find_by_spec(spec)
        assert p.name == "kubernetes.io/storageos" and p.volume_name(spec) == "default.vol-1"
        d1, d2 = _dir(h, p.name, "v", "u1"), _dir(h, p.name, "v", "u2")
        run(p.set_up(spec, POD, d1))
        run(p.set_up(spec, POD, d2))
        gp = p.global_path("default.vol-1")
        assert ["losetup", "--find", "--show", os.path.join(devdir, vid)] in ex.calls
        mounts = h.mounter.actions("mount")
        assert mounts[0][1:4] == (gp, "/dev/loop7", "ext4")          # device mounted once, at the global path
        assert [a[1] for a in mounts[1:]] == [d1, d2]
        assert f.mounts[("default", "vol-1")]["client"] == "node-a"
        run(p.tear_down(d1))
        assert h.mounter.is_mount_point(gp) and ("default", "vol-1") in f.mounts   # a second pod still uses it
        run(p.tear_down(d2))
        assert not h.mounter.is_mount_point(gp) and ("default", "vol-1") not in f.mounts
        assert ["losetup", "-d", "/dev/loop7"] in ex.calls
        # provisioning with the admin secret; deletion on reclaim
        prov = vendor.StorageOSProvisioner()
        src, _ = run(prov.aprovision(client, "pvc-9", 3, {"pool": "gpu", "adminSecretName": "sos", "adminSecretNamespace": "default"},
                                     {"kubernetes.io/created-for/pvc/namespace": "default"}, "claim"))
        assert f.volumes[("default", "pvc-9")]["size"] == 3 and f.volumes[("default", "pvc-9")]["pool"] == "gpu"
        assert src["secretRef"] == {"name": "sos", "namespace": "default"}
        run(prov.adelete(client, src))
        assert ("default", "pvc-9") not in f.volumes
        # wrong credentials: the API refuses
        bad = FakeClient({("secrets", "default", "sos"): _secret(apiAddress=f.url, apiPassword="nope")})
        p.host.client = bad
        with pytest.raises(VolumeError):
            run(p.set_up(spec, POD, _dir(h, p.name, "v", "u3")))
    finally:
        f.stop()


def test_portworx_attach_mount_and_detach_on_last_unmount(tmp_path, monkeypatch):
    f = FakePortworx().start()
    monkeypatch.setenv("AMDKUBE_PORTWORX_ENDPOINT", f.url)
    try:
        vid = f.add_volume("pxvol")
        h = _host(tmp_path)
        mgr = PluginMgr(default_plugins(), h)
        spec = Spec({"name": "px", "portworxVolume": {"volumeID": vid}})
        p = mgr.find_by_spec(spec)
        d1, d2 = _dir(h, p.name, "px", "u1"), _dir(h, p.name, "px", "u2")
        run(p.set_up(spec, POD, d1))
        run(p.set_up(spec, POD, d2))
        assert [a for _, a in f.actions] == [{"attach": 1}, {"mount": 1, "mount_path": d1}, {"mount": 1, "mount_path": d2}]
        run(p.tear_down(d1))
        assert f.vols[vid]["attached_on"] and f.vols[vid]["attach_path"] == [d2]
        run(p.tear_down(d2))
        assert f.actions[-1][1] == {"attach": 2} and not f.vols[vid]["attached_on"]
        with pytest.raises(VolumeError):
            run(p.set_up(Spec({"name": "y", "portworxVolume": {"volumeID": "404"}}), POD, _dir(h, p.name, "y")))
        prov = vendor.PortworxProvisioner()
        src, _ = run(prov.aprovision(None, "pvc-px", 4, {"repl": "2", "fs": "xfs"}, {"k": "v"}, "claim"))
        v = f.vols[src["volumeID"]]
        assert v["spec"]["size"] == 4 << 30 and v["spec"]["ha_level"] == 2 and v["spec"]["format"] == "xfs"
        assert v["locator"]["name"] == "pvc-px" and src["fsType"] == "xfs"
        run(prov.adelete(None, src))
        assert src["volumeID"] not in f.vols
    finally:
        f.stop()


def test_scaleio_maps_to_this_sdc_and_unmaps(tmp_path):
    by_id = str(tmp_path / "root" / "dev/disk/by-id")
    f = FakeScaleIO(by_id, sdc_guid="GUID-A").start()
    try:
        vid = f.add_volume("sio-vol")
        client = FakeClient({("secrets", "default", "sio"): _secret(username=f.USER, password=f.PASSWORD),
                             ("nodes", "", "node-a"): {"metadata": {"labels": {"scaleio.sdcGuid": "GUID-A"}}}})
        h = _host(tmp_path, client)
        mgr = PluginMgr(default_plugins(), h)
        src = {"gateway": f.url + "/api", "system": "sio-sys", "secretRef": {"name": "sio"}, "volumeName": "sio-vol"}
        spec = Spec({"name": "s", "scaleIO": src})
        p = mgr.find_by_spec(spec)
        assert p.name == "kubernetes.io/scaleio"
        d = _dir(h, p.name, "s")
        run(p.set_up(spec, POD, d))
        assert f.volumes[vid]["mappedSdcInfo"] == [{"sdcId": "sdc-1"}]
        dev = os.path.join(by_id, f"emc-vol-{f.MDM}-{vid}")
        assert h.mounter.actions("mount")[0][1:4] == (p.global_path("sio-vol"), dev, "xfs")
        run(p.tear_down(d))
        assert f.volumes[vid]["mappedSdcInfo"] == [] and not os.path.exists(dev)
        # no label: drv_cfg answers the GUID
        h2 = _host(tmp_path / "h2", FakeClient({("secrets", "default", "sio"): _secret(username=f.USER, password=f.PASSWORD)}),
                   FakeExec({("/opt/emc/scaleio/sdc/bin/drv_cfg", "--query_guid"): (0, "GUID-A\n")}))
        h2.dev_root = h.dev_root
        p2 = PluginMgr(default_plugins(), h2).find_by_spec(spec)
        run(p2.set_up(spec, POD, _dir(h2, p2.name, "s")))
        assert f.volumes[vid]["mappedSdcInfo"] == [{"sdcId": "sdc-1"}]
        run(p2.tear_down(_dir(h2, p2.name, "s")))
        # provisioning: 8 GiB allocation units in the named pool
        prov = vendor.ScaleIOProvisioner()
        params = {"gateway": f.url + "/api", "system": "sio-sys", "protectionDomain": "pd-gpu", "storagePool": "sp-ssd",
                  "secretRef": "sio", "secretNamespace": "default"}
        out, _ = run(prov.aprovision(client, "pvc-0123456789abcdef0123", 10, params, {}, "claim"))
        nv = next(v for v in f.volumes.values() if v["name"] == out["volumeName"])
        assert nv["sizeInKb"] == 16 << 20 and nv["storagePoolId"] == "sp-1" and nv["volumeType"] == "ThinProvisioned"
        run(prov.adelete(client, out))
        assert all(v["name"] != out["volumeName"] for v in f.volumes.values())
        with pytest.raises(VolumeError):
            run(prov.aprovision(client, "pvc-x", 1, {**params, "storagePool": "nope"}, {}, "claim"))
        bad = FakeClient({("secrets", "default", "sio"): _secret(username=f.USER, password="wrong")})
        with pytest.raises(VolumeError):
            run(prov.aprovision(bad, "pvc-y", 1, params, {}, "claim"))
    finally:
        f.stop()


def test_every_reference_volume_type_has_a_plugin():
    """The v1.9 VolumeSource types all resolve to exactly one plugin."""
    h = VolumeHost("/tmp/unused", "n", FakeClient(), FakeMounter(), FakeExec())
    mgr = PluginMgr(default_plugins(), h)
    for key in ("flocker", "storageos", "portworxVolume", "scaleIO", "photonPersistentDisk", "cinder", "awsElasticBlockStore",
                "gcePersistentDisk", "azureDisk", "vsphereVolume"):
        assert mgr.find_by_spec(Spec({"name": "x", key: {}})).source_key == key
    assert asyncio.iscoroutinefunction(vendor.ScaleIOProvisioner().aprovision)


def test_pv_controller_provisions_and_reclaims_vendor_and_vsphere_volumes(tmp_path, monkeypatch):
    """The PV binder's dynamic provisioning (persistentvolume/pv_controller.go provisionClaim /
    deleteVolumeOperation) through a vendor provisioner (Portworx) and a cloud one (vSphere)."""
    from amdkube.api import meta as m
    from amdkube.client import Client
    from amdkube.cloudprovider import get_cloud_provider
    from amdkube.controllers import ControllerManager, Options
    from amdkube.localcluster import LocalCluster
    from tests.fake_vsphere import FakeVCenter
    px, vc = FakePortworx().start(), FakeVCenter().start()
    monkeypatch.setenv("AMDKUBE_PORTWORX_ENDPOINT", px.url)

    async def go():
        async with LocalCluster(gpus="fake", n_gpus=1, with_controllers=False, relist_period=0.2) as lc:
            c = lc.client
            for name, prov, params in (("px", "kubernetes.io/portworx-volume", {"repl": "3"}),
                                       ("vs", "kubernetes.io/vsphere-volume", {"diskformat": "thin"})):
                await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": name},
                                "provisioner": prov, "parameters": params})
                await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": "default"},
                                "spec": {"storageClassName": name, "accessModes": ["ReadWriteOnce"],
                                         "resources": {"requests": {"storage": "3Gi"}}}}, "default")
            cmc = Client(lc.api.url, token=lc.api.loopback_token)
            cm = await ControllerManager(cmc, ["persistentvolume-binder", "pvc-protection", "pv-protection"],
                                         options=Options(cloud=get_cloud_provider("vsphere", vc.config()))).start()
            try:
                async def until(fn, t=30):
                    end = asyncio.get_running_loop().time() + t
                    while asyncio.get_running_loop().time() < end:
                        v = await fn()
                        if v:
                            return v
                        await asyncio.sleep(0.05)
                    raise AssertionError("condition not met")
                pvs = {}
                for name in ("px", "vs"):
                    async def bound(name=name):
                        p = await c.get("persistentvolumeclaims", name, "default")
                        return p if (p.get("status") or {}).get("phase") == "Bound" else None
                    pvs[name] = await c.get("persistentvolumes", (await until(bound))["spec"]["volumeName"])
                vid = pvs["px"]["spec"]["portworxVolume"]["volumeID"]
                assert px.vols[vid]["spec"]["size"] == 3 << 30 and px.vols[vid]["spec"]["ha_level"] == 3
                path = pvs["vs"]["spec"]["vsphereVolume"]["volumePath"]
                assert path in vc.disks and m.annotations_of(pvs["vs"])["pv.kubernetes.io/provisioned-by"] == "kubernetes.io/vsphere-volume"
                for name in ("px", "vs"):
                    await c.delete("persistentvolumeclaims", name, "default")

                async def gone():
                    return vid not in px.vols and path not in vc.disks
                await until(gone)
            finally:
                await cm.stop()
                await cmc.close()
    try:
        run(go(), 90)
    finally:
        px.stop()
        vc.stop()
