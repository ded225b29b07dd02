"""DeviceManager + plugin framework: ports of the reference's devicemanager test semantics
(pkg/kubelet/cm/devicemanager/{manager,endpoint,endpoint_handler,device_store}_test.go and
pluginregistration/v1beta/plugin_watcher_test.go) plus the AMD plugin
on the fake 8×MI355X backend and wire-golden checks for the runtime-built descriptors."""
import asyncio
import os
import socket
import tempfile

import pytest

from amdkube.deviceplugin import AMDGPUPlugin, StubDevicePlugin
from amdkube.grpcdesc.deviceplugin import REGISTRATION as R, V1ALPHA2 as P
from amdkube.kubelet.devicemanager import (AdmissionError, DeviceStore, ManagerImpl, PluginWatcher, merge_container_specs)
from amdkube.smi import FakeBackend
from amdkube.utils.metrics import new_registry, render
from tests.conftest import run


def devs(*ids, health="Healthy", **attrs):
    return [{"ID": i, "health": health, "Attributes": dict(attrs)} for i in ids]


async def wait_for(pred, timeout=5.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        if pred():
            return True
        await asyncio.sleep(0.01)
    raise AssertionError("condition not met in time")


def short_tmp():
    # UDS paths must stay < 108 bytes
    return tempfile.mkdtemp(prefix="ak", dir="/tmp")


def test_wire_golden_bytes():
    assert P.Device(ID="a", health="Healthy", Attributes={"k": "v"}).SerializeToString().hex() == \
        "0a016112074865616c7468791a060a016b120176"
    assert P.GetPluginInfoResponse(init_timeout=5, labels={"x": "y"}).SerializeToString().hex() == "080512060a0178120179"
    assert R.RegistrationStatus(success=True, error="e").SerializeToString().hex() == "0801120165"
    assert P.DevicePlugin.full_name == "deviceplugin.DevicePlugin"
    assert [m[0] for m in R.Identity.methods] == ["GetSupportedVersions", "GetPluginIdentity", "PluginRegistrationStatus"]


def test_device_store_diff():
    s = DeviceStore()
    a, u, d = s.update(devs("1", "2"))
    assert [x["ID"] for x in a] == ["1", "2"] and not u and not d
    a, u, d = s.update(devs("1") + devs("2", health="Unhealthy") + devs("3"))
    assert [x["ID"] for x in a] == ["3"] and [x["ID"] for x in u] == ["2"] and not d
    a, u, d = s.update(devs("1", m="x") + devs("3"))  # attribute change counts (fix #11)
    assert [x["ID"] for x in u] == ["1"] and [x["ID"] for x in d] == ["2"]


def test_watcher_layout_rules():
    async def go():
        root = short_tmp()
        w = await PluginWatcher(root).start()
        srv = socket.socket(socket.AF_UNIX)
        os.makedirs(os.path.join(root, "amd.com"))
        await asyncio.sleep(0.05)
        srv.bind(os.path.join(root, "amd.com", "gpu.sock"))
        assert await asyncio.wait_for(w.added.get(), 2) == os.path.join(root, "amd.com", "gpu.sock")
        bad = socket.socket(socket.AF_UNIX)
        bad.bind(os.path.join(root, "gpu.sock"))  # socket in root: rejected
        os.makedirs(os.path.join(root, "amd.com", "nested"))  # nested dir: rejected
        await wait_for(lambda: len(w.errors) >= 2)
        assert w.added.empty()
        os.unlink(os.path.join(root, "amd.com", "gpu.sock"))
        assert await asyncio.wait_for(w.removed.get(), 2) == os.path.join(root, "amd.com", "gpu.sock")
        await w.stop()
    run(go())


def test_manager_plugin_handling_and_reregistration():
    async def go():
        root = short_tmp()
        reg = new_registry()
        m = await ManagerImpl(root, registry=reg).start()
        p1 = await StubDevicePlugin("amd.com/gpu", devs("g0", "g1"), plugins_dir=root).start()
        p2 = await StubDevicePlugin("example.com/fpga", devs("f0"), plugins_dir=root).start()
        await p1.wait_for_registration()
        await p2.wait_for_registration()
        await wait_for(lambda: len(m.store.peek()) == 2)
        cap = m.store.peek()
        assert sorted(cap["amd.com/gpu"]["resources"]) == ["g0", "g1"] and list(cap["example.com/fpga"]["resources"]) == ["f0"]
        # shrink
        p1.update(devs("g0"))
        await wait_for(lambda: list(m.store.peek().get("amd.com/gpu", {}).get("resources", {})) == ["g0"])
        # re-registration with the same resource name: devices are not deleted (no flap)
        updates = []
        m.store.listeners.append(updates.append)
        p1b = StubDevicePlugin("amd.com/gpu", devs("g0"), plugins_dir=root, sock_name="gpu2")
        await p1b.start()
        await p1b.wait_for_registration()
        await asyncio.sleep(0.2)
        assert "amd.com/gpu" in m.store.peek() and updates == []
        await p1.stop()  # old endpoint was replaced; its stop must not remove capacity
        await asyncio.sleep(0.2)
        assert "amd.com/gpu" in m.store.peek()
        # plugin death: resource removed and reported once
        await p2.stop()
        await wait_for(lambda: "example.com/fpga" not in m.store.peek())
        cap, removed = m.get_capacity()
        assert removed == ["example.com/fpga"] and m.get_capacity()[1] == []
        assert b'kubelet_device_plugin_registration_count{resource_name="amd.com/gpu"} 2.0' in render(reg)
        await p1b.stop()
        await m.stop()
    run(go())


def test_registration_rejects_wrong_domain_and_version():
    async def go():
        root = short_tmp()
        m = await ManagerImpl(root).start()
        bad = await StubDevicePlugin("other.com/gpu", devs("x"), plugins_dir=root, sock_name="x").start()
        os.makedirs(os.path.join(root, "amd.com"), exist_ok=True)
        # plugin claims other.com/gpu but lives under amd.com/
        bad2 = StubDevicePlugin("other.com/gpu", devs("x"), plugins_dir=os.path.join(root, "_"), sock_name="y")
        bad2.socket = os.path.join(root, "amd.com", "y.sock")
        await bad2.start()
        old = await StubDevicePlugin("amd.com/old", devs("x"), plugins_dir=root, sock_name="old",
                                     supported_versions=("v1alpha1",)).start()
        await bad.wait_for_registration()
        with pytest.raises(RuntimeError):
            await bad2.wait_for_registration()
        with pytest.raises(RuntimeError):
            await old.wait_for_registration()
        await wait_for(lambda: "other.com/gpu" in m.store.peek())
        assert "amd.com/old" not in m.store.peek()
        for p in (bad, bad2, old):
            await p.stop()
        await m.stop()
    run(go())


def gpu_pod(ids, uid="u1"):
    return {"metadata": {"name": "p", "namespace": "default", "uid": uid},
            "spec": {"containers": [{"name": "c", "extendedResourceRequests": ["g"]}, {"name": "side"}],
                     "extendedResources": [{"name": "g", "resources": {"limits": {"amd.com/gpu": str(len(ids))}},
                                            "assigned": ids}]}}


def test_admit_and_init_container_with_amd_plugin():
    async def go():
        root = short_tmp()
        fb = FakeBackend()
        plugin = AMDGPUPlugin(fb, plugins_dir=root, health_interval=0.05)
        pods = []
        m = await ManagerImpl(root, active_pods=lambda: pods).start()
        await plugin.start()
        await plugin.wait_for_registration()
        await wait_for(lambda: len(m.store.peek().get("amd.com/gpu", {}).get("resources", {})) == 8)
        dev = m.store.peek()["amd.com/gpu"]["resources"]["GPU-5b4a00c0d1e2f3a0"]
        assert dev["attributes"]["amd.com/gpu-type"] == "MI355X"
        assert dev["attributes"]["amd.com/gpu-memory"] == str(288 * 1024)
        assert dev["attributes"]["amd.com/numa-node"] == "0" and dev["attributes"]["amd.com/gfx"] == "gfx950"
        assert "amd.com/gpu-topology" in m.plugin_labels
        ids = ["GPU-5b4a00c0d1e2f3a0", "GPU-5b4a01c0d1e2f3a1"]
        pod = gpu_pod(ids)
        pods.append(pod)
        await m.admit_pod(pod)
        assert m.pod_resources(pod) == {"amd.com/gpu-devices": ",".join(ids)}
        opts = await m.init_container(pod, pod["spec"]["containers"][0])
        assert opts["envs"]["ROCR_VISIBLE_DEVICES"] == "GPU-5b4a00c0d1e2f3a0,GPU-5b4a01c0d1e2f3a1"
        assert [d["host_path"] for d in opts["devices"]] == ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/card1",
                                                             "/dev/dri/renderD129", "/dev/dri/card2"]
        assert (await m.init_container(pod, pod["spec"]["containers"][1]))["devices"] == []
        # health flip via injected ECC error → Unhealthy pushed → admission refuses
        fb.inject_ecc(1)
        await wait_for(lambda: m.store.peek()["amd.com/gpu"]["resources"]["GPU-5b4a01c0d1e2f3a1"]["health"] == "Unhealthy")
        with pytest.raises(AdmissionError):
            await m.admit_pod(gpu_pod(ids, "u2"))
        with pytest.raises(AdmissionError):
            await m.admit_pod(gpu_pod(["GPU-nope"], "u3"))
        # lazy delete of dead pods' cached annotations
        pods.clear()
        await m.admit_pod({"metadata": {"uid": "u4"}, "spec": {"containers": [{"name": "c"}]}})
        assert m.pod_resources(pod) == {}
        await plugin.stop()
        await m.stop()
    run(go())


def test_v1beta1_adapter_registration():
    async def go():
        root = short_tmp()
        ksock = os.path.join(root, "dp", "kubelet.sock")
        m = await ManagerImpl(os.path.join(root, "plugins"), v1beta1_socket=ksock).start()
        p = StubDevicePlugin("vendor.com/acc", devs("a0", "a1"), plugins_dir=os.path.join(root, "x"))
        p.socket = os.path.join(root, "dp", "acc.sock")
        await p.start()
        await p.register_v1beta1(ksock)
        await wait_for(lambda: len(m.store.peek().get("vendor.com/acc", {}).get("resources", {})) == 2)
        pod = {"metadata": {"uid": "x", "name": "p"}, "spec": {"containers": [{"name": "c", "extendedResourceRequests": ["r"]}],
               "extendedResources": [{"name": "r", "resources": {"limits": {"vendor.com/acc": "1"}}, "assigned": ["a1"]}]}}
        await m.admit_pod(pod)
        opts = await m.init_container(pod, pod["spec"]["containers"][0])
        assert opts["envs"]["STUB_DEVICES"] == "a1"
        await p.stop()
        await m.stop()
    run(go())


def test_merge_container_specs_first_wins():
    out = merge_container_specs([
        {"envs": {"A": "1"}, "devices": [{"container_path": "/dev/x", "host_path": "/dev/x"}], "annotations": {"k": "1"}},
        {"envs": {"A": "2", "B": "3"}, "devices": [{"container_path": "/dev/x", "host_path": "/dev/y"}], "annotations": {"k": "2"}},
    ])
    assert out["envs"] == {"A": "1", "B": "3"} and len(out["devices"]) == 1 and out["annotations"] == {"k": "1"}


def test_topology_label_costs_scale_with_reported_xgmi_bandwidth():
    """Where amd-smi reports every pair's xGMI bandwidth the link cost is inverse to it (the
    fastest pair costs 15); otherwise the driver's link weight is used as is."""
    import json
    from amdkube.deviceplugin.amd import topology_label
    from amdkube.smi import FakeBackend
    fb = FakeBackend(n=4)
    gpus, topo = fb.gpus(), fb.topology()
    plain = json.loads(topology_label(gpus, topo))
    for i, row in enumerate(topo):
        for j, e in enumerate(row):
            if i != j:
                e["max_bw_mbps"] = 64000 if {i, j} != {0, 3} else 32000
    bw = json.loads(topology_label(gpus, topo))
    assert bw["link"][0][1] == 15 and bw["link"][0][3] == bw["link"][3][0] == 30
    assert all(bw["link"][i][i] == 0 for i in range(4))
    assert plain["link"] != bw["link"] and plain["ids"] == bw["ids"]
