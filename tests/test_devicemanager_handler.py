"""Endpoint / EndpointHandler / EndpointStore / PluginWatcher semantics, one test per reference
test:

  TestRun (pkg/kubelet/cm/devicemanager/endpoint_test.go:40-154)       -> test_endpoint_run_diff_semantics
  TestReRegistration (endpoint_handler_test.go:153-264, with the
    instrumented endpointStoreShim, endpoint_store_shim.go:33-60)       -> test_reregistration_hands_store_over_before_swap
  TestTrackEndpoint / TestHandlerNewEndpoint (endpoint_handler_test.go:30-151)
                                                                        -> test_track_endpoint_removes_only_its_own_endpoint
  TestEndpointStore / TestSwapEndpoint / TestDeleteEndpoint (endpoint_store_test.go:28-103)
                                                                        -> test_endpoint_store_swap_and_delete
  TestAlwaysEmptyDeviceStore (device_store_test.go:69)                 -> test_always_empty_store
  TestAddAndDeletePlugins (plugin_watcher_test.go:65-162)              -> test_watcher_domain_removal_emits_every_socket
"""
import asyncio
import os
import shutil
import socket

from amdkube.deviceplugin import StubDevicePlugin
from amdkube.kubelet.devicemanager import (AlwaysEmptyDeviceStore, DeviceStore, Endpoint, EndpointHandler, EndpointStore,
                                           PluginWatcher)
from amdkube.kubelet.devicemanager.endpoint import dial
from tests.conftest import run
from tests.test_devicemanager import devs, short_tmp, wait_for


def ids(xs):
    return sorted(x["ID"] for x in xs)


def test_endpoint_run_diff_semantics():
    async def go():
        root = short_tmp()
        p = await StubDevicePlugin("amd.com/gpu", devs("a", "b", "c"), plugins_dir=root, init_timeout=3).start()
        events = []
        e = Endpoint("amd.com/gpu", p.socket, await dial(p.socket), None,
                     lambda r, a, u, d: events.append((r, ids(a), ids(u), ids(d))))
        await e.init()
        assert e.init_timeout == 3.0
        task = asyncio.create_task(e.run())
        await wait_for(lambda: len(events) == 1)
        assert events[0] == ("amd.com/gpu", ["a", "b", "c"], [], [])
        # b -> Unhealthy (updated), c removed (deleted), d new (added): exactly one callback
        p.update(devs("a") + devs("b", health="Unhealthy") + devs("d"))
        await wait_for(lambda: len(events) == 2)
        assert events[1] == ("amd.com/gpu", ["d"], ["b"], ["c"])
        assert ids(e.devices()) == ["a", "b", "d"] and ids(e.healthy_devices()) == ["a", "d"]
        # an identical resend produces no callback
        p.update(devs("a") + devs("b", health="Unhealthy") + devs("d"))
        await asyncio.sleep(0.1)
        assert len(events) == 2
        spec = await e.init_container("ctr", ["a", "d"])
        assert spec["envs"] == {"STUB_DEVICES": "a,d"} and [d["container_path"] for d in spec["devices"]] == ["/dev/stub-a", "/dev/stub-d"]
        assert p.inited == [("ctr", ["a", "d"])]
        ann = await e.admit_pod("pod-1", {"ctr": ["a"]}, {})
        assert ann == {"amd.com/admitted": "pod-1"}
        # stream end (plugin stops) -> every device deleted through the callback
        await p.stop()
        await asyncio.wait_for(task, 5)
        assert events[-1] == ("amd.com/gpu", [], [], ["a", "b", "d"])
        assert e.devices() == []
    run(go())


class InstrumentedEndpointStore(EndpointStore):
    """endpointStoreShim: records what the new endpoint holds at the moment of the swap."""

    def __init__(self):
        super().__init__()
        self.swaps = []

    def swap_endpoint(self, e):
        old = self.endpoints.get(e.resource_name)
        self.swaps.append((e, old, e.store is (old.store if old is not None else None), ids(e.store.devs())))
        return super().swap_endpoint(e)


def test_reregistration_hands_store_over_before_swap():
    async def go():
        root = short_tmp()
        store = InstrumentedEndpointStore()
        events = []
        h = EndpointHandler(store, lambda r, a, u, d: events.append((ids(a), ids(u), ids(d))))
        p1 = await StubDevicePlugin("amd.com/gpu", devs("g0", "g1"), plugins_dir=root).start()
        e1 = await h.new_endpoint(p1.socket, "amd.com")
        await wait_for(lambda: events == [(["g0", "g1"], [], [])])
        p2 = await StubDevicePlugin("amd.com/gpu", devs("g0", "g1"), plugins_dir=root, sock_name="gpu-b").start()
        e2 = await h.new_endpoint(p2.socket, "amd.com")
        # the new endpoint already owned the old device store when it was swapped in ...
        new, old, same_store, held = store.swaps[-1]
        assert new is e2 and old is e1 and same_store and held == ["g0", "g1"]
        # ... and the old endpoint got the null store, so its shutdown deletes nothing
        assert isinstance(e1.store, AlwaysEmptyDeviceStore)
        await asyncio.sleep(0.2)
        assert events == [(["g0", "g1"], [], [])]  # exactly one callback: the registration
        assert store.endpoint("amd.com/gpu") is e2
        await p2.stop()
        await wait_for(lambda: len(events) == 2)
        assert events[-1] == ([], [], ["g0", "g1"])  # and exactly one at stop
        await p1.stop()
        await h.stop()
    run(go())


def test_track_endpoint_removes_only_its_own_endpoint():
    async def go():
        root = short_tmp()
        store = EndpointStore()
        h = EndpointHandler(store, lambda *a: None)
        p = await StubDevicePlugin("amd.com/gpu", devs("g0"), plugins_dir=root).start()
        e = await h.new_endpoint(p.socket, "amd.com")
        assert store.endpoint("amd.com/gpu") is e
        await p.stop()
        await wait_for(lambda: store.endpoint("amd.com/gpu") is None)
        # a replaced endpoint ending must not delete its replacement
        p1 = await StubDevicePlugin("amd.com/gpu", devs("g0"), plugins_dir=root).start()
        e1 = await h.new_endpoint(p1.socket, "amd.com")
        p2 = await StubDevicePlugin("amd.com/gpu", devs("g0"), plugins_dir=root, sock_name="gpu-b").start()
        e2 = await h.new_endpoint(p2.socket, "amd.com")
        await p1.stop()
        await asyncio.sleep(0.2)
        assert store.endpoint("amd.com/gpu") is e2 and e1 is not e2
        await p2.stop()
        await h.stop()
    run(go())


def test_endpoint_store_swap_and_delete():
    class E:
        def __init__(self, r):
            self.resource_name = r
    s = EndpointStore()
    a, b = E("x/a"), E("x/a")
    assert s.swap_endpoint(a) is None and s.endpoint("x/a") is a
    assert s.swap_endpoint(b) is a and s.endpoint("x/a") is b
    assert not s.delete_endpoint("x/a", only_if=a) and s.endpoint("x/a") is b
    assert s.delete_endpoint("x/a", only_if=b) and s.endpoint("x/a") is None
    assert not s.delete_endpoint("x/a")
    s.swap_endpoint(E("x/b"))
    assert list(s.all()) == ["x/b"]


def test_always_empty_store():
    s = AlwaysEmptyDeviceStore()
    assert s.update(devs("a", "b")) == ([], [], []) and s.devs() == []
    d = DeviceStore()
    d.update(devs("a"))
    assert d.update([]) == ([], [], [{"ID": "a", "health": "Healthy", "Attributes": {}}])


def test_watcher_domain_removal_emits_every_socket():
    async def go():
        root = short_tmp()
        w = await PluginWatcher(root).start()
        dom = os.path.join(root, "amd.com")
        os.makedirs(dom)
        await asyncio.sleep(0.05)
        socks = []
        for name in ("gpu.sock", "cpx.sock"):
            s = socket.socket(socket.AF_UNIX)
            s.bind(os.path.join(dom, name))
            socks.append(s)
        got = {await asyncio.wait_for(w.added.get(), 2) for _ in range(2)}
        assert got == {os.path.join(dom, "gpu.sock"), os.path.join(dom, "cpx.sock")}
        shutil.rmtree(dom)
        gone = {await asyncio.wait_for(w.removed.get(), 2) for _ in range(2)}
        assert gone == got
        # a domain dir created with sockets already inside is walked on creation
        dom2 = os.path.join(root, "example.com")
        tmp = os.path.join(root + "-stage")
        os.makedirs(tmp)
        s = socket.socket(socket.AF_UNIX)
        s.bind(os.path.join(tmp, "fpga.sock"))
        os.rename(tmp, dom2)
        assert await asyncio.wait_for(w.added.get(), 2) == os.path.join(dom2, "fpga.sock")
        await w.stop()
        shutil.rmtree(root, ignore_errors=True)
    run(go())
