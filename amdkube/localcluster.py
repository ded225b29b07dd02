"""In-process single-node cluster: apiserver + scheduler + controller-manager + rocshim +
AMD device plugin + kubelet on one event loop (the reference's integration framework
starts the master in-process over httptest, test/integration/framework/master_utils.go:174,
and hack/local-up-cluster.sh wires the same components as processes, :394-784).

Used by the integration tests, `bench.py` and `python -m amdkube local-up`.
"""
from __future__ import annotations

import asyncio
import logging
import os
import shutil
import tempfile

from .apiserver import APIServer
from .client import Client
from .deviceplugin.amd import make_plugins
from .kubelet.kubelet import Kubelet, KubeletConfig
from .runtime import RocShim
from .scheduler import Scheduler
from .smi import open_backend

log = logging.getLogger("amdkube.localcluster")


class LocalCluster:
    def __init__(self, gpus: str = "fake", n_gpus: int | None = None, node_name: str = "mi355x-node-0",
                 base_dir: str | None = None, with_controllers: bool = True, relist_period: float = 1.0,
                 node_status_update_frequency: float = 10.0, scheduler_kw: dict | None = None, isolation: str | None = None,
                 health_probe: str = "none", kubelet_kw: dict | None = None, with_kubelet: bool = True,
                 partition: str | None = None, resource_naming: str = "single", api_kw: dict | None = None,
                 controllers_kw: dict | None = None, shim_kw: dict | None = None, runtime: str = "rocshim"):
        self.gpus, self.n_gpus, self.node_name = gpus, n_gpus, node_name
        self.partition, self.resource_naming = partition, resource_naming
        self.plugins: list = []
        self._own_dir = base_dir is None
        self.base = base_dir or tempfile.mkdtemp(prefix="ak-", dir="/tmp")
        self.with_controllers = with_controllers
        self.relist_period = relist_period
        self.nsuf = node_status_update_frequency
        self.scheduler_kw = scheduler_kw or {}
        self.kubelet_kw = kubelet_kw or {}
        # a node on real GPUs isolates devices with the strongest mechanism it has (rocshim
        # isolation=auto); the fake backend keeps the advisory env mode unless asked
        self.isolation = isolation or ("env" if gpus in ("fake", "none") else "auto")
        self.health_probe = health_probe
        self.with_kubelet = with_kubelet
        self.api_kw, self.controllers_kw, self.shim_kw = api_kw or {}, controllers_kw or {}, shim_kw or {}
        self.runtime = runtime        # "rocshim" (default) or "rkt" (runtime/rktshim.py; shim_kw: rkt=…)
        self.api = self.client = self.scheduler = self.controllers = self.shim = self.plugin = self.kubelet = None
        self.backend = None

    async def start(self):
        b = self.base
        self.api = await APIServer(**self.api_kw).start()
        self.client = Client(self.api.url, token=self.api.loopback_token, pool=256)
        self.scheduler = await Scheduler(Client(self.api.url, token=self.api.loopback_token, pool=256), **self.scheduler_kw).start()
        if self.with_controllers:
            from .controllers import ControllerManager
            self.controllers = await ControllerManager(Client(self.api.url, token=self.api.loopback_token), **self.controllers_kw).start()
        if not self.with_kubelet:
            return self
        if self.runtime == "rkt":
            from .runtime.rktshim import RktShim
            self.shim = await RktShim(os.path.join(b, "rocshim.sock"), os.path.join(b, "rktshim"), **self.shim_kw).start()
        else:
            self.shim = await RocShim(os.path.join(b, "rocshim.sock"), os.path.join(b, "rocshim"),
                                      hooks_dir=os.path.join(b, "hooks.d"), isolation=self.isolation, **self.shim_kw).start()
        if self.gpus != "none":
            self.backend = open_backend(self.gpus, n=self.n_gpus, partition=self.partition)
            self.plugins = make_plugins(self.backend, self.resource_naming, plugins_dir=os.path.join(b, "plugins"),
                                        health_interval=5.0, health_probe=self.health_probe,
                                        health_state=os.path.join(b, "amdkube-gpu-health.json"))
            self.plugin = self.plugins[0]
        kw = dict(self.kubelet_kw)
        # the in-process harness mounts nothing unless a test asks for real mounts (and then
        # stop() unmounts whatever is left under its directory)
        kw.setdefault("volume_mounter", "none")
        cfg = KubeletConfig(node_name=self.node_name, root_dir=os.path.join(b, "kubelet"), plugins_dir=os.path.join(b, "plugins"),
                            cri_socket=os.path.join(b, "rocshim.sock"), port=0, relist_period=self.relist_period,
                            node_status_update_frequency=self.nsuf, **kw)
        self.kubelet = await Kubelet(Client(self.api.url, token=self.api.loopback_token, pool=128), cfg, smi_backend=self.backend).start()
        for p in self.plugins:
            await p.start()
            await p.wait_for_registration(10)
        return self

    async def wait_gpus(self, n: int, timeout: float = 15.0, resource: str = "amd.com/gpu"):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end:
            node = await self.client.get_or_none("nodes", self.node_name)
            if node and int(((node.get("status") or {}).get("allocatable") or {}).get(resource, 0)) >= n:
                ext = (node.get("status") or {}).get("extendedResources") or {}
                if len(((ext.get(resource) or {}).get("resources") or {})) >= n:
                    return node
            await asyncio.sleep(0.05)
        raise TimeoutError(f"node never advertised {n} GPUs")

    async def stop(self):
        for comp in (self.kubelet, *self.plugins):
            if comp is not None:
                try:
                    await comp.stop()
                except Exception as e:
                    log.debug("stop %s: %r", comp, e)
        if self.shim is not None:
            await self.shim.stop(kill_pods=True)
        for comp in (self.controllers, self.scheduler):
            if comp is not None:
                await comp.stop()
                await comp.client.close()
        if self.kubelet is not None:
            await self.kubelet.client.close()
        if self.client is not None:
            await self.client.close()
        if self.api is not None:
            await self.api.stop()
        if self.backend is not None:
            try:
                self.backend.close()
            except Exception:
                pass
        if self._own_dir:
            from .volume.mount import unmount_under
            unmount_under(self.base)
            shutil.rmtree(self.base, ignore_errors=True)

    async def __aenter__(self):
        return await self.start()

    async def __aexit__(self, *exc):
        await self.stop()


async def wait_pod(client: Client, ns: str, name: str, phases=("Running",), timeout: float = 30.0) -> dict:
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    last = None
    while loop.time() < end:
        last = await client.get_or_none("pods", name, ns)
        if last and (last.get("status") or {}).get("phase") in phases:
            return last
        await asyncio.sleep(0.02)
    raise TimeoutError(f"pod {ns}/{name} did not reach {phases}: {(last or {}).get('status')}")
