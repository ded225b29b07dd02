"""DeviceManager (`ManagerImpl`) — the kubelet-side hub of the device-plugin machinery.

Reference pkg/kubelet/cm/devicemanager/: types.go:31-44 (Manager interface), manager.go
:97-148 (Start: watcher + run loop, domain = dir name :129-130), :152-176 (AdmitPod:
lazyPodDelete, HasDevices per assigned list, one AdmitPod RPC per resource, latency
metric, annotation cache), :245-291 (InitContainer: group the container's
extendedResourceRequests by resource, one RPC per plugin, merge), :187-190 (GetCapacity),
:318-339 (Stop, 5 s); manager_stub.go:25-71 (no-op when the DevicePlugins gate is off);
metrics pkg/kubelet/metrics/metrics.go:48-49,137-152.

Deliberate fixes: #3 (no cache write / nil deref on a failed AdmitPod), #4 (AdmitPod is
bounded by the plugin's init timeout), #12 (registration_count is actually incremented).
Also serves the upstream v1beta1 `Registration` socket so stock plugins can register.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time

import grpc

from ...api.helpers import (pod_extended_resource, pod_extended_resource_name, ExtendedResourceError)
from ...grpcdesc.deviceplugin import DEVICE_PLUGINS_PATH, V1BETA1 as B
from ...utils.metrics import Counter
from ...utils.quantiles import QuantileSummary as Summary
from .endpoint import EndpointHandler, RegistrationError
from .run_options import merge_container_specs
from .stores import EndpointStore, ManagerStore, PodResourceCache
from .watcher import PluginWatcher

log = logging.getLogger("amdkube.devicemanager")


class AdmissionError(Exception):
    def __init__(self, reason: str, message: str):
        super().__init__(message)
        self.reason, self.message = reason, message


def container_device_requests(pod: dict, container: dict) -> dict[str, list[str]]:
    """resource name -> assigned device IDs for one container (InitContainer grouping)."""
    out: dict[str, list[str]] = {}
    for ref in container.get("extendedResourceRequests") or []:
        pres = pod_extended_resource(pod, ref)
        if pres is None:
            continue
        try:
            rname = pod_extended_resource_name(pres)
        except ExtendedResourceError:
            continue
        out.setdefault(rname, []).extend(pres.get("assigned") or [])
    return out


class ManagerImpl:
    def __init__(self, plugins_dir: str = DEVICE_PLUGINS_PATH, active_pods=None, registry=None,
                 v1beta1_socket: str | None = None, use_inotify: bool = True):
        self.plugins_dir = plugins_dir
        self.active_pods = active_pods or (lambda: [])
        self.store = ManagerStore()
        self.endpoints = EndpointStore()
        self.cache = PodResourceCache()
        self.handler = EndpointHandler(self.endpoints, self.store.update_capacity, on_registered=self._registered)
        self.watcher = PluginWatcher(plugins_dir, use_inotify=use_inotify)
        self.v1beta1_socket = v1beta1_socket
        self._tasks: list[asyncio.Task] = []
        self._v1b_server = None
        self.plugin_labels: dict[str, str] = {}
        self.registration_errors: list[str] = []
        self.m_reg = self.m_alloc = None
        if registry is not None:
            self.m_reg = Counter("kubelet_device_plugin_registration_count", "Cumulative number of device plugin registrations. Broken down by resource name.",
                                 ["resource_name"], registry=registry)
            self.m_alloc = Summary("kubelet_device_plugin_alloc_latency_microseconds", "Latency in microseconds to serve a device plugin Allocation request. Broken down by resource name.",
                                   ["resource_name"], registry=registry)

    # ---------------------------------------------------------------- lifecycle
    async def start(self):
        await self.watcher.start()
        self._initial = set(self.watcher._known)  # sockets that existed before this kubelet started
        self._settled: set[str] = set()
        self._tasks.append(asyncio.create_task(self._run(), name="devicemanager-run"))
        self._tasks.append(asyncio.create_task(self._run_removed(), name="devicemanager-removed"))
        if self.v1beta1_socket:
            await self._serve_v1beta1()
        return self

    async def stop(self):
        await self.watcher.stop()
        for t in self._tasks:
            t.cancel()
        await self.handler.stop(timeout=5.0)
        if self._v1b_server is not None:
            await self._v1b_server.stop(0.5)

    async def _run(self):
        while True:
            path = await self.watcher.added.get()
            domain = os.path.basename(os.path.dirname(path))
            log.info("new device plugin socket %s (domain %s)", path, domain)
            asyncio.create_task(self._add(path, domain))

    async def _add(self, path, domain, kind="v1alpha2"):
        try:
            e = await self.handler.new_endpoint(path, domain, kind)
            # settled once the first ListAndWatch snapshot has been applied
            for _ in range(100):
                if e.store.devs() or e.ch.get_state() not in (grpc.ChannelConnectivity.READY, grpc.ChannelConnectivity.IDLE):
                    break
                await asyncio.sleep(0.01)
        except RegistrationError as e:
            self.registration_errors.append(str(e))
            log.warning("device plugin registration failed: %s", e)
        finally:
            getattr(self, "_settled", set()).add(path)

    async def wait_initial_registration(self, timeout: float = 5.0):
        """Kubelet restart: give plugins whose sockets already existed a bounded grace period to
        re-register before pods are (re-)admitted (their devices must be known by then)."""
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end and not self._initial <= self._settled:
            await asyncio.sleep(0.02)

    async def _run_removed(self):
        while True:
            path = await self.watcher.removed.get()
            log.info("device plugin socket %s removed", path)  # the endpoint's stream end handles cleanup

    def _registered(self, e):
        self.plugin_labels.update(e.labels)
        if self.m_reg is not None:
            self.m_reg.labels(e.resource_name).inc()

    async def _serve_v1beta1(self):
        os.makedirs(os.path.dirname(self.v1beta1_socket), exist_ok=True)
        if os.path.exists(self.v1beta1_socket):
            os.unlink(self.v1beta1_socket)
        mgr = self

        class Reg:
            async def Register(self, req, ctx):
                path = os.path.join(os.path.dirname(mgr.v1beta1_socket), req.endpoint)
                asyncio.create_task(mgr._add(path, req.resource_name, "v1beta1"))
                return B.Empty()
        self._v1b_server = grpc.aio.server()
        self._v1b_server.add_generic_rpc_handlers((B.Registration.handler(Reg()),))
        self._v1b_server.add_insecure_port("unix://" + self.v1beta1_socket)
        await self._v1b_server.start()

    # ------------------------------------------------------------ capacity
    def get_capacity(self):
        return self.store.get_capacity()

    def has_devices(self, rname, ids):
        return self.store.has_devices(rname, ids)

    # ------------------------------------------------------------ admission
    def _lazy_pod_delete(self):
        active = {((p.get("metadata") or {}).get("uid")) for p in self.active_pods()}
        for uid in self.cache.uids():
            if uid not in active:
                self.cache.delete(uid)

    async def admit_pod(self, pod: dict):
        """Raise AdmissionError if the pod's assigned devices are missing/unhealthy or a plugin rejects it."""
        self._lazy_pod_delete()
        spec = pod.get("spec") or {}
        per_res: dict[str, dict[str, dict[str, list[str]]]] = {}
        for pres in spec.get("extendedResources") or []:
            try:
                rname = pod_extended_resource_name(pres)
            except ExtendedResourceError as e:
                raise AdmissionError("UnexpectedAdmissionError", str(e))
            ids = pres.get("assigned") or []
            if not ids:
                raise AdmissionError("UnexpectedAdmissionError",
                                     f"extended resource {pres.get('name')} ({rname}) has no assigned devices")
            ok, why = self.store.has_devices(rname, ids)
            if not ok:
                raise AdmissionError("UnexpectedAdmissionError", why)
        for kind in ("initContainers", "containers"):
            for c in spec.get(kind) or []:
                for rname, ids in container_device_requests(pod, c).items():
                    per_res.setdefault(rname, {"containers": {}, "initContainers": {}})[kind][c["name"]] = ids
        uid = (pod.get("metadata") or {}).get("uid", "")
        name = (pod.get("metadata") or {}).get("name", "")
        for rname, groups in per_res.items():
            e = self.endpoints.endpoint(rname)
            if e is None:
                raise AdmissionError("UnexpectedAdmissionError", f"no device plugin registered for {rname}")
            t0 = time.perf_counter()
            try:
                ann = await e.admit_pod(name, groups["containers"], groups["initContainers"])
            except grpc.RpcError as err:
                raise AdmissionError("UnexpectedAdmissionError", f"device plugin {rname} rejected pod: {err.details()}")
            finally:
                if self.m_alloc is not None:
                    self.m_alloc.labels(rname).observe((time.perf_counter() - t0) * 1e6)
            self.cache.cache(uid, ann)

    async def init_container(self, pod: dict, container: dict) -> dict:
        """Run options for a container: merged envs/devices/mounts/annotations of every plugin."""
        specs = []
        for rname, ids in container_device_requests(pod, container).items():
            e = self.endpoints.endpoint(rname)
            if e is None:
                raise AdmissionError("DeviceUnavailable", f"no device plugin registered for {rname}")
            specs.append(await e.init_container(container["name"], ids))
        return merge_container_specs(specs)

    def pod_resources(self, pod: dict) -> dict:
        return self.cache.get((pod.get("metadata") or {}).get("uid", ""))


class ManagerStub:
    """DevicePlugins gate off: no devices, every admission passes."""

    plugin_labels: dict = {}

    async def start(self):
        return self

    async def stop(self):
        pass

    async def wait_initial_registration(self, timeout: float = 5.0):
        pass

    def get_capacity(self):
        return {}, []

    def has_devices(self, rname, ids):
        return False, "device plugins disabled"

    async def admit_pod(self, pod):
        if (pod.get("spec") or {}).get("extendedResources"):
            raise AdmissionError("UnexpectedAdmissionError", "device plugins are disabled on this node")

    async def init_container(self, pod, container):
        return {"envs": {}, "devices": [], "mounts": [], "annotations": {}}

    def pod_resources(self, pod):
        return {}
