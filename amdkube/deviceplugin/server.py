"""Device-plugin server framework (the plugin side of the kubelet ↔ plugin contract).

One gRPC (asyncio) server on a Unix socket at `<plugins-dir>/<domain>/<name>.sock`
(reference constants.go:32-35) serves three services at once:
  * deviceplugin.DevicePlugin v1alpha2 — GetPluginInfo / ListAndWatch / AdmitPod / InitContainer
    (pkg/kubelet/apis/deviceplugin/v1alpha/api.proto:17-31);
  * pluginregistration.Identity — GetSupportedVersions / GetPluginIdentity /
    PluginRegistrationStatus (pkg/kubelet/apis/pluginregistration/v1beta/api.proto:16-24);
  * v1beta1.DevicePlugin — the upstream surface (GetDevicePluginOptions / ListAndWatch /
    Allocate / PreStartContainer), so the same plugin also works with an upstream-style
    kubelet via Registration.Register (`register_v1beta1`).

Subclasses provide `admit_pod(pod_name, containers) -> annotations` and
`init_container(name, device_ids) -> ContainerSpec dict`. `update(devices)` pushes a new
device list to every open ListAndWatch stream (the reference stub's Update,
pkg/kubelet/cm/devicemanager/device_plugin_stub.go:220-222).
"""
from __future__ import annotations

import asyncio
import logging
import os

import grpc

from ..grpcdesc.deviceplugin import (DEVICE_PLUGINS_PATH, HEALTHY, REGISTRATION as R, V1ALPHA2 as P, V1BETA1 as B,
                                     VERSION, V1BETA1_VERSION)
from ..utils.grpcutil import uds_channel

log = logging.getLogger("amdkube.deviceplugin")


def socket_path(resource_name: str, plugins_dir: str = DEVICE_PLUGINS_PATH, sock_name: str | None = None) -> str:
    domain, _, name = resource_name.partition("/")
    return os.path.join(plugins_dir, domain, (sock_name or name or "plugin") + ".sock")


class DevicePluginServer:
    def __init__(self, resource_name: str, plugins_dir: str = DEVICE_PLUGINS_PATH, init_timeout: int = 10,
                 sock_name: str | None = None, labels: dict | None = None, supported_versions=(VERSION,)):
        self.resource_name = resource_name
        self.socket = socket_path(resource_name, plugins_dir, sock_name)
        self.init_timeout = init_timeout
        self.labels = dict(labels or {})
        self.supported_versions = list(supported_versions)
        self.devices: list[dict] = []  # {"ID", "health", "Attributes"}
        self._streams: set[asyncio.Queue] = set()
        self.server: grpc.aio.Server | None = None
        self.registered = asyncio.Event()
        self.registration_error = ""
        self.admit_calls = 0
        self.init_calls = 0
        self.list_and_watch_opened = 0

    # ------------------------------------------------------------ lifecycle
    async def start(self):
        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        if os.path.exists(self.socket):
            os.unlink(self.socket)
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((
            P.DevicePlugin.handler(_V1Alpha2(self)),
            R.Identity.handler(_Identity(self)),
            B.DevicePlugin.handler(_V1Beta1(self)),
        ))
        self.server.add_insecure_port("unix://" + self.socket)
        await self.server.start()
        log.info("device plugin %s serving on %s", self.resource_name, self.socket)
        return self

    async def stop(self, grace: float = 0.5):
        for q in list(self._streams):
            q.put_nowait(None)
        if self.server is not None:
            await self.server.stop(grace)
            self.server = None
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass

    async def wait_for_registration(self, timeout: float = 10.0):
        await asyncio.wait_for(self.registered.wait(), timeout)
        if self.registration_error:
            raise RuntimeError(self.registration_error)

    # --------------------------------------------------------------- devices
    def update(self, devices: list[dict]):
        self.devices = [dict(d) for d in devices]
        for q in list(self._streams):
            q.put_nowait(self.devices)

    def set_health(self, device_id: str, health: str):
        devs = [dict(d, health=health) if d["ID"] == device_id else d for d in self.devices]
        if devs != self.devices:
            self.update(devs)

    # ------------------------------------------------------------- overridable
    def admit_pod(self, pod_name: str, containers: dict[str, list[str]], init_containers: dict[str, list[str]]) -> dict:
        return {}

    def init_container(self, name: str, device_ids: list[str]) -> dict:
        """-> {"envs": {}, "mounts": [{container_path, host_path, read_only}], "devices": [...], "annotations": {}}"""
        return {}

    # ------------------------------------------------------------- helpers
    @staticmethod
    def _pb_devices(devs):
        return [P.Device(ID=d["ID"], health=d.get("health", HEALTHY), Attributes=d.get("Attributes") or {}) for d in devs]

    async def _stream(self):
        q: asyncio.Queue = asyncio.Queue()
        self._streams.add(q)
        self.list_and_watch_opened += 1
        q.put_nowait(self.devices)
        try:
            while True:
                devs = await q.get()
                if devs is None:
                    return
                yield devs
        finally:
            self._streams.discard(q)

    async def register_v1beta1(self, kubelet_socket: str, endpoint: str | None = None):
        """Upstream-style registration: call Registration.Register on the kubelet socket."""
        async with uds_channel(kubelet_socket) as ch:
            stub = B.Registration.stub(ch)
            await stub.Register(B.RegisterRequest(version=V1BETA1_VERSION, endpoint=endpoint or os.path.basename(self.socket),
                                                  resource_name=self.resource_name,
                                                  options=B.DevicePluginOptions(pre_start_required=True)), timeout=5)


def _spec_pb(spec: dict) -> P.ContainerSpec:
    return P.ContainerSpec(
        envs=spec.get("envs") or {},
        mounts=[P.Mount(container_path=m["container_path"], host_path=m["host_path"], read_only=bool(m.get("read_only")))
                for m in spec.get("mounts") or []],
        devices=[P.DeviceSpec(container_path=d["container_path"], host_path=d["host_path"],
                              permissions=d.get("permissions", "rw")) for d in spec.get("devices") or []],
        annotations=spec.get("annotations") or {})


class _V1Alpha2:
    def __init__(self, s: DevicePluginServer):
        self.s = s

    async def GetPluginInfo(self, req, ctx):
        return P.GetPluginInfoResponse(init_timeout=self.s.init_timeout, labels=self.s.labels)

    async def ListAndWatch(self, req, ctx):
        async for devs in self.s._stream():
            yield P.ListAndWatchResponse(devices=self.s._pb_devices(devs))

    async def AdmitPod(self, req, ctx):
        self.s.admit_calls += 1
        ann = self.s.admit_pod(req.pod_name, {k: list(v.devices) for k, v in req.containers.items()},
                               {k: list(v.devices) for k, v in req.init_containers.items()})
        if asyncio.iscoroutine(ann):
            ann = await ann
        return P.AdmitPodResponse(pod=P.PodSpec(annotations=ann or {}))

    async def InitContainer(self, req, ctx):
        self.s.init_calls += 1
        spec = self.s.init_container(req.container.name, list(req.container.devices))
        if asyncio.iscoroutine(spec):
            spec = await spec
        return P.InitContainerResponse(spec=_spec_pb(spec or {}))


class _Identity:
    def __init__(self, s: DevicePluginServer):
        self.s = s

    async def GetSupportedVersions(self, req, ctx):
        return R.GetSupportedVersionsResponse(supported_versions=self.s.supported_versions)

    async def GetPluginIdentity(self, req, ctx):
        return R.GetPluginIdentityResponse(resource_name=self.s.resource_name)

    async def PluginRegistrationStatus(self, req, ctx):
        self.s.registration_error = "" if req.success else (req.error or "registration failed")
        self.s.registered.set()
        if req.success:
            log.info("plugin %s registered with kubelet", self.s.resource_name)
        else:
            log.warning("plugin %s registration failed: %s", self.s.resource_name, req.error)
        return R.Empty()


class _V1Beta1:
    def __init__(self, s: DevicePluginServer):
        self.s = s

    async def GetDevicePluginOptions(self, req, ctx):
        return B.DevicePluginOptions(pre_start_required=True)

    async def ListAndWatch(self, req, ctx):
        async for devs in self.s._stream():
            yield B.ListAndWatchResponse(devices=[B.Device(ID=d["ID"], health=d.get("health", HEALTHY)) for d in devs])

    async def Allocate(self, req, ctx):
        out = []
        for cr in req.container_requests:
            spec = self.s.init_container("", list(cr.devices_ids))
            if asyncio.iscoroutine(spec):
                spec = await spec
            spec = spec or {}
            out.append(B.ContainerAllocateResponse(
                envs=spec.get("envs") or {}, annotations=spec.get("annotations") or {},
                mounts=[B.Mount(container_path=m["container_path"], host_path=m["host_path"], read_only=bool(m.get("read_only")))
                        for m in spec.get("mounts") or []],
                devices=[B.DeviceSpec(container_path=d["container_path"], host_path=d["host_path"],
                                      permissions=d.get("permissions", "rw")) for d in spec.get("devices") or []]))
        return B.AllocateResponse(container_responses=out)

    async def PreStartContainer(self, req, ctx):
        return B.PreStartContainerResponse()


class StubDevicePlugin(DevicePluginServer):
    """In-process fake plugin (reference DevicePluginStub, device_plugin_stub.go:41-277):
    static devices, `update()` to push changes, records every AdmitPod/InitContainer call and
    can inject faults (delay InitContainer, fail AdmitPod, break the stream)."""

    def __init__(self, resource_name: str, devices: list[dict] | None = None, plugins_dir: str = DEVICE_PLUGINS_PATH,
                 sock_name: str | None = None, init_timeout: int = 5, labels: dict | None = None,
                 supported_versions=(VERSION,)):
        super().__init__(resource_name, plugins_dir, init_timeout, sock_name, labels, supported_versions)
        self.devices = [dict(d) for d in devices or []]
        self.admitted: list[tuple] = []
        self.inited: list[tuple] = []
        self.init_delay = 0.0
        self.fail_admit = False

    def admit_pod(self, pod_name, containers, init_containers):
        self.admitted.append((pod_name, containers, init_containers))
        if self.fail_admit:
            raise RuntimeError("injected AdmitPod failure")
        return {f"{self.resource_name.split('/')[0]}/admitted": pod_name}

    async def init_container(self, name, device_ids):
        self.inited.append((name, device_ids))
        if self.init_delay:
            await asyncio.sleep(self.init_delay)
        return {"envs": {"STUB_DEVICES": ",".join(device_ids)},
                "devices": [{"container_path": f"/dev/stub-{d}", "host_path": f"/dev/null", "permissions": "rw"} for d in device_ids],
                "mounts": [{"container_path": "/usr/local/stub", "host_path": "/tmp", "read_only": True}],
                "annotations": {"stub/devices": ",".join(device_ids)}}
