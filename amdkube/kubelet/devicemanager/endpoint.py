"""Registration validator, per-plugin Endpoint and the EndpointHandler.

Reference (pkg/kubelet/):
  apis/pluginregistration/v1beta/validation.go:57-141 — dial the UDS (1 s), require
      GetSupportedVersions ∋ v1alpha2, GetPluginIdentity → resource name which must be an
      extended resource name starting with the socket's domain dir (:116-122), then
      PluginRegistrationStatus; each RPC has a 1 s timeout.
  cm/devicemanager/endpoint.go:63-174 — init via GetPluginInfo (1 s) → initTimeout; Run
      consumes ListAndWatch, diffs into the device store and fires the callback; on stream
      error fires "delete all" and closes; InitContainer uses the plugin's timeout; AdmitPod
      had none (fix #4: amdkube bounds it with the same timeout).
  cm/devicemanager/endpoint_handler.go:72-136 — NewEndpoint reuses the old device store on
      re-registration (no capacity flap), swaps, stops the old endpoint after handing it an
      always-empty store; trackEndpoint deletes the endpoint only if it was not replaced.
A v1beta1 (upstream) endpoint adapts Allocate to the InitContainer contract.
"""
from __future__ import annotations

import asyncio
import logging
import time

import grpc

from ...api.helpers import is_extended_resource_name
from ...grpcdesc.deviceplugin import REGISTRATION as R, V1ALPHA2 as P, V1BETA1 as B, VERSION
from .stores import AlwaysEmptyDeviceStore, DeviceStore
from ...utils.grpcutil import uds_channel

log = logging.getLogger("amdkube.devicemanager")

DIAL_TIMEOUT = 1.0
RPC_TIMEOUT = 1.0


class RegistrationError(Exception):
    pass


async def dial(path: str, timeout: float = DIAL_TIMEOUT) -> grpc.aio.Channel:
    ch = uds_channel(path)
    try:
        await asyncio.wait_for(ch.channel_ready(), timeout)
    except (asyncio.TimeoutError, Exception) as e:
        await ch.close()
        raise RegistrationError(f"failed to dial device plugin at {path}: {e!r}")
    return ch


class Validator:
    async def validate(self, path: str, domain: str) -> tuple[str, grpc.aio.Channel]:
        ch = await dial(path)
        try:
            ident = R.Identity.stub(ch)
            vers = await ident.GetSupportedVersions(R.GetSupportedVersionsRequest(), timeout=RPC_TIMEOUT)
            if VERSION not in list(vers.supported_versions):
                raise RegistrationError(f"plugin {path} does not support version {VERSION} (supports {list(vers.supported_versions)})")
            idr = await ident.GetPluginIdentity(R.GetPluginIdentityRequest(version=VERSION), timeout=RPC_TIMEOUT)
            name = idr.resource_name
            if not is_extended_resource_name(name):
                raise RegistrationError(f"invalid name of device plugin socket: {name} is not an extended resource name")
            if not name.startswith(domain):
                raise RegistrationError(f"resource name {name} does not start with the plugin domain {domain}")
            return name, ch
        except RegistrationError as e:
            await self.notify(ch, False, str(e))
            await ch.close()
            raise
        except grpc.RpcError as e:
            await ch.close()
            raise RegistrationError(f"registration RPC failed for {path}: {e.code()} {e.details()}")

    async def notify(self, ch, success: bool, error: str = ""):
        try:
            await R.Identity.stub(ch).PluginRegistrationStatus(R.RegistrationStatus(success=success, error=error),
                                                                timeout=RPC_TIMEOUT)
        except grpc.RpcError as e:
            log.debug("PluginRegistrationStatus failed: %s", e)


class Endpoint:
    """One registered v1alpha2 plugin."""

    def __init__(self, resource_name: str, socket: str, channel, store: DeviceStore | None, callback):
        self.resource_name, self.socket, self.ch = resource_name, socket, channel
        self.store = store or DeviceStore()
        self.callback = callback  # fn(rname, added, updated, deleted)
        self.stub = P.DevicePlugin.stub(channel)
        self.init_timeout = 10.0
        self.labels: dict[str, str] = {}
        self._stopped = asyncio.Event()
        self._stream = None
        self.started_at = time.time()

    async def init(self):
        info = await self.stub.GetPluginInfo(P.GetPluginInfoRequest(), timeout=RPC_TIMEOUT)
        if info.init_timeout > 0:
            self.init_timeout = float(info.init_timeout)
        self.labels = dict(info.labels)

    def set_store(self, store):
        self.store = store

    def devices(self):
        return self.store.devs()

    def healthy_devices(self):
        return self.store.healthy()

    async def run(self):
        try:
            self._stream = self.stub.ListAndWatch(P.ListAndWatchRequest())
            async for resp in self._stream:
                added, updated, deleted = self.store.update(resp.devices)
                if added or updated or deleted:
                    self.callback(self.resource_name, added, updated, deleted)
        except (grpc.RpcError, asyncio.CancelledError) as e:
            if not self._stopped.is_set():
                log.warning("ListAndWatch for %s ended: %s", self.resource_name, getattr(e, "details", lambda: e)())
        finally:
            devs = self.store.devs()
            self.store.update([])
            if devs:
                self.callback(self.resource_name, [], [], devs)
            await self.ch.close()

    async def admit_pod(self, pod_name: str, containers: dict, init_containers: dict) -> dict:
        req = P.AdmitPodRequest(pod_name=pod_name,
                                containers={k: P.Container(name=k, devices=v) for k, v in containers.items()},
                                init_containers={k: P.Container(name=k, devices=v) for k, v in init_containers.items()})
        resp = await self.stub.AdmitPod(req, timeout=self.init_timeout)
        return dict(resp.pod.annotations) if resp is not None and resp.HasField("pod") else {}

    async def init_container(self, name: str, devices: list[str]) -> dict:
        resp = await self.stub.InitContainer(P.InitContainerRequest(container=P.Container(name=name, devices=devices)),
                                             timeout=self.init_timeout)
        s = resp.spec
        return {"envs": dict(s.envs), "annotations": dict(s.annotations),
                "mounts": [{"container_path": m.container_path, "host_path": m.host_path, "read_only": m.read_only} for m in s.mounts],
                "devices": [{"container_path": d.container_path, "host_path": d.host_path, "permissions": d.permissions} for d in s.devices]}

    async def stop(self):
        self._stopped.set()
        if self._stream is not None:
            self._stream.cancel()
        await self.ch.close()


class V1Beta1Endpoint(Endpoint):
    """Adapter for upstream v1beta1 plugins: ListAndWatch(Empty), Allocate ≙ InitContainer."""

    def __init__(self, resource_name, socket, channel, store, callback):
        super().__init__(resource_name, socket, channel, store, callback)
        self.stub = B.DevicePlugin.stub(channel)

    async def init(self):
        await self.stub.GetDevicePluginOptions(B.Empty(), timeout=RPC_TIMEOUT)

    async def run(self):
        try:
            self._stream = self.stub.ListAndWatch(B.Empty())
            async for resp in self._stream:
                devs = [{"ID": d.ID, "health": d.health, "Attributes": {}} for d in resp.devices]
                added, updated, deleted = self.store.update(devs)
                if added or updated or deleted:
                    self.callback(self.resource_name, added, updated, deleted)
        except (grpc.RpcError, asyncio.CancelledError):
            pass
        finally:
            devs = self.store.devs()
            self.store.update([])
            if devs:
                self.callback(self.resource_name, [], [], devs)
            await self.ch.close()

    async def admit_pod(self, pod_name, containers, init_containers):
        return {}

    async def init_container(self, name, devices):
        await self.stub.PreStartContainer(B.PreStartContainerRequest(devices_ids=devices), timeout=self.init_timeout)
        resp = await self.stub.Allocate(B.AllocateRequest(container_requests=[B.ContainerAllocateRequest(devices_ids=devices)]),
                                        timeout=self.init_timeout)
        s = resp.container_responses[0]
        return {"envs": dict(s.envs), "annotations": dict(s.annotations),
                "mounts": [{"container_path": m.container_path, "host_path": m.host_path, "read_only": m.read_only} for m in s.mounts],
                "devices": [{"container_path": d.container_path, "host_path": d.host_path, "permissions": d.permissions} for d in s.devices]}


class EndpointHandler:
    def __init__(self, store, callback, validator: Validator | None = None, on_registered=None):
        self.store = store  # EndpointStore
        self.callback = callback
        self.validator = validator or Validator()
        self.on_registered = on_registered
        self.tasks: set[asyncio.Task] = set()

    async def new_endpoint(self, path: str, domain: str, kind: str = "v1alpha2") -> Endpoint:
        if kind == "v1beta1":
            ch = await dial(path)
            rname = domain  # v1beta1 registration names the resource explicitly
        else:
            rname, ch = await self.validator.validate(path, domain)
        old = self.store.endpoint(rname)
        dstore = old.store if old is not None and not isinstance(old.store, AlwaysEmptyDeviceStore) else None
        cls = V1Beta1Endpoint if kind == "v1beta1" else Endpoint
        e = cls(rname, path, ch, dstore, self.callback)
        try:
            await e.init()
        except grpc.RpcError as err:
            if kind != "v1beta1":
                await self.validator.notify(ch, False, f"GetPluginInfo failed: {err.details()}")
            await ch.close()
            raise RegistrationError(f"failed to initialise endpoint {rname}: {err.details()}")
        prev = self.store.swap_endpoint(e)
        if prev is not None:
            prev.set_store(AlwaysEmptyDeviceStore())
            await prev.stop()
        if kind != "v1beta1":
            await self.validator.notify(ch, True)
        if self.on_registered:
            self.on_registered(e)
        t = asyncio.create_task(self.track_endpoint(e), name=f"endpoint-{rname}")
        self.tasks.add(t)
        t.add_done_callback(self.tasks.discard)
        return e

    async def track_endpoint(self, e: Endpoint):
        await e.run()
        self.store.delete_endpoint(e.resource_name, only_if=e)

    async def stop(self, timeout: float = 5.0):
        eps = list(self.store.all().values())
        await asyncio.gather(*(e.stop() for e in eps), return_exceptions=True)
        if self.tasks:
            await asyncio.wait(list(self.tasks), timeout=timeout)
