"""Hollow nodes (kubemark) with simulated MI355X GPUs.

Reference: cmd/kubemark/hollow-node.go:90-167 and pkg/kubemark/hollow_kubelet.go:33-75 run a
real kubelet against fake docker/cadvisor — but with the stub container manager, so hollow
nodes have NO GPUs (pkg/kubelet/cm/container_manager_stub.go:73-90; SURVEY §4.3 gap).

An amdkube hollow node is the real Kubelet + a real (in-process) AMD device plugin on the
fake 8×MI355X backend + a fake CRI runtime (FakeRuntime: sandboxes/containers are records,
"running" containers exit after `run_seconds`), so density and scheduling benchmarks exercise
the full device path (registration → ListAndWatch → capacity → AdmitPod → InitContainer) on
as many nodes as the host can simulate.
"""
from __future__ import annotations

import asyncio
import os
import tempfile
import time
import uuid

import grpc

from ..client import Client
from ..deviceplugin.amd import make_plugins
from ..grpcdesc.cri import API_VERSION, CRI as C, EVENT_TRAILER
from ..kubelet.kubelet import Kubelet, KubeletConfig
from ..smi import FakeBackend


class FakeRuntime:
    """In-memory CRI server (reference pkg/kubelet/apis/cri/testing/fake_runtime_service.go).

    It speaks the same evented contract as rocshim (the runtime a real MI355X node runs): every
    lifecycle change emits a ContainerEventResponse with the sandbox's full status and all its
    container statuses, and mutating calls return the `amdkube-event` trailer naming the newest
    event of their sandbox, so a hollow kubelet does the same (list-free) work per pod as a
    real one."""

    def __init__(self, socket_path: str, run_seconds: float | None = None):
        self.socket = socket_path
        self.run_seconds = run_seconds
        self.sandboxes: dict[str, dict] = {}
        self.containers: dict[str, dict] = {}
        self.server = None
        self.streams: set[asyncio.Queue] = set()
        self.calls: dict[str, int] = {}
        self._last_ev: dict[str, int] = {}
        self._removed_meta: dict[str, object] = {}
        self.node_ip = "127.0.0.1"

    def _count(self, name):
        self.calls[name] = self.calls.get(name, 0) + 1

    async def start(self):
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((C.RuntimeService.handler(self), C.ImageService.handler(_FakeImages())))
        self.server.add_insecure_port("unix://" + self.socket)
        await self.server.start()
        return self

    async def stop(self):
        if self.server:
            await self.server.stop(0.2)

    def _emit(self, cid, sid, etype):
        if not self.streams:
            return
        ts = max(time.time_ns(), self._last_ev.get(sid, 0) + 1)   # strictly increasing per sandbox
        self._last_ev[sid] = ts
        s = self.sandboxes.get(sid)
        if s is None:     # removed: identity only
            meta = self._removed_meta.pop(sid, None)
            sst = C.PodSandboxStatus(id=sid, metadata=meta) if meta is not None else C.PodSandboxStatus(id=sid)
            cst = []
        else:
            sst = C.PodSandboxStatus(network=C.PodSandboxNetworkStatus(ip=self.node_ip), **self._sb(sid, s))
            cst = [self._cstatus(x, c) for x, c in self.containers.items() if c["sid"] == sid]
        ev = C.ContainerEventResponse(container_id=cid, container_event_type=etype, created_at=ts,
                                      pod_sandbox_status=sst, containers_statuses=cst)
        for q in list(self.streams):
            q.put_nowait(ev)

    def _mark(self, ctx, sid):
        ts = self._last_ev.get(sid or "", 0)
        if sid and ts and sid not in self.sandboxes:
            self._last_ev.pop(sid, None)
        ctx.set_trailing_metadata(((EVENT_TRAILER, f"{sid}:{ts}" if sid and ts else ""),))

    async def Version(self, req, ctx):
        return C.VersionResponse(version=API_VERSION, runtime_name="fake", runtime_version="0.1", runtime_api_version="v1alpha1")

    async def Status(self, req, ctx):
        return C.StatusResponse(status=C.RuntimeStatus(conditions=[C.RuntimeCondition(type="RuntimeReady", status=True),
                                                                   C.RuntimeCondition(type="NetworkReady", status=True)]))

    async def RunPodSandbox(self, req, ctx):
        self._count("RunPodSandbox")
        sid = uuid.uuid4().hex
        self.sandboxes[sid] = {"config": req.config, "state": C.SANDBOX_READY, "created": time.time_ns()}
        self._emit(sid, sid, C.CONTAINER_STARTED_EVENT)
        self._mark(ctx, sid)
        return C.RunPodSandboxResponse(pod_sandbox_id=sid)

    async def StopPodSandbox(self, req, ctx):
        sid = req.pod_sandbox_id
        s = self.sandboxes.get(sid)
        if s:
            for cid, c in self.containers.items():
                if c["sid"] == sid and c["state"] == C.CONTAINER_RUNNING:
                    self._exit(cid, 137)
            if s["state"] != C.SANDBOX_NOTREADY:
                s["state"] = C.SANDBOX_NOTREADY
                self._emit(sid, sid, C.CONTAINER_STOPPED_EVENT)
        self._mark(ctx, sid)
        return C.StopPodSandboxResponse()

    async def RemovePodSandbox(self, req, ctx):
        sid = req.pod_sandbox_id
        s = self.sandboxes.pop(sid, None)
        for cid in [k for k, c in self.containers.items() if c["sid"] == sid]:
            del self.containers[cid]
        if s is not None:
            cfg = s["config"]
            self._removed_meta[sid] = cfg.metadata
            self._emit(sid, sid, C.CONTAINER_DELETED_EVENT)
        self._mark(ctx, sid)
        return C.RemovePodSandboxResponse()

    def _sb(self, sid, s):
        cfg = s["config"]
        return dict(id=sid, metadata=cfg.metadata, state=s["state"], created_at=s["created"], labels=cfg.labels,
                    annotations=cfg.annotations)

    async def PodSandboxStatus(self, req, ctx):
        self._count("PodSandboxStatus")
        s = self.sandboxes.get(req.pod_sandbox_id)
        if s is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "not found")
        return C.PodSandboxStatusResponse(status=C.PodSandboxStatus(**self._sb(req.pod_sandbox_id, s)))

    async def ListPodSandbox(self, req, ctx):
        self._count("ListPodSandbox")
        out = []
        for sid, s in self.sandboxes.items():
            f = req.filter
            if any(s["config"].labels.get(k) != v for k, v in f.label_selector.items()):
                continue
            out.append(C.PodSandbox(**self._sb(sid, s)))
        return C.ListPodSandboxResponse(items=out)

    async def CreateContainer(self, req, ctx):
        self._count("CreateContainer")
        cid = uuid.uuid4().hex
        self.containers[cid] = {"sid": req.pod_sandbox_id, "config": req.config, "state": C.CONTAINER_CREATED,
                                "created": time.time_ns(), "started": 0, "finished": 0, "exit": 0}
        self._emit(cid, req.pod_sandbox_id, C.CONTAINER_CREATED_EVENT)
        self._mark(ctx, req.pod_sandbox_id)
        return C.CreateContainerResponse(container_id=cid)

    def _exit(self, cid, code):
        c = self.containers.get(cid)
        if c and c["state"] == C.CONTAINER_RUNNING:
            c["state"], c["finished"], c["exit"] = C.CONTAINER_EXITED, time.time_ns(), code
            self._emit(cid, c["sid"], C.CONTAINER_STOPPED_EVENT)

    async def StartContainer(self, req, ctx):
        c = self.containers[req.container_id]
        c["state"], c["started"] = C.CONTAINER_RUNNING, time.time_ns()
        self._emit(req.container_id, c["sid"], C.CONTAINER_STARTED_EVENT)
        if self.run_seconds is not None:
            asyncio.get_running_loop().call_later(self.run_seconds, self._exit, req.container_id, 0)
        self._mark(ctx, c["sid"])
        return C.StartContainerResponse()

    def _sid_of(self, cid):
        c = self.containers.get(cid)
        return c["sid"] if c is not None else None

    async def StopContainer(self, req, ctx):
        sid = self._sid_of(req.container_id)
        self._exit(req.container_id, 137)
        self._mark(ctx, sid)
        return C.StopContainerResponse()

    async def RemoveContainer(self, req, ctx):
        sid = self._sid_of(req.container_id)
        if self.containers.pop(req.container_id, None) is not None:
            self._emit(req.container_id, sid, C.CONTAINER_DELETED_EVENT)
        self._mark(ctx, sid)
        return C.RemoveContainerResponse()

    def _c(self, cid, c):
        cfg = c["config"]
        return dict(id=cid, metadata=cfg.metadata, image=cfg.image, state=c["state"], created_at=c["created"],
                    labels=cfg.labels, annotations=cfg.annotations)

    async def ListContainers(self, req, ctx):
        f = req.filter
        out = [C.Container(pod_sandbox_id=c["sid"], image_ref="fake", **self._c(cid, c)) for cid, c in self.containers.items()
               if (not f.pod_sandbox_id or f.pod_sandbox_id == c["sid"]) and (not f.id or f.id == cid)]
        return C.ListContainersResponse(containers=out)

    @staticmethod
    def _cstatus(cid, c):
        cfg = c["config"]
        return C.ContainerStatus(
            id=cid, metadata=cfg.metadata, state=c["state"], created_at=c["created"], started_at=c["started"],
            finished_at=c["finished"], exit_code=c["exit"], image=cfg.image, image_ref="fake",
            reason="Completed" if c["state"] == C.CONTAINER_EXITED and c["exit"] == 0 else "",
            labels=cfg.labels, annotations=cfg.annotations)

    async def ContainerStatus(self, req, ctx):
        self._count("ContainerStatus")
        c = self.containers.get(req.container_id)
        if c is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "not found")
        return C.ContainerStatusResponse(status=self._cstatus(req.container_id, c))

    async def ListContainerStats(self, req, ctx):
        return C.ListContainerStatsResponse()

    async def ExecSync(self, req, ctx):
        return C.ExecSyncResponse(stdout=b"", exit_code=0)

    async def GetContainerEvents(self, req, ctx):
        q: asyncio.Queue = asyncio.Queue()
        self.streams.add(q)
        try:
            while True:
                yield await q.get()
        finally:
            self.streams.discard(q)


class _FakeImages:
    async def ImageStatus(self, req, ctx):
        return C.ImageStatusResponse(image=C.Image(id="fake", repo_tags=[req.image.image]))

    async def PullImage(self, req, ctx):
        return C.PullImageResponse(image_ref="fake")

    async def ListImages(self, req, ctx):
        return C.ListImagesResponse()

    async def RemoveImage(self, req, ctx):
        return C.RemoveImageResponse()

    async def ImageFsInfo(self, req, ctx):
        return C.ImageFsInfoResponse()


class HollowNode:
    def __init__(self, server: str, name: str, gpus: int = 8, run_seconds: float | None = None, base_dir: str | None = None,
                 status_period: float = 10.0, partition: str = "SPX/NPS1", resource_naming: str = "single"):
        self.server, self.name, self.gpus, self.run_seconds = server, name, gpus, run_seconds
        self.partition, self.resource_naming = partition, resource_naming
        self.plugins: list = []
        self.base = base_dir or tempfile.mkdtemp(prefix="hollow-", dir="/tmp")
        self.status_period = status_period
        self.runtime = self.plugin = self.kubelet = None

    async def start(self):
        b = self.base
        self.runtime = await FakeRuntime(os.path.join(b, "cri.sock"), self.run_seconds).start()
        cp, _, mp = self.partition.partition("/")
        backend = FakeBackend(n=self.gpus, compute_partition=cp or "SPX", memory_partition=mp or "NPS1") if self.gpus else None
        cfg = KubeletConfig(node_name=self.name, root_dir=os.path.join(b, "kubelet"), plugins_dir=os.path.join(b, "plugins"),
                            cri_socket=os.path.join(b, "cri.sock"), port=0, relist_period=2.0,
                            node_status_update_frequency=self.status_period, eviction_interval=3600.0,
                            cpu_capacity=64, memory_capacity=1024 * 2 ** 30, volume_mounter="none",
                            oom_watcher=False)   # kubemark: fake cAdvisor, no kernel OOM stream
        self.kubelet = await Kubelet(Client(self.server, pool=16), cfg, smi_backend=backend).start()
        if backend is not None:
            # per-node unique device IDs (a real cluster has distinct GPUs on every node)
            for g in backend.data["gpus"]:
                g["uuid"] = g["hip_uuid"] = f"{g['uuid']}-{self.name}"
            self.plugins = make_plugins(backend, self.resource_naming, plugins_dir=os.path.join(b, "plugins"),
                                        health_interval=30.0)
            self.plugin = self.plugins[0]
            for p in self.plugins:
                await p.start()
                await p.wait_for_registration(10)
        return self

    async def stop(self):
        for c in (self.kubelet, *self.plugins, self.runtime):
            if c is not None:
                try:
                    await c.stop()
                except Exception:
                    pass
        if self.kubelet is not None:
            await self.kubelet.client.close()
