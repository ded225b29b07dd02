"""Remote CRI client (reference pkg/kubelet/remote/remote_runtime.go:42,177 and
remote_image.go): typed async wrappers over the RuntimeService/ImageService stubs with
per-call timeouts and operation metrics (kubelet_runtime_operations{operation_type})."""
from __future__ import annotations

import contextvars
import time

import grpc

from ..grpcdesc.cri import CRI as C, EVENT_TRAILER
from ..utils.grpcutil import uds_channel

# the pod a kubelet pod worker is syncing (set once per worker task; asyncio copies it into
# every await chain the worker starts)
CURRENT_POD: contextvars.ContextVar[str | None] = contextvars.ContextVar("amdkube_current_pod", default=None)


class CRIClient:
    def __init__(self, socket_path: str, timeout: float = 10.0, metrics=None, image_socket: str | None = None):
        self._pod_mut: dict[str, int] = {}
        self._cid_sid: dict[str, str] = {}
        # uid -> {sandbox id: created_at of the runtime event that carries the sandbox's state after
        # the pod worker's last mutating call on it}; None: a call's final event is unknown
        self._touched: dict[str, dict[str, int] | None] = {}
        self.socket = socket_path
        self.image_socket = image_socket        # --image-service-endpoint (None: the runtime's socket)
        self.timeout = timeout
        self.ch = self.img_ch = None
        self.rt = self.img = None
        self.metrics = metrics  # (ops Counter, errs Counter, latency Summary) or None

    async def connect(self, wait: float = 10.0):
        self.ch = uds_channel(self.socket)
        import asyncio
        await asyncio.wait_for(self.ch.channel_ready(), wait)
        self.rt = C.RuntimeService.stub(self.ch)
        if self.image_socket and self.image_socket != self.socket:
            self.img_ch = uds_channel(self.image_socket)
            await asyncio.wait_for(self.img_ch.channel_ready(), wait)
            self.img = C.ImageService.stub(self.img_ch)
        else:
            self.img = C.ImageService.stub(self.ch)
        return self

    async def close(self):
        if self.ch is not None:
            await self.ch.close()
        if self.img_ch is not None:
            await self.img_ch.close()

    _MUTATING = frozenset(("run_podsandbox", "stop_podsandbox", "remove_podsandbox", "create_container", "start_container",
                           "stop_container", "remove_container"))
    mutations = 0  # mutating RPCs issued (invalidates the kubelet's runtime-status cache)

    def pod_mutations(self, uid: str) -> int:
        """Mutating RPCs issued on behalf of one pod: its cached runtime status stays valid across
        other pods' container starts (a global counter made 30 concurrent pods refetch ~6× each)."""
        return self._pod_mut.get(uid, 0)

    def forget_pod(self, uid: str):
        self._pod_mut.pop(uid, None)
        self._touched.pop(uid, None)

    def take_touched(self, uid: str):
        """Sandboxes the pod's worker mutated since the last call, each with the created_at of the
        runtime event that reflects the last of those mutations (None when some call's final event
        is unknown: a runtime that does not return the event trailer)."""
        return self._touched.pop(uid, {})

    def _touch(self, mark: str | None):
        """Record a mutating call's event trailer for the pod being synced: "" means the call
        emitted nothing to wait for (e.g. removing an already-removed container)."""
        uid = CURRENT_POD.get()
        if uid is None:
            return
        cur = self._touched.get(uid, {})
        if cur is None:
            return
        if mark is None:
            self._touched[uid] = None
        elif mark:
            sid, _, ts = mark.rpartition(":")
            cur[sid] = max(cur.get(sid, 0), int(ts))
            self._touched[uid] = cur

    async def _call(self, op, fn, req, timeout=None):
        t0 = time.perf_counter()
        mutating = op in self._MUTATING
        if mutating:
            self.mutations += 1
            uid = CURRENT_POD.get()
            if uid is not None:
                self._pod_mut[uid] = self._pod_mut.get(uid, 0) + 1
        try:
            if not mutating:
                return await fn(req, timeout=timeout or self.timeout)
            call = fn(req, timeout=timeout or self.timeout)
            resp = await call
            mark = None
            for k, v in (await call.trailing_metadata()) or ():
                if k == EVENT_TRAILER:
                    mark = v
            self._touch(mark)
            return resp
        except grpc.RpcError:
            if self.metrics:
                self.metrics[1].labels(op).inc()
            raise
        finally:
            if self.metrics:
                self.metrics[0].labels(op).inc()
                self.metrics[2].labels(op).observe((time.perf_counter() - t0) * 1e6)

    # ------------------------------------------------------------- runtime
    async def version(self):
        return await self._call("version", self.rt.Version, C.VersionRequest(version="v1alpha1"))

    async def status(self):
        return await self._call("status", self.rt.Status, C.StatusRequest(verbose=True))

    async def run_pod_sandbox(self, cfg) -> str:
        return (await self._call("run_podsandbox", self.rt.RunPodSandbox, C.RunPodSandboxRequest(config=cfg))).pod_sandbox_id

    async def stop_pod_sandbox(self, sid):
        await self._call("stop_podsandbox", self.rt.StopPodSandbox, C.StopPodSandboxRequest(pod_sandbox_id=sid), timeout=60)

    async def remove_pod_sandbox(self, sid):
        await self._call("remove_podsandbox", self.rt.RemovePodSandbox, C.RemovePodSandboxRequest(pod_sandbox_id=sid), timeout=60)

    async def list_pod_sandbox(self, uid: str | None = None):
        f = C.PodSandboxFilter(label_selector={"io.kubernetes.pod.uid": uid}) if uid else None
        req = C.ListPodSandboxRequest(filter=f) if f else C.ListPodSandboxRequest()
        return list((await self._call("list_podsandbox", self.rt.ListPodSandbox, req)).items)

    async def update_runtime_config(self, pod_cidr: str):
        req = C.UpdateRuntimeConfigRequest(runtime_config=C.RuntimeConfig(network_config=C.NetworkConfig(pod_cidr=pod_cidr)))
        await self._call("update_runtime_config", self.rt.UpdateRuntimeConfig, req)

    async def pod_sandbox_status(self, sid):
        return (await self._call("podsandbox_status", self.rt.PodSandboxStatus, C.PodSandboxStatusRequest(pod_sandbox_id=sid))).status

    async def pod_sandbox_info(self, sid) -> dict:
        """PodSandboxStatus(verbose=true).info: runtime-specific details (rocshim: the pause pid)."""
        resp = await self._call("podsandbox_status", self.rt.PodSandboxStatus,
                                C.PodSandboxStatusRequest(pod_sandbox_id=sid, verbose=True))
        return dict(resp.info)

    async def create_container(self, sid, cfg, sandbox_cfg) -> str:
        req = C.CreateContainerRequest(pod_sandbox_id=sid, config=cfg, sandbox_config=sandbox_cfg)
        cid = (await self._call("create_container", self.rt.CreateContainer, req)).container_id
        self._cid_sid[cid] = sid
        return cid

    async def start_container(self, cid):
        await self._call("start_container", self.rt.StartContainer, C.StartContainerRequest(container_id=cid))

    async def stop_container(self, cid, timeout: int):
        await self._call("stop_container", self.rt.StopContainer, C.StopContainerRequest(container_id=cid, timeout=timeout),
                         timeout=timeout + 30)

    async def remove_container(self, cid):
        self._cid_sid.pop(cid, None)
        await self._call("remove_container", self.rt.RemoveContainer, C.RemoveContainerRequest(container_id=cid))

    async def update_container_resources(self, cid, cpuset_cpus: str = "", **res):
        lr = C.LinuxContainerResources(cpuset_cpus=cpuset_cpus, **res)
        await self._call("update_container_resources", self.rt.UpdateContainerResources,
                         C.UpdateContainerResourcesRequest(container_id=cid, linux=lr))

    async def list_containers(self, sandbox_id: str | None = None):
        f = C.ContainerFilter(pod_sandbox_id=sandbox_id) if sandbox_id else None
        req = C.ListContainersRequest(filter=f) if f else C.ListContainersRequest()
        return list((await self._call("list_containers", self.rt.ListContainers, req)).containers)

    async def container_status(self, cid, verbose=False):
        r = await self._call("container_status", self.rt.ContainerStatus, C.ContainerStatusRequest(container_id=cid, verbose=verbose))
        return r.status, dict(r.info)

    async def exec_sync(self, cid, cmd, timeout=10):
        r = await self._call("exec_sync", self.rt.ExecSync, C.ExecSyncRequest(container_id=cid, cmd=cmd, timeout=timeout),
                             timeout=timeout + 5)
        return r.stdout, r.stderr, r.exit_code

    async def exec_url(self, cid, cmd, tty=False, stdin=False, stdout=True, stderr=True) -> str:
        req = C.ExecRequest(container_id=cid, cmd=cmd, tty=tty, stdin=stdin, stdout=stdout, stderr=stderr)
        return (await self._call("exec", self.rt.Exec, req)).url

    async def attach_url(self, cid, tty=False, stdin=False, stdout=True, stderr=True) -> str:
        req = C.AttachRequest(container_id=cid, tty=tty, stdin=stdin, stdout=stdout, stderr=stderr)
        return (await self._call("attach", self.rt.Attach, req)).url

    async def port_forward_url(self, sid, ports) -> str:
        return (await self._call("port_forward", self.rt.PortForward, C.PortForwardRequest(pod_sandbox_id=sid, port=ports))).url

    async def list_container_stats(self):
        return list((await self._call("list_container_stats", self.rt.ListContainerStats, C.ListContainerStatsRequest())).stats)

    def container_events(self):
        return self.rt.GetContainerEvents(C.GetEventsRequest())

    # --------------------------------------------------------------- images
    async def image_status(self, image):
        r = await self._call("image_status", self.img.ImageStatus, C.ImageStatusRequest(image=C.ImageSpec(image=image)))
        return r.image if r.HasField("image") else None

    async def pull_image(self, image, auth=None) -> str:
        req = C.PullImageRequest(image=C.ImageSpec(image=image))
        if auth is not None:
            req.auth.CopyFrom(auth)
        return (await self._call("pull_image", self.img.PullImage, req, timeout=300)).image_ref

    async def remove_image(self, image):
        await self._call("remove_image", self.img.RemoveImage, C.RemoveImageRequest(image=C.ImageSpec(image=image)))

    async def list_images(self):
        return list((await self._call("list_images", self.img.ListImages, C.ListImagesRequest())).images)

    async def image_fs_info(self):
        return list((await self._call("image_fs_info", self.img.ImageFsInfo, C.ImageFsInfoRequest())).image_filesystems)
