"""rktshim — a CRI runtime over rkt (pkg/kubelet/rkt, pkg/kubelet/rktshim).

The reference kubelet drives rkt in two ways: the in-tree `--container-runtime=rkt` integration
(pkg/kubelet/rkt/rkt.go: an appc pod manifest per pod, `rkt prepare` + a systemd unit running
`rkt run-prepared`, pod state read back from rkt's API service) and `rktshim`, the CRI stub that
was to replace it (pkg/kubelet/rktshim: app-interface.go, pod-level-interface.go, imagestore.go —
every method "not implemented"). The design rktshim was heading for, and the one its
successor rktlet shipped, maps CRI one to one onto rkt's app-level commands; that is what this
module does, over the `rkt` command line:

  RunPodSandbox       `rkt app sandbox --uuid-file-save=F --hostname=H --net=host|default
                       --annotation=coreos.com/rkt/experiment/logmode=k8s
                       --annotation=coreos.com/rkt/experiment/kubernetes-log-dir=<log dir>`
                      (kept running as the pod's stage1 process, like the rktlet systemd unit)
  CreateContainer     `rkt app add <uuid> <image id> --name=<app> --exec=<argv0> --environment=K=V …
                       --mnt-volume=name=…,kind=host,source=…,target=…,readOnly=… [--working-dir=…]
                       [--user=… --group=…] --stdout=log --stderr=log
                       --annotation=coreos.com/rkt/experiment/kubernetes-log-path=<CRI log path> -- <args…>`
                      (the app's output lands in CRI log format at <log dir>/<log path>)
                      GPU devices from the device plugin's InitContainer response become host
                      volumes of their device nodes (/dev/kfd, /dev/dri/renderD*), which rkt's
                      stage1 adds to the pod's device allow-list.
  Start/Stop/RemoveContainer  `rkt app start|stop|rm <uuid> --app=<app>`
  ContainerStatus     `rkt app status <uuid> --app=<app> --format=json`
  Stop/RemovePodSandbox, PodSandboxStatus  `rkt stop|rm|status <uuid> [--format=json]`
  Exec                `rkt enter --app=<app> <uuid> <cmd…>` (the shared streaming server)
  Pull/List/Remove/ImageStatus  `rkt fetch docker://…`, `rkt image list|rm|cat-manifest`

rkt is not installed on MI355X hosts, so the tests drive this shim against a scripted rkt
(tests/fake_rkt.py) that implements the same command surface over host processes: parity with a
real rkt binary is unpinned.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import shlex
import signal
import subprocess
import time
import uuid

import grpc

from ..grpcdesc.cri import API_VERSION, CRI as C
from .rocshim import _abort, container_status_msg, sandbox_meta, sandbox_status_msg

log = logging.getLogger("amdkube.rktshim")
RUNTIME_NAME = "rkt"
LOGMODE_ANN = "coreos.com/rkt/experiment/logmode"
LOGDIR_ANN = "coreos.com/rkt/experiment/kubernetes-log-dir"
LOGPATH_ANN = "coreos.com/rkt/experiment/kubernetes-log-path"    # per app, relative to the log dir


class RktError(RuntimeError):
    pass


class _Net:
    def __init__(self, node_ip):
        self.node_ip = node_ip

    def status(self):
        return True, ""


class RktSandbox:
    def __init__(self, sid, meta, labels, annotations, log_dir, host_network):
        self.id, self.meta, self.labels, self.annotations = sid, meta, labels, annotations
        self.log_dir, self.host_network = log_dir, host_network
        self.uuid = ""
        self.state = C.SANDBOX_READY
        self.created_at = time.time_ns()
        self.ip = ""
        self.proc: subprocess.Popen | None = None

    def to_json(self):
        return {k: getattr(self, k) for k in ("id", "meta", "labels", "annotations", "log_dir", "host_network", "uuid",
                                              "state", "created_at", "ip")}


class RktContainer:
    def __init__(self, cid, sid, name, attempt, image, image_ref, app, env, log_path, labels, annotations, mounts, devices):
        self.id, self.sandbox_id, self.name, self.attempt = cid, sid, name, attempt
        self.image, self.image_ref, self.app, self.env = image, image_ref, app, env
        self.log_path, self.labels, self.annotations = log_path, labels, annotations
        self.mounts, self.devices = mounts, devices
        self.state = C.CONTAINER_CREATED
        self.created_at = time.time_ns()
        self.started_at = self.finished_at = 0
        self.exit_code = 0
        self.reason = self.message = ""
        self.pid = None
        self.cwd = None

    def to_json(self):
        return {k: getattr(self, k) for k in ("id", "sandbox_id", "name", "attempt", "image", "image_ref", "app", "env",
                                              "log_path", "labels", "annotations", "mounts", "devices", "state",
                                              "created_at", "started_at", "finished_at", "exit_code", "reason", "pid")}


_APP_STATES = {"created": C.CONTAINER_CREATED, "running": C.CONTAINER_RUNNING, "exited": C.CONTAINER_EXITED}


def app_name(name: str) -> str:
    """rkt app names are ACNames (lower-case alphanumerics and '-')."""
    out = "".join(ch if ch.isalnum() else "-" for ch in name.lower()).strip("-")
    return out or "app"


class RktShim:
    def __init__(self, socket_path: str, state_dir: str, rkt: str = "rkt", insecure_options: str = "image",
                 node_ip: str = "127.0.0.1", streaming_port: int = 0, rkt_env: dict | None = None):
        self.socket, self.state_dir = socket_path, state_dir
        self.rkt_cmd = shlex.split(rkt) if isinstance(rkt, str) else list(rkt)
        self.insecure_options = insecure_options
        self.rkt_env = dict(os.environ, **(rkt_env or {}))
        self.network = _Net(node_ip)
        self.streaming_port = streaming_port
        self.sandboxes: dict[str, RktSandbox] = {}
        self.containers: dict[str, RktContainer] = {}
        self.server = None
        self.streaming = None
        os.makedirs(state_dir, exist_ok=True)

    # ------------------------------------------------------------------ rkt CLI
    def _run(self, *args, timeout: float = 120.0) -> str:
        r = subprocess.run([*self.rkt_cmd, *args], capture_output=True, text=True, timeout=timeout, env=self.rkt_env)
        if r.returncode != 0:
            raise RktError(f"rkt {' '.join(args[:2])} failed ({r.returncode}): {r.stderr.strip()[-400:]}")
        return r.stdout

    async def rkt(self, *args, timeout: float = 120.0) -> str:
        return await asyncio.to_thread(self._run, *args, timeout=timeout)

    async def rkt_json(self, *args):
        out = await self.rkt(*args, "--format=json")
        return json.loads(out) if out.strip() else None

    # ------------------------------------------------------------------ state
    def _ckpt(self):
        data = {"sandboxes": [s.to_json() for s in self.sandboxes.values()],
                "containers": [c.to_json() for c in self.containers.values()]}
        tmp = os.path.join(self.state_dir, "state.json.tmp")
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, os.path.join(self.state_dir, "state.json"))

    def _recover(self):
        try:
            data = json.load(open(os.path.join(self.state_dir, "state.json")))
        except (OSError, ValueError):
            return
        for d in data.get("sandboxes") or []:
            s = RktSandbox(d["id"], d["meta"], d["labels"], d["annotations"], d["log_dir"], d["host_network"])
            s.uuid, s.state, s.created_at, s.ip = d["uuid"], d["state"], d["created_at"], d.get("ip", "")
            self.sandboxes[s.id] = s
        for d in data.get("containers") or []:
            c = RktContainer(d["id"], d["sandbox_id"], d["name"], d["attempt"], d["image"], d["image_ref"], d["app"], d["env"],
                             d["log_path"], d["labels"], d["annotations"], d["mounts"], d["devices"])
            for k in ("state", "created_at", "started_at", "finished_at", "exit_code", "reason", "pid"):
                setattr(c, k, d.get(k, getattr(c, k)))
            self.containers[c.id] = c

    # ------------------------------------------------------------------ sandboxes
    async def run_sandbox(self, cfg) -> str:
        meta = {"name": cfg.metadata.name, "uid": cfg.metadata.uid, "namespace": cfg.metadata.namespace,
                "attempt": cfg.metadata.attempt}
        host_net = bool(cfg.HasField("linux") and cfg.linux.HasField("security_context")
                        and cfg.linux.security_context.HasField("namespace_options")
                        and cfg.linux.security_context.namespace_options.host_network)
        sid = uuid.uuid4().hex
        log_dir = cfg.log_directory or os.path.join(self.state_dir, "logs", sid)
        os.makedirs(log_dir, exist_ok=True)
        s = RktSandbox(sid, meta, dict(cfg.labels), dict(cfg.annotations), log_dir, host_net)
        uuid_file = os.path.join(self.state_dir, f"{sid}.uuid")
        argv = [*self.rkt_cmd, "app", "sandbox", f"--uuid-file-save={uuid_file}", f"--hostname={cfg.hostname or cfg.metadata.name}",
                "--net=host" if host_net else "--net=default", f"--annotation={LOGMODE_ANN}=k8s",
                f"--annotation={LOGDIR_ANN}={log_dir}"]
        for k, v in sorted(cfg.annotations.items()):
            argv.append(f"--annotation={k}={v}")
        for pm in cfg.port_mappings:
            argv.append(f"--port={'tcp' if pm.protocol == 0 else 'udp'}-{pm.container_port}:{pm.host_port}")
        s.proc = subprocess.Popen(argv, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                  env=self.rkt_env, start_new_session=True)
        deadline = time.monotonic() + 60
        while not (os.path.exists(uuid_file) and open(uuid_file).read().strip()):
            if s.proc.poll() is not None:
                raise RktError(f"rkt app sandbox exited with {s.proc.returncode}")
            if time.monotonic() > deadline:
                s.proc.kill()
                raise RktError("rkt app sandbox did not report its pod UUID")
            await asyncio.sleep(0.02)
        s.uuid = open(uuid_file).read().strip()
        try:
            st = await self.rkt_json("status", s.uuid)
            nets = (st or {}).get("networks") or []
            s.ip = nets[0].get("ip", "") if nets else ""
        except RktError:
            pass
        self.sandboxes[sid] = s
        self._ckpt()
        return sid

    async def stop_sandbox(self, sid: str):
        s = self.sandboxes.get(sid)
        if s is None:
            return
        for c in [c for c in self.containers.values() if c.sandbox_id == sid and c.state == C.CONTAINER_RUNNING]:
            await self.stop_container(c.id, 10)
        if s.state == C.SANDBOX_READY:
            try:
                await self.rkt("stop", "--force", s.uuid)
            except RktError as e:
                log.debug("rkt stop %s: %s", s.uuid, e)
            if s.proc is not None:
                try:
                    await asyncio.to_thread(s.proc.wait, 10)
                except subprocess.TimeoutExpired:
                    s.proc.kill()
            s.state = C.SANDBOX_NOTREADY
            self._ckpt()

    async def remove_sandbox(self, sid: str):
        s = self.sandboxes.get(sid)
        if s is None:
            return
        await self.stop_sandbox(sid)
        for cid in [c.id for c in self.containers.values() if c.sandbox_id == sid]:
            self.containers.pop(cid, None)
        try:
            await self.rkt("rm", s.uuid)
        except RktError as e:
            log.debug("rkt rm %s: %s", s.uuid, e)
        self.sandboxes.pop(sid, None)
        self._ckpt()

    # ------------------------------------------------------------------ containers
    async def create_container(self, sid: str, cfg) -> str:
        s = self.sandboxes.get(sid)
        if s is None or s.state != C.SANDBOX_READY:
            raise LookupError(f"sandbox {sid} not found or not ready")
        image_id = await self.image_id(cfg.image.image)
        if image_id is None:
            raise LookupError(f"image {cfg.image.image!r} not present (PullImage first)")
        app = app_name(cfg.metadata.name)
        argv = [*cfg.command, *cfg.args] if cfg.command else None
        env = {kv.key: kv.value for kv in cfg.envs}
        devices = [{"container_path": d.container_path, "host_path": d.host_path, "permissions": d.permissions}
                   for d in cfg.devices]
        if not any(d["host_path"].endswith("/kfd") for d in devices):
            env.pop("ROCR_VISIBLE_DEVICES", None)
            env["HIP_VISIBLE_DEVICES"] = "-1"       # non-GPU apps see no GPU, as under rocshim
        mounts = [{"container_path": m.container_path, "host_path": m.host_path, "readonly": m.readonly} for m in cfg.mounts]
        rel_log = cfg.log_path or f"{app}_{cfg.metadata.attempt}.log"
        args = ["app", "add", s.uuid, image_id, f"--name={app}", "--stdout=log", "--stderr=log",
                f"--annotation={LOGPATH_ANN}={rel_log}"]
        for k, v in sorted(env.items()):
            args.append(f"--environment={k}={v}")
        for i, m in enumerate(mounts):
            args.append(f"--mnt-volume=name=vol-{i},kind=host,source={m['host_path']},target={m['container_path']},"
                        f"readOnly={'true' if m['readonly'] else 'false'}")
        for i, d in enumerate(devices):
            args.append(f"--mnt-volume=name=dev-{i},kind=host,source={d['host_path']},target={d['container_path']},readOnly=false")
        if cfg.working_dir:
            args.append(f"--working-dir={cfg.working_dir}")
        sc = cfg.linux.security_context if cfg.HasField("linux") and cfg.linux.HasField("security_context") else None
        if sc is not None and sc.HasField("run_as_user"):
            args.append(f"--user={sc.run_as_user.value}")
        if argv:
            args.append(f"--exec={argv[0]}")
            if argv[1:]:
                args += ["--", *argv[1:]]
        await self.rkt(*args)
        cid = uuid.uuid4().hex
        log_path = os.path.join(s.log_dir, rel_log)
        c = RktContainer(cid, sid, cfg.metadata.name, cfg.metadata.attempt, cfg.image.image, image_id, app, env, log_path,
                         dict(cfg.labels), dict(cfg.annotations), mounts, devices)
        self.containers[cid] = c
        self._ckpt()
        return cid

    async def start_container(self, cid: str):
        c = self._get(cid)
        s = self.sandboxes[c.sandbox_id]
        await self.rkt("app", "start", s.uuid, f"--app={c.app}")
        await self.refresh(c)

    async def stop_container(self, cid: str, timeout: int):
        c = self.containers.get(cid)
        if c is None:
            return
        s = self.sandboxes.get(c.sandbox_id)
        if s is not None and c.state == C.CONTAINER_RUNNING:
            try:
                await self.rkt("app", "stop", s.uuid, f"--app={c.app}", timeout=max(10, timeout + 10))
            except RktError as e:
                log.debug("rkt app stop: %s", e)
            await self.refresh(c)

    async def remove_container(self, cid: str):
        c = self.containers.get(cid)
        if c is None:
            return
        s = self.sandboxes.get(c.sandbox_id)
        if s is not None:
            try:
                await self.rkt("app", "rm", s.uuid, f"--app={c.app}")
            except RktError as e:
                log.debug("rkt app rm: %s", e)
        self.containers.pop(cid, None)
        self._ckpt()

    def _get(self, cid) -> RktContainer:
        c = self.containers.get(cid)
        if c is None:
            raise LookupError(f"container {cid} not found")
        return c

    async def refresh(self, c: RktContainer):
        """rkt app status → the CRI view of one app."""
        s = self.sandboxes.get(c.sandbox_id)
        if s is None or c.state == C.CONTAINER_EXITED:
            return
        try:
            st = await self.rkt_json("app", "status", s.uuid, f"--app={c.app}") or {}
        except RktError:
            if s.state != C.SANDBOX_READY:
                c.state = C.CONTAINER_EXITED
            return
        c.state = _APP_STATES.get(st.get("state", ""), C.CONTAINER_UNKNOWN)
        c.started_at = int(st.get("started_at") or c.started_at)
        c.finished_at = int(st.get("finished_at") or c.finished_at)
        c.pid = st.get("pid") or c.pid
        if c.state == C.CONTAINER_EXITED:
            c.exit_code = int(st.get("exit_code") or 0)
            c.reason = "Completed" if c.exit_code == 0 else "Error"
            c.pid = None
        self._ckpt()

    async def refresh_all(self):
        for c in list(self.containers.values()):
            if c.state in (C.CONTAINER_CREATED, C.CONTAINER_RUNNING):
                await self.refresh(c)

    def exec_argv(self, c: RktContainer, cmd: list[str]) -> list[str]:
        s = self.sandboxes[c.sandbox_id]
        return [*self.rkt_cmd, "enter", f"--app={c.app}", s.uuid, *cmd]

    def exec_cwd(self, c) -> None:
        return None

    async def exec_sync(self, cid: str, cmd: list[str], timeout: int):
        c = self._get(cid)
        proc = await asyncio.create_subprocess_exec(*self.exec_argv(c, cmd), stdout=asyncio.subprocess.PIPE,
                                                    stderr=asyncio.subprocess.PIPE, env=self.rkt_env)
        try:
            out, err = await asyncio.wait_for(proc.communicate(), timeout or None)
        except asyncio.TimeoutError:
            proc.kill()
            raise
        return out, err, proc.returncode

    # ------------------------------------------------------------------ images
    async def images(self) -> list[dict]:
        return await self.rkt_json("image", "list") or []

    async def image_id(self, ref: str) -> str | None:
        want = _normalize(ref)
        for im in await self.images():
            if im.get("id") == ref or _normalize(im.get("name", "")) == want:
                return im["id"]
        return None

    async def pull(self, ref: str) -> str:
        out = await self.rkt("fetch", f"--insecure-options={self.insecure_options}", "--full", f"docker://{ref}", timeout=600)
        lines = [x.strip() for x in out.splitlines() if x.strip()]
        if not lines:
            raise RktError(f"rkt fetch printed no image ID for {ref}")
        return lines[-1]

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        self._recover()
        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        if os.path.exists(self.socket):
            os.unlink(self.socket)
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((C.RuntimeService.handler(_Runtime(self)), C.ImageService.handler(_Images(self))))
        self.server.add_insecure_port("unix://" + self.socket)
        await self.server.start()
        from .streaming import StreamingServer
        self.streaming = await StreamingServer(self, port=self.streaming_port).start()
        log.info("rktshim serving CRI on %s over %s", self.socket, " ".join(self.rkt_cmd))
        return self

    async def stop(self, kill_pods: bool = False):
        if kill_pods:
            for sid in list(self.sandboxes):
                await self.stop_sandbox(sid)
        if self.streaming is not None:
            await self.streaming.stop()
        if self.server:
            await self.server.stop(0.5)
        for s in self.sandboxes.values():
            if s.proc is not None and s.proc.poll() is None and kill_pods:
                os.killpg(s.proc.pid, signal.SIGKILL)


def _normalize(ref: str) -> str:
    """docker.io/library/busybox:latest ≡ busybox ≡ busybox:latest."""
    r = ref.strip()
    for p in ("docker://", "docker.io/library/", "docker.io/", "registry-1.docker.io/library/"):
        if r.startswith(p):
            r = r[len(p):]
    if ":" not in r.rsplit("/", 1)[-1] and "@" not in r:
        r += ":latest"
    return r


class _Runtime:
    def __init__(self, r: RktShim):
        self.r = r

    async def Version(self, req, ctx):
        try:
            v = (await self.r.rkt("version")).splitlines()
            ver = next((x.split(":", 1)[1].strip() for x in v if x.lower().startswith("rkt version")), "unknown")
        except RktError:
            ver = "unknown"
        return C.VersionResponse(version=API_VERSION, runtime_name=RUNTIME_NAME, runtime_version=ver, runtime_api_version="v1alpha1")

    async def Status(self, req, ctx):
        conds = [C.RuntimeCondition(type="RuntimeReady", status=True), C.RuntimeCondition(type="NetworkReady", status=True)]
        return C.StatusResponse(status=C.RuntimeStatus(conditions=conds))

    async def RunPodSandbox(self, req, ctx):
        try:
            sid = await self.r.run_sandbox(req.config)
        except Exception as e:
            await _abort(ctx, e)
        return C.RunPodSandboxResponse(pod_sandbox_id=sid)

    async def StopPodSandbox(self, req, ctx):
        await self.r.stop_sandbox(req.pod_sandbox_id)
        return C.StopPodSandboxResponse()

    async def RemovePodSandbox(self, req, ctx):
        await self.r.remove_sandbox(req.pod_sandbox_id)
        return C.RemovePodSandboxResponse()

    async def PodSandboxStatus(self, req, ctx):
        s = self.r.sandboxes.get(req.pod_sandbox_id)
        if s is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"sandbox {req.pod_sandbox_id} not found")
        if s.state == C.SANDBOX_READY:
            try:
                st = await self.r.rkt_json("status", s.uuid) or {}
                if st.get("state") not in ("running", "embryo", "preparing", "prepared"):
                    s.state = C.SANDBOX_NOTREADY
            except RktError:
                s.state = C.SANDBOX_NOTREADY
        return C.PodSandboxStatusResponse(status=sandbox_status_msg(s, self.r.network.node_ip),
                                          info={"uuid": s.uuid} if req.verbose else {})

    async def ListPodSandbox(self, req, ctx):
        f = req.filter if req.HasField("filter") else None
        out = []
        for s in self.r.sandboxes.values():
            if f is not None and ((f.id and f.id != s.id) or (f.HasField("state") and f.state.state != s.state)
                                  or any(s.labels.get(k) != v for k, v in f.label_selector.items())):
                continue
            out.append(C.PodSandbox(id=s.id, metadata=sandbox_meta(s), state=s.state, created_at=s.created_at,
                                    labels=s.labels, annotations=s.annotations))
        return C.ListPodSandboxResponse(items=out)

    async def CreateContainer(self, req, ctx):
        try:
            cid = await self.r.create_container(req.pod_sandbox_id, req.config)
        except Exception as e:
            await _abort(ctx, e)
        return C.CreateContainerResponse(container_id=cid)

    async def StartContainer(self, req, ctx):
        try:
            await self.r.start_container(req.container_id)
        except Exception as e:
            await _abort(ctx, e)
        return C.StartContainerResponse()

    async def StopContainer(self, req, ctx):
        await self.r.stop_container(req.container_id, req.timeout)
        return C.StopContainerResponse()

    async def RemoveContainer(self, req, ctx):
        await self.r.remove_container(req.container_id)
        return C.RemoveContainerResponse()

    async def UpdateContainerResources(self, req, ctx):
        await ctx.abort(grpc.StatusCode.UNIMPLEMENTED, "rkt apps cannot be resized in place")

    async def ListContainers(self, req, ctx):
        await self.r.refresh_all()
        f = req.filter if req.HasField("filter") else None
        out = []
        for c in self.r.containers.values():
            if f is not None and ((f.id and f.id != c.id) or (f.pod_sandbox_id and f.pod_sandbox_id != c.sandbox_id)
                                  or (f.HasField("state") and f.state.state != c.state)
                                  or any(c.labels.get(k) != v for k, v in f.label_selector.items())):
                continue
            out.append(C.Container(id=c.id, pod_sandbox_id=c.sandbox_id, metadata=C.ContainerMetadata(name=c.name, attempt=c.attempt),
                                   image=C.ImageSpec(image=c.image), image_ref=c.image_ref, state=c.state,
                                   created_at=c.created_at, labels=c.labels, annotations=c.annotations))
        return C.ListContainersResponse(containers=out)

    async def ContainerStatus(self, req, ctx):
        c = self.r.containers.get(req.container_id)
        if c is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} not found")
        await self.r.refresh(c)
        info = {"app": c.app, "pod_uuid": self.r.sandboxes[c.sandbox_id].uuid} if req.verbose else {}
        return C.ContainerStatusResponse(status=container_status_msg(c), info=info)

    async def Exec(self, req, ctx):
        c = self.r.containers.get(req.container_id)
        if c is None or c.state != C.CONTAINER_RUNNING:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} is not running")
        c.pid = c.pid or 1
        return C.ExecResponse(url=self.r.streaming.get_exec(req.container_id, req.cmd, req.tty, req.stdin, req.stdout, req.stderr))

    async def Attach(self, req, ctx):
        if req.container_id not in self.r.containers:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} not found")
        return C.AttachResponse(url=self.r.streaming.get_attach(req.container_id, req.tty, req.stdin, req.stdout, req.stderr))

    async def PortForward(self, req, ctx):
        s = self.r.sandboxes.get(req.pod_sandbox_id)
        if s is None or s.state != C.SANDBOX_READY:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"sandbox {req.pod_sandbox_id} is not ready")
        return C.PortForwardResponse(url=self.r.streaming.get_portforward(req.pod_sandbox_id, list(req.port)))

    async def ExecSync(self, req, ctx):
        try:
            out, err, rc = await self.r.exec_sync(req.container_id, list(req.cmd), req.timeout)
        except Exception as e:
            await _abort(ctx, e)
        return C.ExecSyncResponse(stdout=out, stderr=err, exit_code=rc)

    async def ContainerStats(self, req, ctx):
        await ctx.abort(grpc.StatusCode.UNIMPLEMENTED, "container stats come from the node's cgroups for rkt pods")

    async def ListContainerStats(self, req, ctx):
        return C.ListContainerStatsResponse(stats=[])

    async def UpdateRuntimeConfig(self, req, ctx):
        return C.UpdateRuntimeConfigResponse()


class _Images:
    def __init__(self, r: RktShim):
        self.r = r

    @staticmethod
    def _img(im):
        return C.Image(id=im["id"], repo_tags=[_normalize(im.get("name", ""))], size=int(im.get("size") or 0))

    async def ListImages(self, req, ctx):
        return C.ListImagesResponse(images=[self._img(im) for im in await self.r.images()])

    async def ImageStatus(self, req, ctx):
        want = _normalize(req.image.image)
        for im in await self.r.images():
            if im.get("id") == req.image.image or _normalize(im.get("name", "")) == want:
                return C.ImageStatusResponse(image=self._img(im))
        return C.ImageStatusResponse()

    async def PullImage(self, req, ctx):
        try:
            return C.PullImageResponse(image_ref=await self.r.pull(req.image.image))
        except RktError as e:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, str(e))

    async def RemoveImage(self, req, ctx):
        iid = await self.r.image_id(req.image.image)
        if iid is not None:
            if any(c.image_ref == iid for c in self.r.containers.values()):
                await ctx.abort(grpc.StatusCode.FAILED_PRECONDITION, f"image {req.image.image} is in use by a container")
            await self.r.rkt("image", "rm", iid)
        return C.RemoveImageResponse()

    async def ImageFsInfo(self, req, ctx):
        return C.ImageFsInfoResponse(image_filesystems=[])
