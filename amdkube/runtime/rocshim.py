"""rocshim — amdkube's CRI runtime for MI355X nodes (replaces dockershim + dockerd + the
nvidia OCI runtime hook; reference pkg/kubelet/dockershim).

CRI v1alpha1 RuntimeService + ImageService over a Unix socket. A pod sandbox is a `pause`
process (native/pause.cpp, child subreaper); containers are process trees started with
their own session so the whole tree can be signalled. GPU injection follows the device
plugin's InitContainer response as carried in the CRI ContainerConfig:
  * env  — ROCR_VISIBLE_DEVICES from the plugin; inherited HIP/CUDA/ROCR visibility
           variables are scrubbed so a container sees exactly its assigned GPUs, and a
           container with no GPU devices gets HIP_VISIBLE_DEVICES=-1 (sees none);
  * devices — /dev/kfd + /dev/dri/renderD<N>, enforced by the kernel through the native
           `amdkube-nsexec` launcher (native/devguard.h), strongest mechanism first
           (`isolation=auto` probes the node once, `amdkube-nsexec --probe`):
           `namespaces` (root): a private mount namespace whose /dev/dri holds only the
                 container's render nodes, /dev/kfd masked for non-GPU containers, a cgroup-v2
                 leaf with cpu/memory limits and a BPF device filter (226:* only the kept
                 minors, kfd only with a GPU), Landlock layered under it, the capability
                 bounding set cut to Docker's default, no_new_privs;
           `userns` (unprivileged, user namespaces enabled): the same private /dev/dri in a
                 mount namespace owned by a user namespace;
           `landlock` (unprivileged, no user namespaces — the MI355X gpurun box): a Landlock
                 ruleset under which every GPU node the container was not given is refused
                 and mknod of device nodes fails; the `rocm` handler's devview preload makes
                 those nodes read as absent, which ROCr skips (an EACCES it would not);
           `env`: visibility variables only (advisory).
The runtime handler for a container is chosen by the hooks.d service (F21 semantics). As the
reference's `nvidia` OCI runtime is what makes a GPU usable inside a container
(docker_container.go:132,157), the `rocm` handler is what gives one its GPUs here: the
device view of the CRI device list plus the ROCm user space (an image rootfs gets /opt/rocm
bound in read-only). Under `default` (runc semantics) the CRI devices are passed as they are,
with no ROCm injection and no device-view preload.

State (sandboxes + containers) is checkpointed as JSON so a restarted rocshim re-adopts
running pods instead of orphaning them; exit codes of re-adopted processes
are recovered from the per-container exit file written by the launcher.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import shutil
import signal
import subprocess
import threading
import time
import uuid

import grpc

from ..grpcdesc.cri import API_VERSION, CRI as C, EVENT_TRAILER
from .hooks import DEFAULT_HOOKS_DIR, HookService
from .images import NATIVE_BIN, ImageStore
from .network import HostNetwork

log = logging.getLogger("amdkube.rocshim")

RUNTIME_NAME = "rocshim"
RUNTIME_VERSION = "0.1.0"
HANDLERS = {"rocm", "default"}
ISOLATION_MODES = ("env", "landlock", "userns", "namespaces", "auto")
DEVVIEW_LIB = os.path.join(os.path.dirname(NATIVE_BIN), "lib", "libamdkube-devview.so")
# Docker's default capability set: what a non-privileged container keeps in guarded modes
DEFAULT_CAPS = ("CHOWN", "DAC_OVERRIDE", "FSETID", "FOWNER", "MKNOD", "NET_RAW", "SETGID", "SETUID", "SETFCAP", "SETPCAP",
                "NET_BIND_SERVICE", "SYS_CHROOT", "KILL", "AUDIT_WRITE")
_PROBE: dict | None = None
DEFAULT_PATH = "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin"
# what the rocm handler binds into an image rootfs: ROCm and the amdgpu marketing-name table
ROCM_INJECT = ("/opt/rocm", "/usr/share/libdrm")


def _with_argv(c, argv):
    """A shallow view of container `c` with another argv (the checkpointed argv stays the image's)."""
    v = Container.__new__(Container)
    v.__dict__.update(c.__dict__)
    v.argv = argv
    return v


def probe_isolation(nsexec_bin: str | None = None) -> dict:
    """What the node offers (`amdkube-nsexec --probe`, cached per process)."""
    global _PROBE
    if _PROBE is None:
        try:
            out = subprocess.run([nsexec_bin or os.path.join(NATIVE_BIN, "amdkube-nsexec"), "--probe"],
                                 capture_output=True, text=True, timeout=10).stdout
            _PROBE = json.loads(out.strip().splitlines()[-1])
        except (OSError, ValueError, IndexError, subprocess.SubprocessError):
            _PROBE = {"root": os.geteuid() == 0, "landlock_abi": 0, "userns": False, "cgroup2": False,
                      "cgroup2_writable": False}
    return _PROBE


def resolve_isolation(mode: str, probe: dict) -> str:
    """`auto` → the strongest mechanism the node has (root+cgroup2 → namespaces, user namespaces
    → userns, Landlock → landlock, else env). An explicit mode is taken as asked."""
    if mode not in ISOLATION_MODES:
        raise ValueError(f"unknown isolation mode {mode!r} (one of {', '.join(ISOLATION_MODES)})")
    if mode != "auto":
        return mode
    if probe.get("root") and probe.get("cgroup2_writable"):
        return "namespaces"
    if probe.get("userns") and not probe.get("root"):
        return "userns"
    if probe.get("landlock_abi", 0) >= 1:
        return "landlock"
    return "env"


def container_caps(sc) -> str:
    """Bounding set for a container from its CRI security context: privileged keeps all,
    else Docker's default set plus adds minus drops ("ALL" honoured on either side)."""
    if sc is None:
        return ",".join(DEFAULT_CAPS)
    if sc.privileged:
        return "all"
    caps = set(DEFAULT_CAPS)
    add = [c.upper().removeprefix("CAP_") for c in sc.capabilities.add_capabilities] if sc.HasField("capabilities") else []
    drop = [c.upper().removeprefix("CAP_") for c in sc.capabilities.drop_capabilities] if sc.HasField("capabilities") else []
    if "ALL" in add:
        return "all"
    caps |= set(add)
    caps = set() if "ALL" in drop else caps - set(drop)
    return ",".join(sorted(caps)) or "none"
SCRUB_ENV = ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL",
             "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", "RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
             "TORCHELASTIC_RUN_ID", "GROUP_RANK", "LOCAL_WORLD_SIZE", "ROLE_RANK")


def now_ns() -> int:
    return time.time_ns()



class PidProc:
    """A child process watched through a pidfd on the event loop (Linux ≥ 5.3): no transport,
    pipes or per-child waiter thread, which asyncio.create_subprocess_exec costs per spawn
    (ThreadedChildWatcher). `wait()` returns the returncode as subprocess does (−signal).
    `pump` is the container's log pump (a future resolved when it has exited and been reaped)."""
    __slots__ = ("pid", "returncode", "_popen", "_fd", "_fut", "pump")

    def __init__(self, popen: subprocess.Popen, fd: int):
        loop = asyncio.get_running_loop()
        self.pid, self.returncode, self._popen, self._fd = popen.pid, None, popen, fd
        self.pump = None
        self._fut = loop.create_future()
        loop.add_reader(fd, self._exited)

    def _exited(self):
        asyncio.get_running_loop().remove_reader(self._fd)
        os.close(self._fd)
        self.returncode = self._popen.wait()
        if not self._fut.done():
            self._fut.set_result(self.returncode)

    async def wait(self):
        return await asyncio.shield(self._fut)

    async def logs_flushed(self, timeout: float = 2.0):
        """Wait (bounded) for the log pump to write the container's last output: it exits once
        every writer of the pipes is gone, which a daemon the container left behind can delay."""
        if self.pump is not None and not self.pump.done():
            try:
                await asyncio.wait_for(asyncio.shield(self.pump), timeout)
            except asyncio.TimeoutError:
                pass


def _reap_later(pid: int, pidfd: int | None):
    """A future resolved once `pid` (our child) exits, reaped on the event loop through its
    pidfd — or by a waiter thread on kernels without pidfds."""
    loop = asyncio.get_running_loop()
    fut = loop.create_future()

    def reaped(_=None):
        if not fut.done():
            fut.set_result(None)
    if pidfd is None:
        loop.run_in_executor(None, os.waitpid, pid, 0).add_done_callback(reaped)
        return fut

    def exited():
        loop.remove_reader(pidfd)
        os.close(pidfd)
        try:
            os.waitpid(pid, 0)
        except ChildProcessError:
            pass
        reaped()
    loop.add_reader(pidfd, exited)
    return fut


LOGPUMP_BIN = os.path.join(NATIVE_BIN, "amdkube-logpump")


def logpump_bin() -> str | None:
    """native/logpump.cpp, the CRI-format log writer; None when it was not built (the
    container's output then goes to its log file untagged — refused when AMDKUBE_REQUIRE_NATIVE
    is set, as on the GPU box)."""
    if os.access(LOGPUMP_BIN, os.X_OK):
        return LOGPUMP_BIN
    if os.environ.get("AMDKUBE_REQUIRE_NATIVE"):
        raise RuntimeError(f"{LOGPUMP_BIN} is not built (python native/build.py)")
    return None


def _spawn_pump(pump: str, log_path: str, out_r: int, err_r: int) -> int:
    """posix_spawn (vfork-fast, unlike a fork of this whole process) of the log pump in a
    session of its own, its read ends as fds 3 and 4 (dup2 clears close-on-exec on them only)."""
    return os.posix_spawn(pump, [pump, "--log", log_path, "--stdout-fd", "3", "--stderr-fd", "4"], os.environ,
                          file_actions=[(os.POSIX_SPAWN_DUP2, out_r, 3), (os.POSIX_SPAWN_DUP2, err_r, 4)], setsid=True)


def _popen(argv, stdout, stderr, env, cwd, log_path, oom_score_adj=None, pass_fds=(), pump=None):
    """fork/exec (and the log file's open, and the child's oom_score_adj) off the event loop: a
    spawn is ~1 ms of syscalls that would otherwise stall every other CRI call the runtime is
    serving. With a log path and `pump` (the logpump binary) the container's stdout and stderr
    are pipes whose read ends the pump owns: it writes the CRI log format (timestamp, stream,
    partial/full tag per line) and outlives this runtime process; without one they are the log
    file itself. The container is started first; the pump follows (the pipes buffer meanwhile)."""
    logf = None
    pipes = None
    if log_path and pump:
        out_r, out_w = os.pipe()
        err_r, err_w = os.pipe()
        pipes = (out_r, out_w, err_r, err_w)
        out, err = out_w, err_w
    else:
        logf = open(log_path, "ab", buffering=0) if log_path else None
        out = logf if logf is not None else (stdout if stdout is not None else subprocess.DEVNULL)
        err = logf if logf is not None else (stderr if stderr is not None else subprocess.DEVNULL)
    pump_pid = None
    try:
        p = subprocess.Popen(argv, stdin=subprocess.DEVNULL, stdout=out, stderr=err, env=env, cwd=cwd,
                             start_new_session=True, pass_fds=pass_fds)
        if pipes:
            os.close(pipes[1])
            os.close(pipes[3])     # the pump sees EOF once the container's copies are gone
            pipes = (pipes[0], None, pipes[2], None)
            try:
                pump_pid = _spawn_pump(pump, log_path, pipes[0], pipes[2])
            except OSError:
                # no log writer: the container must not run unobserved (or die on SIGPIPE later)
                _killpg(p.pid, signal.SIGKILL)
                p.wait()
                raise
    finally:
        if logf is not None:
            logf.close()
        for fd in pipes or ():
            if fd is not None:
                os.close(fd)
    try:
        fd = os.pidfd_open(p.pid)
    except (AttributeError, OSError):
        fd = None
    pump_fd = None
    if pump_pid is not None:
        try:
            pump_fd = os.pidfd_open(pump_pid)
        except (AttributeError, OSError):
            pump_fd = None
    if oom_score_adj:
        _set_oom_score_adj(p.pid, oom_score_adj)
    return p, fd, (pump_pid, pump_fd) if pump_pid is not None else None


async def spawn(argv, stdout=None, stderr=None, env=None, cwd=None, log_path=None, oom_score_adj=None, pass_fds=(),
                log_pump=False):
    """Start argv in its own session with stdin from /dev/null (stdout and stderr appended to
    `log_path` when given — through the log pump with `log_pump`); pidfd-watched when
    possible."""
    pump = logpump_bin() if log_pump and log_path else None
    p, fd, pump_info = await asyncio.to_thread(_popen, argv, stdout, stderr, env, cwd, log_path, oom_score_adj, pass_fds, pump)
    if fd is None:   # old kernel: a thread waits for the child
        loop = asyncio.get_running_loop()
        proc = PidProc.__new__(PidProc)
        proc.pid, proc.returncode, proc._popen, proc._fd, proc.pump = p.pid, None, p, -1, None
        proc._fut = loop.run_in_executor(None, p.wait)
    else:
        proc = PidProc(p, fd)
    if pump_info is not None:
        proc.pump = _reap_later(*pump_info)
    return proc

class Sandbox:
    def __init__(self, sid, config_bytes, meta, labels, annotations, log_dir):
        self.id, self.config_bytes = sid, config_bytes
        self.meta, self.labels, self.annotations, self.log_dir = meta, labels, annotations, log_dir
        self.state = C.SANDBOX_READY
        self.created_at = now_ns()
        self.pid = 0
        self.proc = None
        self.ip = ""
        self.pod_network = False   # the network plugin set this sandbox up (CNI DEL on teardown)
        self.own_ns = False        # the sandbox holds its own net/ipc/uts namespaces (pod networking)
        self.resolv = False        # rootfs/<id>/resolv.conf was written (the pod's DNS config)
        self.port_mappings: list[dict] = []

    def to_json(self):
        return {"id": self.id, "meta": self.meta, "labels": self.labels, "annotations": self.annotations,
                "log_dir": self.log_dir, "state": self.state, "created_at": self.created_at, "pid": self.pid,
                "ip": self.ip, "pod_network": self.pod_network, "own_ns": self.own_ns, "port_mappings": self.port_mappings}


class Container:
    def __init__(self, cid, sandbox_id, name, attempt, image, image_ref, argv, env, cwd, log_path, labels, annotations,
                 mounts, devices, handler, resources):
        self.id, self.sandbox_id, self.name, self.attempt = cid, sandbox_id, name, attempt
        self.image, self.image_ref, self.argv, self.env, self.cwd = image, image_ref, argv, env, cwd
        self.log_path, self.labels, self.annotations = log_path, labels, annotations
        self.mounts, self.devices, self.handler, self.resources = mounts, devices, handler, resources
        self.state = C.CONTAINER_CREATED
        self.created_at = now_ns()
        self.started_at = 0
        self.finished_at = 0
        self.exit_code = 0
        self.reason = ""
        self.message = ""
        self.pid = 0
        self.proc: PidProc | None = None
        self.waiter: asyncio.Task | None = None

    def to_json(self):
        d = {k: getattr(self, k) for k in ("id", "sandbox_id", "name", "attempt", "image", "image_ref", "argv", "env", "cwd",
                                            "log_path", "labels", "annotations", "mounts", "devices", "handler", "resources",
                                            "state", "created_at", "started_at", "finished_at", "exit_code", "reason",
                                            "message", "pid")}
        return d


def _prepare_sandbox_fs(log_dir: str, rootfs: str, resolv: str | None):
    os.makedirs(log_dir, exist_ok=True)
    os.makedirs(rootfs, exist_ok=True)
    if resolv is not None:
        with open(os.path.join(rootfs, "resolv.conf"), "w") as f:
            f.write(resolv)


def _prepare_container_fs(root: str, log_dir: str, links: list[tuple[str, str]]):
    """A container's directories and volume links (run in a worker thread: directory creation
    costs ~0.2 ms a call on a journaled filesystem, several per container)."""
    os.makedirs(root, exist_ok=True)
    os.makedirs(log_dir, exist_ok=True)
    made = set()
    for link, target in links:
        parent = os.path.dirname(link)
        if parent not in made:
            os.makedirs(parent, exist_ok=True)
            made.add(parent)
        if not os.path.lexists(link):
            os.symlink(target, link)


class CheckpointWriter:
    """Sandbox/container checkpoints written off the event loop (the image filesystem of a busy
    node makes every open/replace/unlink cost ~0.3-1 ms, and a pod costs ~6 of them). One
    writer thread drains the latest payload per file (None = delete), so a burst of updates to
    one object costs one write. flush() (stop, tests) waits until everything queued is on disk;
    a crash can lose at most the updates of the last few milliseconds, which recovery treats
    like a missed event (the processes themselves are re-adopted from their pid/exit files)."""

    def __init__(self):
        self._pending: dict[str, bytes | None] = {}
        self._cv = threading.Condition()
        self._busy = False
        self._stop = False
        self._t = threading.Thread(target=self._run, name="rocshim-ckpt", daemon=True)
        self._t.start()

    def put(self, path: str, data: bytes | None):
        with self._cv:
            self._pending[path] = data
            self._cv.notify_all()

    def _run(self):
        while True:
            with self._cv:
                while not self._pending and not self._stop:
                    self._cv.wait()
                if not self._pending and self._stop:
                    return
                batch, self._pending = self._pending, {}
                self._busy = True
            for path, data in batch.items():
                try:
                    if data is None:
                        try:
                            os.unlink(path)
                        except FileNotFoundError:
                            pass
                    else:
                        tmp = path + ".tmp"
                        with open(tmp, "wb") as f:
                            f.write(data)
                        os.replace(tmp, path)
                except OSError as e:
                    log.warning("checkpoint %s: %s", path, e)
            with self._cv:
                self._busy = False
                self._cv.notify_all()

    def flush(self, timeout: float = 10.0):
        end = time.monotonic() + timeout
        with self._cv:
            while (self._pending or self._busy) and time.monotonic() < end:
                self._cv.wait(0.05)

    def close(self):
        self.flush()
        with self._cv:
            self._stop = True
            self._cv.notify_all()


class RocShim:
    cgroup_driver = "cgroupfs"               # --cgroup-driver (systemd: slices and transient scopes)
    systemd = None                           # kubelet.cgroups.SystemdUnits under the systemd driver

    def __init__(self, socket_path: str, state_dir: str, hooks_dir: str = DEFAULT_HOOKS_DIR, isolation: str = "env",
                 cgroup_root: str = "/sys/fs/cgroup/amdkube", dev_root: str = "/dev", network=None,
                 pod_namespaces: bool = False, registry_dir: str | None = None, insecure_registries=(),
                 registry_ca: str | None = None, cgroup_driver: str = "cgroupfs", systemd_units=None):
        self.socket = socket_path
        self.state_dir = state_dir
        # the node's environment minus GPU visibility, read once (iterating os.environ per
        # container start re-decodes every variable)
        self._host_env = {k: v for k, v in os.environ.items() if k not in SCRUB_ENV}
        os.makedirs(os.path.join(state_dir, "sandboxes"), exist_ok=True)
        os.makedirs(os.path.join(state_dir, "containers"), exist_ok=True)
        os.makedirs(os.path.join(state_dir, "rootfs"), exist_ok=True)
        from .registry import RegistryClient
        self.images = ImageStore(state_dir, registry_dir, RegistryClient(insecure_registries, registry_ca))
        self.ckpt = CheckpointWriter()
        self.hooks = HookService(hooks_dir, HANDLERS)
        self.isolation_probe = probe_isolation() if isolation in ("auto", "landlock", "namespaces", "userns") else {}
        self.isolation = resolve_isolation(isolation, self.isolation_probe)
        self.network = network or HostNetwork()
        # pod networking: non-hostNetwork sandboxes get their own net/ipc/uts namespaces (needs
        # a privileged rocshim) wired by the network plugin (amdkube-bridge); containers join them
        self.pod_namespaces = pod_namespaces
        from .hostport import HostPortManager
        from ..monitoring.cadvisor import DuCache
        self.hostports = HostPortManager()
        self.du = DuCache(10.0)
        # cgroupfs: the runtime's own tree under cgroup_root (kubepods/... leaves it makes itself);
        # systemd: systemd owns the hierarchy from the cgroup mount, pods are slices the kubelet
        # names (kubepods-burstable-pod<uid>.slice) and each container a transient scope
        from ..kubelet.cgroups import CGROUPFS, SYSTEMD, CgroupError, SystemdUnits, use_systemd
        if cgroup_driver not in (CGROUPFS, SYSTEMD):
            raise CgroupError(f"invalid cgroup driver {cgroup_driver!r} (cgroupfs or systemd)")
        if cgroup_driver == SYSTEMD and systemd_units is None and not (use_systemd() or os.environ.get("AMDKUBE_SYSTEMD_BUS")):
            raise CgroupError("--cgroup-driver=systemd: systemd is not the init system of this node (no /run/systemd/system)")
        self.cgroup_driver = cgroup_driver
        self.systemd = (systemd_units or SystemdUnits()) if cgroup_driver == SYSTEMD else None
        self._slices: set[str] = set()       # pod slices this runtime started (systemd driver)
        self.cgroup_root = cgroup_root
        if cgroup_driver == SYSTEMD:
            from ..kubelet.cgroups import RUNTIME_DEFAULT_ROOT, systemd_cgroup_root
            self.cgroup_root = systemd_cgroup_root(cgroup_root)
            if self.cgroup_root == RUNTIME_DEFAULT_ROOT:       # no cgroup2 mount in view: the usual one
                self.cgroup_root = "/sys/fs/cgroup"
        self.dev_root = dev_root
        self.sandboxes: dict[str, Sandbox] = {}
        self.containers: dict[str, Container] = {}
        self.server: grpc.aio.Server | None = None
        self.pause_bin = os.path.join(NATIVE_BIN, "pause")
        self.nsexec_bin = os.path.join(NATIVE_BIN, "amdkube-nsexec")
        self.started = 0
        self._adopt_tasks: set = set()
        self._event_streams: set[asyncio.Queue] = set()
        self._starting: set[str] = set()     # container ids whose process is being launched
        self._launching = 0                  # process launches in flight (worker threads)
        self._closing = False
        self._last_ev: dict[str, int] = {}   # sandbox id -> created_at of the newest event emitted for it
        self.streaming = None
        self.streaming_port = 0     # loopback port of the exec/attach/port-forward server (0: any)

    def _emit(self, c: "Container | None", etype: int, sid: str | None = None):
        """Evented PLEG (KEP-3386 ContainerEventResponse): every event carries the sandbox's full
        status and the statuses of all its containers as of emission, so the kubelet updates its
        runtime cache from the stream instead of re-listing (3 RPCs per pod sync). Sandbox
        lifecycle events use the sandbox id as container_id."""
        if not self._event_streams:
            return
        sid = sid or c.sandbox_id
        sb = self.sandboxes.get(sid)
        ts = max(now_ns(), self._last_ev.get(sid, 0) + 1)   # strictly increasing per sandbox
        self._last_ev[sid] = ts
        sst = sandbox_status_msg(sb, self.network.node_ip) if sb is not None else C.PodSandboxStatus(id=sid)
        ev = C.ContainerEventResponse(container_id=c.id if c is not None else sid, container_event_type=etype, created_at=ts,
                                      pod_sandbox_status=sst,
                                      containers_statuses=[container_status_msg(x) for x in self.containers.values()
                                                           if x.sandbox_id == sid])
        for q in list(self._event_streams):
            q.put_nowait(ev)

    def _emit_removed(self, s: "Sandbox"):
        if not self._event_streams:
            return
        ts = max(now_ns(), self._last_ev.get(s.id, 0) + 1)
        self._last_ev[s.id] = ts
        ev = C.ContainerEventResponse(container_id=s.id, container_event_type=C.CONTAINER_DELETED_EVENT, created_at=ts,
                                      pod_sandbox_status=C.PodSandboxStatus(id=s.id, metadata=sandbox_meta(s)))
        for q in list(self._event_streams):
            q.put_nowait(ev)

    def event_mark(self, sid: str | None) -> str:
        """Trailer of a mutating CRI call: `<sandbox id>:<created_at>` of the newest event emitted
        for the call's sandbox when the call returns (its state as of the return is the one that
        event carries), or empty when no event exists to wait for (unknown target, no stream).
        The kubelet matches its runtime cache to exactly that event (a container
        event emitted before the sandbox's own STOPPED event must not count as the final state)."""
        ts = self._last_ev.get(sid or "", 0)
        if not sid or not ts:
            return ""
        if sid not in self.sandboxes:
            self._last_ev.pop(sid, None)     # removed: nothing more will be emitted for it
        return f"{sid}:{ts}"

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        await self.hooks.start()
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
        log.info("rocshim serving CRI on %s (isolation=%s)", self.socket, self.isolation)
        return self

    async def _launch(self, argv, **kw):
        """spawn() for a sandbox or container; a launch that completes after stop() began is
        killed at once (otherwise it would outlive the runtime that no longer tracks it)."""
        if self._closing:
            raise RuntimeError("the runtime is shutting down")
        self._launching += 1
        try:
            proc = await spawn(argv, **kw)
        finally:
            self._launching -= 1
        if self._closing:
            _killpg(proc.pid, signal.SIGKILL)
            await proc.wait()
            raise RuntimeError("the runtime is shutting down")
        return proc

    async def stop(self, kill_pods: bool = False):
        self._closing = True
        deadline = time.monotonic() + 5.0
        while self._launching and time.monotonic() < deadline:     # launches in worker threads land first
            await asyncio.sleep(0.01)
        if kill_pods:
            for s in list(self.sandboxes.values()):
                await self.stop_sandbox(s.id)
        await self.hooks.stop()
        await self.hostports.close()
        if self.streaming is not None:
            await self.streaming.stop()
        if self.server:
            await self.server.stop(0.5)
        for t in list(self._adopt_tasks):
            t.cancel()
        await asyncio.to_thread(self.ckpt.flush)

    # --------------------------------------------------------------- checkpoints
    def _ckpt(self, kind: str, obj):
        # encoded now (the state as of this call), written by the checkpoint thread
        self.ckpt.put(os.path.join(self.state_dir, kind, obj.id + ".json"),
                      json.dumps(obj.to_json(), separators=(",", ":")).encode())

    def _unckpt(self, kind: str, oid: str):
        self.ckpt.put(os.path.join(self.state_dir, kind, oid + ".json"), None)

    def _recover(self):
        for name in os.listdir(os.path.join(self.state_dir, "sandboxes")):
            if not name.endswith(".json"):
                continue
            try:
                d = json.load(open(os.path.join(self.state_dir, "sandboxes", name)))
            except (OSError, ValueError):
                continue
            s = Sandbox(d["id"], b"", d["meta"], d["labels"], d["annotations"], d["log_dir"])
            s.state, s.created_at, s.pid = d["state"], d["created_at"], d["pid"]
            s.ip, s.pod_network = d.get("ip", ""), d.get("pod_network", False)
            s.own_ns, s.port_mappings = d.get("own_ns", False), d.get("port_mappings") or []
            s.resolv = os.path.exists(os.path.join(self.state_dir, "rootfs", s.id, "resolv.conf"))
            if s.state == C.SANDBOX_READY and not _alive(s.pid):
                s.state = C.SANDBOX_NOTREADY
            self.sandboxes[s.id] = s
        for name in os.listdir(os.path.join(self.state_dir, "containers")):
            if not name.endswith(".json"):
                continue
            try:
                d = json.load(open(os.path.join(self.state_dir, "containers", name)))
            except (OSError, ValueError):
                continue
            c = Container(d["id"], d["sandbox_id"], d["name"], d["attempt"], d["image"], d["image_ref"], d["argv"], d["env"],
                          d["cwd"], d["log_path"], d["labels"], d["annotations"], d["mounts"], d["devices"], d["handler"],
                          d["resources"])
            for k in ("state", "created_at", "started_at", "finished_at", "exit_code", "reason", "message", "pid"):
                setattr(c, k, d[k])
            self.containers[c.id] = c
            if c.state == C.CONTAINER_RUNNING:
                if _alive(c.pid):
                    t = asyncio.create_task(self._adopt(c))
                    self._adopt_tasks.add(t)
                    t.add_done_callback(self._adopt_tasks.discard)
                else:
                    self._finish(c, self._exit_code_file(c))
        log.info("recovered %d sandboxes, %d containers", len(self.sandboxes), len(self.containers))

    def _exit_code_file(self, c) -> int | None:
        try:
            with open(os.path.join(self.state_dir, "containers", c.id + ".exit")) as f:
                return int(f.read().strip())
        except (OSError, ValueError):
            return None

    async def _adopt(self, c: Container):
        while _alive(c.pid):
            await asyncio.sleep(0.2)
        self._finish(c, self._exit_code_file(c))

    # ----------------------------------------------------------------- sandboxes
    async def run_sandbox(self, cfg) -> str:
        sid = uuid.uuid4().hex
        meta = {"name": cfg.metadata.name, "uid": cfg.metadata.uid, "namespace": cfg.metadata.namespace,
                "attempt": cfg.metadata.attempt}
        log_dir = cfg.log_directory or os.path.join(self.state_dir, "logs", sid)
        sysctls = dict(cfg.linux.sysctls) if cfg.HasField("linux") else {}
        nso = None
        try:
            nso = cfg.linux.security_context.namespace_options
        except AttributeError:
            pass
        host_net = bool(nso.host_network) if nso is not None else True
        host_ipc = bool(nso.host_ipc) if nso is not None else True
        own_ns = self.pod_namespaces and not host_net and not isinstance(self.network, HostNetwork)
        for k in sysctls:
            # a namespaced sysctl is only safe inside the pod's own namespace: net.* needs the
            # pod network namespace, the IPC ones (kernel.shm*, kernel.msg*, kernel.sem,
            # fs.mqueue.*) its IPC namespace — otherwise it would change the host
            ipc_key = not k.startswith("net.")
            if not own_ns or (ipc_key and host_ipc):
                raise ValueError(f"sysctl {k}: the sandbox shares the host's {'ipc' if ipc_key else 'net'} namespace "
                                 f"(pod namespaces={'on' if self.pod_namespaces else 'off'}); refusing to change host "
                                 f"kernel parameters")
        s = Sandbox(sid, cfg.SerializeToString(), meta, dict(cfg.labels), dict(cfg.annotations), log_dir)
        s.port_mappings = [{"host_ip": pm.host_ip, "host_port": pm.host_port, "container_port": pm.container_port,
                            "protocol": {0: "TCP", 1: "UDP"}.get(int(pm.protocol), "TCP")} for pm in cfg.port_mappings]
        dns = cfg.dns_config if cfg.HasField("dns_config") else None
        resolv = None
        if dns is not None and (dns.servers or dns.searches or dns.options):
            # the pod's resolv.conf (dockershim rewriteResolvFile), mounted at /etc/resolv.conf
            lines = [f"nameserver {x}" for x in dns.servers]
            if dns.searches:
                lines.append("search " + " ".join(dns.searches))
            if dns.options:
                lines.append("options " + " ".join(dns.options))
            resolv = "\n".join(lines) + "\n"
        await asyncio.to_thread(_prepare_sandbox_fs, log_dir, os.path.join(self.state_dir, "rootfs", sid), resolv)
        s.resolv = resolv is not None
        if own_ns:
            # the pause process owns the pod's namespaces; sysctls are written inside them
            argv = [self.nsexec_bin, "--no-namespaces", "--unshare", "net,uts" if host_ipc else "net,ipc,uts"]
            if cfg.hostname:
                argv += ["--hostname", cfg.hostname]
            for k, v in sorted(sysctls.items()):
                argv += ["--sysctl", f"{k}={v}"]
            proc = await self._launch(argv + ["--", self.pause_bin])
        else:
            proc = await self._launch([self.pause_bin])
        s.proc, s.pid = proc, proc.pid
        s.own_ns = own_ns
        if host_net or isinstance(self.network, HostNetwork):
            s.ip = self.network.node_ip
        else:
            try:
                if own_ns:
                    await _wait_ns(s.pid, proc)
                s.ip = await self.network.setup(sid, meta, f"/proc/{s.pid}/ns/net")
                s.pod_network = True
                if own_ns:
                    await self.hostports.add(sid, s.ip, s.port_mappings)
            except Exception:
                await self.network.teardown(sid, meta, f"/proc/{s.pid}/ns/net")  # release a partial ADD
                _kill(s.pid, signal.SIGKILL)
                await proc.wait()
                raise
        self.sandboxes[sid] = s
        self._ckpt("sandboxes", s)
        self._emit(None, C.CONTAINER_STARTED_EVENT, sid)
        return sid

    async def stop_sandbox(self, sid: str):
        s = self.sandboxes.get(sid)
        if s is None:
            return
        await asyncio.gather(*(self.stop_container(c.id, 2) for c in list(self.containers.values()) if c.sandbox_id == sid))
        await self.hostports.remove(sid)
        if s.pod_network and s.own_ns and s.pid and _alive(s.pid):
            # the pod's network namespace dies with pause: tear the network down first
            # (dockershim StopPodSandbox: TearDownPod before stopping the infra container)
            await self.network.teardown(sid, s.meta, f"/proc/{s.pid}/ns/net")
            s.pod_network = False
        if s.pid and _alive(s.pid):
            _kill(s.pid, signal.SIGTERM)
            if s.proc is not None:
                try:
                    await asyncio.wait_for(s.proc.wait(), 2)
                except asyncio.TimeoutError:
                    _kill(s.pid, signal.SIGKILL)
        if s.pod_network:
            await self.network.teardown(sid, s.meta, f"/proc/{s.pid}/ns/net")
            s.pod_network = False
        s.state = C.SANDBOX_NOTREADY
        self._ckpt("sandboxes", s)
        self._emit(None, C.CONTAINER_STOPPED_EVENT, sid)

    async def remove_sandbox(self, sid: str):
        s = self.sandboxes.get(sid)
        if s is None:
            return
        if s.state == C.SANDBOX_READY:
            await self.stop_sandbox(sid)
        for c in [c for c in self.containers.values() if c.sandbox_id == sid]:
            await self.remove_container(c.id)
        self.sandboxes.pop(sid, None)
        self._unckpt("sandboxes", sid)
        if self.systemd is not None:
            slice_name = self._sandbox_slice(s)
            if slice_name in self._slices:
                self._slices.discard(slice_name)
                try:
                    await asyncio.to_thread(self.systemd.stop, slice_name)
                except Exception as e:
                    log.debug("systemd: stopping %s: %r", slice_name, e)
        self._emit_removed(s)
        await asyncio.to_thread(shutil.rmtree, os.path.join(self.state_dir, "rootfs", sid), True)

    # --------------------------------------------------------------- containers
    async def create_container(self, sid: str, cfg, sandbox_cfg) -> str:
        s = self.sandboxes.get(sid)
        if s is None or s.state != C.SANDBOX_READY:
            raise LookupError(f"sandbox {sid} not found or not ready")
        res = self.images.resolve(cfg.image.image)
        if res is None:
            raise LookupError(f"image {cfg.image.image!r} not present (PullImage first)")
        iname, ispec = res
        entry = list(cfg.command) or list(ispec.get("entrypoint") or [])
        args = list(cfg.args) if (cfg.args or cfg.command) else list(ispec.get("cmd") or [])
        argv = entry + args
        if not argv:
            raise ValueError("no command specified and the image has no entrypoint")
        image_root = ispec.get("rootfs") if ispec.get("kind") == "rootfs" else None
        if image_root:
            # a real image: its own environment (docker's image Env + the container's), not the host's
            env = {"PATH": DEFAULT_PATH}
        else:
            env = dict(self._host_env)
        env.update(ispec.get("env") or {})
        for kv in cfg.envs:
            env[kv.key] = kv.value
        devices = [{"container_path": d.container_path, "host_path": d.host_path, "permissions": d.permissions}
                   for d in cfg.devices]
        has_gpu = any(d["host_path"].endswith("/kfd") for d in devices)
        if not has_gpu:
            env.pop("ROCR_VISIBLE_DEVICES", None)
            env["HIP_VISIBLE_DEVICES"] = "-1"  # non-GPU containers see no GPU
        for d in devices:
            if not os.path.exists(d["host_path"]) and self.isolation in ("namespaces", "userns", "landlock"):
                raise FileNotFoundError(f"device {d['host_path']} does not exist on this host")
        tags = [iname] + [t for t in ispec.get("repo_tags") or [] if t != iname]
        handler = self.hooks.get_runtime(tags, dict(cfg.annotations), dict(sandbox_cfg.annotations) if sandbox_cfg else {})
        if not handler:
            handler = "rocm" if has_gpu else "default"
        if image_root and handler == "rocm":
            # the rocm handler brings the node's ROCm runtime settings into the image
            env.update({k: v for k, v in self._host_env.items() if k.startswith("HSA_") and k not in env})
        cid = uuid.uuid4().hex
        root = os.path.join(self.state_dir, "rootfs", sid, cfg.metadata.name)
        if image_root:
            workdir = cfg.working_dir or ispec.get("workdir") or "/"
            cwd = os.path.join(image_root, workdir.lstrip("/"))    # path-rooted launch; nsexec chdirs itself
            if not os.path.isdir(cwd):
                cwd = image_root
        else:
            workdir = ""
            cwd = cfg.working_dir or ispec.get("workdir") or root
            if cwd != root and not os.path.isdir(cwd):      # root itself is created below
                cwd = root
        log_path = os.path.join(s.log_dir, cfg.log_path) if cfg.log_path else os.path.join(s.log_dir, f"{cfg.metadata.name}_{cfg.metadata.attempt}.log")
        mounts = [{"container_path": m.container_path, "host_path": m.host_path, "readonly": m.readonly} for m in cfg.mounts]
        resolv = os.path.join(self.state_dir, "rootfs", sid, "resolv.conf")
        if s.resolv and not any(x["container_path"] == "/etc/resolv.conf" for x in mounts):
            mounts.append({"container_path": "/etc/resolv.conf", "host_path": resolv, "readonly": True})
        # without a mount namespace, expose volumes as symlinks under the container's root
        links = [(os.path.join(root, mnt["container_path"].lstrip("/")), mnt["host_path"]) for mnt in mounts
                 if not self.private_mounts and mnt["container_path"].startswith("/")]
        await asyncio.to_thread(_prepare_container_fs, root, os.path.dirname(log_path), links)
        if self.sandboxes.get(sid) is not s or s.state != C.SANDBOX_READY:
            raise LookupError(f"sandbox {sid} went away while container {cfg.metadata.name} was created")
        env["AMDKUBE_ROOTFS"] = root
        if image_root and not self.private_mounts:
            # no mount namespace: the rootview preload makes the image's root the process's `/`
            from .rootless import rootview_env
            env.update(rootview_env(image_root, mounts, root, ROCM_INJECT if handler == "rocm" else (), env, workdir))
        r = cfg.linux.resources if cfg.HasField("linux") else None
        resources = {"cpu_quota": r.cpu_quota, "cpu_period": r.cpu_period, "memory_limit": r.memory_limit_in_bytes,
                     "cpu_shares": r.cpu_shares, "oom_score_adj": r.oom_score_adj, "cpuset": r.cpuset_cpus} if r else {}
        if sandbox_cfg is not None and sandbox_cfg.HasField("linux") and sandbox_cfg.linux.cgroup_parent:
            resources["cgroup_parent"] = self._cgroup_parent(sandbox_cfg.linux.cgroup_parent)
        sc = cfg.linux.security_context if cfg.HasField("linux") and cfg.linux.HasField("security_context") else None
        if image_root:
            resources["rootfs"], resources["workdir"] = image_root, workdir
            user = ispec.get("user") or ""
            if sc is not None and sc.HasField("run_as_user"):
                user = str(sc.run_as_user.value)
            if user:
                resources["user"] = user
        resources["caps"] = container_caps(sc)
        resources["privileged"] = bool(sc is not None and sc.privileged)
        if self.isolation in ("landlock", "userns", "namespaces") and handler == "rocm":
            env = self._guarded_env(env, devices)
        sec = cfg.linux.security_context.seccomp_profile_path if cfg.HasField("linux") else ""
        if sec:
            resources["seccomp_profile"] = self._seccomp_file(sec)
        aa = cfg.linux.security_context.apparmor_profile if cfg.HasField("linux") else ""
        if aa.startswith("localhost/"):   # runtime/default and unconfined: no transition
            resources["apparmor_profile"] = aa[len("localhost/"):]
        elif aa not in ("", "runtime/default", "unconfined"):
            raise ValueError(f"unsupported AppArmor profile {aa!r}")
        c = Container(cid, sid, cfg.metadata.name, cfg.metadata.attempt, cfg.image.image, self.images.image_id(iname), argv,
                      env, cwd, log_path, dict(cfg.labels), dict(cfg.annotations), mounts, devices, handler, resources)
        self.containers[cid] = c
        self._ckpt("containers", c)
        self._emit(c, C.CONTAINER_CREATED_EVENT)
        return cid

    @staticmethod
    def _seccomp_file(spec: str) -> str:
        """CRI seccomp_profile_path: runtime/default → rocshim's built-in profile, localhost/<abs path>."""
        if spec in ("runtime/default", "docker/default"):
            return os.path.join(os.path.dirname(__file__), "seccomp_default.json")
        if spec.startswith("localhost/"):
            p = spec[len("localhost"):]
            if not os.path.isfile(p):
                raise LookupError(f"seccomp profile {p} not found")
            return p
        raise ValueError(f"unsupported seccomp profile {spec!r}")

    def _join_args(self, c: Container) -> list[str]:
        s = self.sandboxes.get(c.sandbox_id)
        if s is None or not s.own_ns or not s.pid:
            return []
        out = []
        for t in ("net", "ipc", "uts"):
            p = f"/proc/{s.pid}/ns/{t}"
            if t == "ipc" and os.path.exists(p) and os.path.realpath(p) == os.path.realpath("/proc/self/ns/ipc"):
                continue     # hostIPC pod: nothing to join
            out += ["--join", f"{t}:{p}"]
        return out

    @property
    def private_mounts(self) -> bool:
        """The container gets its own mount namespace (volumes are bind mounts, not links)."""
        return self.isolation in ("namespaces", "userns")

    def _guarded_env(self, env: dict, devices: list[dict]) -> dict:
        """`rocm` handler under a device guard: the container's view is exactly its devices.
        ROCR_VISIBLE_DEVICES ordinals index the host's full GPU list, which the container no
        longer sees, so an ordinal-only list is dropped (the view already selects); UUIDs stay.
        Landlock mode adds the devview preload (absent, not refused, foreign nodes)."""
        env = dict(env)
        vis = env.get("ROCR_VISIBLE_DEVICES")
        if vis and all(t.strip().isdigit() for t in vis.split(",")):
            env.pop("ROCR_VISIBLE_DEVICES")
        if self.isolation == "landlock" and os.path.exists(DEVVIEW_LIB):
            # armed by amdkube-nsexec right before it execs the workload (LD_PRELOAD), so the
            # launcher's own walk of the device root for the Landlock ruleset is unfiltered
            env["AMDKUBE_DEVVIEW_LIB"] = DEVVIEW_LIB
            env["AMDKUBE_DEVVIEW_ROOT"] = self.dev_root
            env["AMDKUBE_DEVVIEW_ALLOW"] = ",".join(d["host_path"] for d in devices)
        return env

    def _device_args(self, c: Container) -> list[str]:
        """--keep (render/card nodes the container was given) and --hide-kfd (no GPU)."""
        if c.resources.get("privileged"):
            return []
        a = []
        for d in c.devices:
            if "/dri/" in d["host_path"]:
                a += ["--keep", d["host_path"]]
        if not any(d["host_path"].endswith("/kfd") for d in c.devices):
            a += ["--hide-kfd"]
        return a

    def _launch_argv(self, c: Container) -> list[str]:
        sec, aa = c.resources.get("seccomp_profile"), c.resources.get("apparmor_profile")
        cpuset = c.resources.get("cpuset") or ""
        join = self._join_args(c)
        argv = c.argv
        if c.resources.get("rootfs") and not self.private_mounts:
            # no mount namespace on this node: run the image's own files through its own loader
            from .rootless import rootfs_argv
            argv = rootfs_argv(c.resources["rootfs"], c.argv, c.env.get("PATH", DEFAULT_PATH), c.resources.get("workdir") or "/")
            c = _with_argv(c, argv)
        if self.isolation == "landlock":
            dev = ([] if c.resources.get("privileged") else ["--landlock"]) + ["--dev-root", self.dev_root] + self._device_args(c)
            return ([self.nsexec_bin, "--no-namespaces"] + dev + join + (["--seccomp", sec] if sec else []) +
                    (["--apparmor", aa] if aa else []) + (["--cpuset", cpuset] if cpuset else []) + ["--"] + c.argv)
        if not self.private_mounts:
            if not (sec or aa or cpuset or join):
                return c.argv
            return ([self.nsexec_bin, "--no-namespaces"] + join + (["--seccomp", sec] if sec else []) +
                    (["--apparmor", aa] if aa else []) + (["--cpuset", cpuset] if cpuset else []) + ["--"] + c.argv)
        # (env isolation: the OOM score is applied to the spawned process directly, see start_container)
        a = [self.nsexec_bin, "--dev-root", self.dev_root] + join
        if c.resources.get("rootfs"):
            a += ["--rootfs", c.resources["rootfs"], "--rootfs-upper", self._upper_of(c),
                  "--workdir", c.resources.get("workdir") or "/"]
            if c.resources.get("user") and self.isolation == "namespaces":
                a += ["--user", c.resources["user"]]
        if self.isolation == "userns":
            a += ["--userns"]
        else:
            # QoS hierarchy from the kubelet (kubepods/[burstable|besteffort]/pod<uid>), else per sandbox
            a += ["--cgroup", self._cgroup_of(c)]
            if self.isolation_probe.get("cgroup2") and not c.resources.get("privileged"):
                a += ["--device-cgroup"]
        if self.isolation_probe.get("landlock_abi", 0) >= 1 and not c.resources.get("privileged"):
            a += ["--landlock"]
        a += ["--caps", c.resources.get("caps") or ",".join(DEFAULT_CAPS)]
        if c.resources.get("cpu_shares"):
            a += ["--cpu-weight", str(_shares_to_weight(c.resources["cpu_shares"]))]
        if c.resources.get("oom_score_adj"):
            a += ["--oom-score-adj", str(c.resources["oom_score_adj"])]
        if sec:
            a += ["--seccomp", sec]
        if aa:
            a += ["--apparmor", aa]
        for mnt in c.mounts:   # volumes and the pod's resolv.conf in the private mount namespace
            if mnt["container_path"].startswith("/") and os.path.exists(mnt["host_path"]):
                a += ["--bind", f"{mnt['host_path']}:{mnt['container_path']}" + (":ro" if mnt.get("readonly") else "")]
        if c.resources.get("rootfs") and c.handler == "rocm":
            # the rocm handler's injection (the nvidia runtime's driver-library hook, re-homed):
            # the node's ROCm user space, read-only, unless a volume already provides it
            taken = {m["container_path"] for m in c.mounts}
            for host in ROCM_INJECT:
                if os.path.exists(host) and host not in taken:
                    a += ["--bind", f"{host}:{host}:ro"]
        a += [x for x in self._device_args(c) if x != "--hide-kfd"]
        if c.resources.get("memory_limit"):
            a += ["--memory-max", str(c.resources["memory_limit"])]
        if c.resources.get("cpu_quota") and c.resources.get("cpu_period"):
            a += ["--cpu-max", f"{c.resources['cpu_quota']} {c.resources['cpu_period']}"]
        if cpuset:
            a += ["--cpuset", cpuset]
        if "--hide-kfd" in self._device_args(c):
            a += ["--hide-kfd"]
        return a + ["--"] + c.argv

    def exec_argv(self, c: Container, cmd: list[str]) -> list[str]:
        """A process started inside a running container (CRI Exec/ExecSync; docker exec): the
        container's mount (and user) namespace, its sandbox's net/ipc/uts, its cgroup, and the
        same device guard, capability bound, seccomp and AppArmor as the container itself."""
        sec, aa = c.resources.get("seccomp_profile"), c.resources.get("apparmor_profile")
        cpuset = c.resources.get("cpuset") or ""
        join = self._join_args(c)
        argv = list(cmd)
        if c.resources.get("rootfs") and not self.private_mounts:
            from .rootless import rootfs_argv
            argv = rootfs_argv(c.resources["rootfs"], argv, c.env.get("PATH", DEFAULT_PATH), c.resources.get("workdir") or "/")
        guard = self.isolation == "landlock" or (self.private_mounts and self.isolation_probe.get("landlock_abi", 0) >= 1)
        if not (self.private_mounts or guard or sec or aa or cpuset or join):
            return argv
        a = [self.nsexec_bin, "--no-namespaces"]
        if self.private_mounts and c.pid:
            if self.isolation == "userns":
                a += ["--join", f"user:/proc/{c.pid}/ns/user"]
            a += ["--join", f"mnt:/proc/{c.pid}/ns/mnt"]
            if c.resources.get("rootfs"):
                a += ["--workdir", c.resources.get("workdir") or "/"]
            if self.isolation != "userns":
                a += ["--cgroup", self._cgroup_of(c)]
        a += join
        if guard and not c.resources.get("privileged"):
            a += ["--landlock", "--dev-root", self.dev_root] + self._device_args(c)
        if self.private_mounts:
            a += ["--caps", c.resources.get("caps") or ",".join(DEFAULT_CAPS)]
        a += (["--seccomp", sec] if sec else []) + (["--apparmor", aa] if aa else []) + (["--cpuset", cpuset] if cpuset else [])
        return a + ["--"] + argv

    def exec_cwd(self, c: Container) -> str | None:
        """Where an exec'd process starts before nsexec moves it (a joined mount namespace
        resets it to the container's root)."""
        return None if self.private_mounts else c.cwd

    def _upper_of(self, c: Container) -> str:
        """The container's writable layer (overlay upper/work and the merged mount point)."""
        return os.path.join(self.state_dir, "rootfs", c.sandbox_id, c.name, ".layer")

    def _sandbox_slice(self, s) -> str:
        try:
            cfg = C.PodSandboxConfig.FromString(s.config_bytes)
            return os.path.basename(self._cgroup_parent(cfg.linux.cgroup_parent)) if cfg.linux.cgroup_parent else ""
        except Exception:
            return ""

    def _cgroup_parent(self, parent: str) -> str:
        """The pod's cgroup as a path under cgroup_root. systemd: a slice name
        (kubepods-burstable-pod<uid>.slice, as dockershim's ConvertCgroupFsNameToSystemd hands
        docker) or its expanded form; anything else is refused, as runc's systemd driver does."""
        if self.cgroup_driver != "systemd":
            return parent.strip("/")
        from ..kubelet.cgroups import CgroupError, expand_slice
        base = os.path.basename(parent.rstrip("/"))
        if not base.endswith(".slice"):
            raise CgroupError(f"cgroup parent {parent!r}: the systemd cgroup driver needs a *.slice parent")
        return expand_slice(base).strip("/")

    def _cgroup_of(self, c: Container) -> str:
        if self.cgroup_driver == "systemd":
            parent = c.resources.get("cgroup_parent") or "amdkube.slice"
            return os.path.join(self.cgroup_root, parent, f"amdkube-{c.id}.scope")
        return os.path.join(self.cgroup_root, c.resources.get("cgroup_parent") or c.sandbox_id, c.id)

    def _scope_properties(self, c: Container, pid: int) -> list:
        """The transient scope of a container (runc's systemd driver: Slice, PIDs, Delegate and
        the resource limits as unit properties)."""
        from ..kubelet.cgroups import unit_properties
        parent = c.resources.get("cgroup_parent") or "amdkube.slice"
        props = [("Description", ("s", f"amdkube container {c.id}")), ("Slice", ("s", os.path.basename(parent))),
                 ("PIDs", ("au", [pid])), ("Delegate", ("b", True)), ("MemoryAccounting", ("b", True)),
                 ("CPUAccounting", ("b", True)), ("DefaultDependencies", ("b", False))]
        return props + unit_properties({"memory": c.resources.get("memory_limit"),
                                        "cpu_weight": _shares_to_weight(c.resources["cpu_shares"]) if c.resources.get("cpu_shares") else 0,
                                        "cpu_quota": c.resources.get("cpu_quota"), "cpu_period": c.resources.get("cpu_period")})

    def _place_in_scope(self, c: Container, pid: int):
        """systemd driver: the pod slice (started once, with its parents implied by the name),
        then the container's scope made with the launcher's pid; blocking D-Bus round trips, run
        off the event loop."""
        slice_name = os.path.basename(c.resources.get("cgroup_parent") or "amdkube.slice")
        if slice_name not in self._slices:
            try:
                self.systemd.start_transient(slice_name, [("Description", ("s", f"amdkube pod {slice_name}"))])
            except Exception as e:
                if "exists" not in str(e):
                    raise
            self._slices.add(slice_name)
        self.systemd.start_transient(f"amdkube-{c.id}.scope", self._scope_properties(c, pid))
        deadline = time.monotonic() + 5
        leaf = self._cgroup_of(c)
        while not os.path.isdir(leaf):
            if time.monotonic() > deadline:
                raise RuntimeError(f"systemd did not create {leaf}")
            time.sleep(0.005)

    def _termination_message(self, c: Container) -> str:
        """kuberuntime_container.go getTerminationMessage: the file the container wrote at its
        terminationMessagePath (≤ 4 KiB), or — policy FallbackToLogsOnError, failed, nothing
        written — the tail of its log (80 lines, 2 KiB)."""
        path = c.annotations.get("io.kubernetes.container.terminationMessagePath", "")
        host = next((mt["host_path"] for mt in c.mounts if mt["container_path"] == path), None) if path else None
        msg = ""
        if host:
            try:
                with open(host, "rb") as f:
                    msg = f.read(4096).decode(errors="replace")
            except OSError:
                pass
        if not msg and c.exit_code and c.annotations.get("io.kubernetes.container.terminationMessagePolicy") == \
                "FallbackToLogsOnError":
            # readLastStringFromContainerLogs: the last 80 lines, at most 2 KiB, decoded
            from ..kubelet.logs import read_text
            msg = read_text(c.log_path, tail=80, keep_last=2048)
        return msg

    def _oom_killed(self, c: Container) -> bool:
        """cgroup v2 memory.events `oom_kill` of the container's leaf (namespaces isolation):
        the container exit was the kernel OOM killer's doing (docker's State.OOMKilled)."""
        if self.isolation != "namespaces":
            return False
        try:
            with open(os.path.join(self._cgroup_of(c), "memory.events")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "oom_kill" and int(v) > 0:
                        return True
        except (OSError, ValueError):
            pass
        return False

    async def start_container(self, cid: str):
        c = self.containers.get(cid)
        if c is None:
            raise LookupError(f"container {cid} not found")
        if c.state != C.CONTAINER_CREATED or cid in self._starting:
            raise ValueError(f"container {cid} is not in created state")
        self._starting.add(cid)          # the launch below yields the loop: no second start meanwhile
        try:
            argv = self._launch_argv(c)
            if self.cgroup_driver == "systemd" and "--cgroup" in argv:
                proc = await self._launch_in_scope(c, argv)
            else:
                proc = await self._launch(argv, env=c.env, cwd=c.cwd, log_path=c.log_path, log_pump=True,
                                          oom_score_adj=c.resources.get("oom_score_adj") if self.isolation != "namespaces" else None)
        except (OSError, ValueError, RuntimeError) as e:
            c.state, c.exit_code, c.reason, c.message = C.CONTAINER_EXITED, 128, "StartError", str(e)
            c.finished_at = now_ns()
            self._ckpt("containers", c)
            raise
        finally:
            self._starting.discard(cid)
        if self.containers.get(cid) is not c:           # removed while it launched
            _killpg(proc.pid, signal.SIGKILL)
            await proc.wait()
            raise LookupError(f"container {cid} was removed while starting")
        c.proc, c.pid = proc, proc.pid
        c.state, c.started_at = C.CONTAINER_RUNNING, now_ns()
        self.started += 1
        self._ckpt("containers", c)
        self._emit(c, C.CONTAINER_STARTED_EVENT)
        c.waiter = asyncio.create_task(self._wait(c))

    async def _launch_in_scope(self, c: Container, argv: list[str]):
        """nsexec waits on a pipe until systemd has put its pid in the container's scope, then
        joins the scope's cgroup (already its own), applies the limits and execs."""
        r, w = os.pipe()
        try:
            argv = argv[:1] + ["--cgroup-wait-fd", str(r)] + argv[1:]
            proc = await self._launch(argv, env=c.env, cwd=c.cwd, log_path=c.log_path, log_pump=True, pass_fds=(r,))
        except BaseException:
            os.close(w)
            raise
        finally:
            os.close(r)
        try:
            await asyncio.to_thread(self._place_in_scope, c, proc.pid)
        except Exception as e:
            os.close(w)                       # EOF: nsexec refuses to run the container
            await proc.wait()
            raise RuntimeError(f"systemd scope for container {c.id}: {e}") from e
        try:
            os.write(w, b"1")
        except OSError as e:
            # nsexec is already gone (BrokenPipeError): reap it and drop the scope made for it
            await proc.wait()
            try:
                await asyncio.to_thread(self.systemd.stop, f"amdkube-{c.id}.scope")
            except Exception as se:
                log.debug("stopping scope of %s: %r", c.id, se)
            raise RuntimeError(f"container {c.id}: launcher exited before joining its scope: {e}") from e
        finally:
            os.close(w)
        return proc

    async def _wait(self, c: Container):
        rc = await c.proc.wait()
        # the exit is reported once the log holds everything the container wrote (as containerd
        # waits for the IO copy): `logs` right after, and the termination-message fallback, see it all
        await c.proc.logs_flushed(0.5)
        # written by the checkpoint thread, ordered before the container's checkpoint and any
        # later removal of the same file
        self.ckpt.put(os.path.join(self.state_dir, "containers", c.id + ".exit"), str(rc).encode())
        self._finish(c, rc)

    def _finish(self, c: Container, rc):
        if c.state == C.CONTAINER_EXITED:
            return
        c.state = C.CONTAINER_EXITED
        c.finished_at = now_ns()
        if rc is None:
            c.exit_code, c.reason = 255, "ContainerStatusUnknown"
        elif rc < 0:
            c.exit_code, c.reason = 128 - rc, "Error"
            if -rc == signal.SIGKILL:
                c.reason = "OOMKilled" if self._oom_killed(c) else "Killed"
        elif rc == 128 + signal.SIGKILL and self._oom_killed(c):   # nsexec reports its child's signal as 128+n
            c.exit_code, c.reason = rc, "OOMKilled"
        else:
            c.exit_code, c.reason = rc, ("Completed" if rc == 0 else "Error")
        c.message = self._termination_message(c)
        self._ckpt("containers", c)
        self._emit(c, C.CONTAINER_STOPPED_EVENT)

    async def stop_container(self, cid: str, timeout: int = 10):
        c = self.containers.get(cid)
        if c is None or c.state != C.CONTAINER_RUNNING:
            return
        _killpg(c.pid, signal.SIGTERM)
        deadline = time.monotonic() + max(0, timeout)
        while c.state == C.CONTAINER_RUNNING and time.monotonic() < deadline:
            await asyncio.sleep(0.02)
        if c.state == C.CONTAINER_RUNNING:
            _killpg(c.pid, signal.SIGKILL)
            if c.waiter is not None:
                try:
                    await asyncio.wait_for(asyncio.shield(c.waiter), 5)
                except asyncio.TimeoutError:
                    pass
            else:
                self._finish(c, -signal.SIGKILL)
        _killpg(c.pid, signal.SIGKILL)  # reap stragglers of the group even after the leader exited

    async def remove_container(self, cid: str):
        c = self.containers.get(cid)
        if c is None:
            return
        if c.state == C.CONTAINER_RUNNING:
            await self.stop_container(cid, 0)
        self.containers.pop(cid, None)
        self._unckpt("containers", cid)
        self._emit(c, C.CONTAINER_DELETED_EVENT)
        if self.isolation == "namespaces":
            if self.systemd is not None:
                try:
                    await asyncio.to_thread(self.systemd.stop, f"amdkube-{c.id}.scope")
                except Exception as e:
                    log.debug("systemd: stopping the scope of %s: %r", c.id, e)
            try:
                os.rmdir(self._cgroup_of(c))   # the container's cgroup leaf (empty once it exited)
            except OSError:
                pass
        self.ckpt.put(os.path.join(self.state_dir, "containers", cid + ".exit"), None)   # unlinked off-loop

    def update_resources(self, cid: str, lr) -> None:
        """CRI UpdateContainerResources (the CPU manager's shared-pool re-pinning): the new
        cpuset applies to every task of the container (its process group; its cgroup leaf too
        under namespaces isolation)."""
        c = self.containers.get(cid)
        if c is None:
            raise LookupError(f"container {cid} not found")
        if lr.cpuset_cpus:
            from ..kubelet.cpumanager import parse_cpuset
            cpus = parse_cpuset(lr.cpuset_cpus)
            c.resources["cpuset"] = lr.cpuset_cpus
            if c.state == C.CONTAINER_RUNNING and c.pid:
                for pid in _group_pids(c.pid):
                    try:
                        os.sched_setaffinity(pid, cpus)
                    except OSError:
                        pass
                if self.isolation == "namespaces":
                    try:
                        with open(os.path.join(self._cgroup_of(c), "cpuset.cpus"), "w") as f:
                            f.write(lr.cpuset_cpus)
                    except OSError:
                        pass
        for k, v in (("memory_limit", lr.memory_limit_in_bytes), ("cpu_quota", lr.cpu_quota), ("cpu_period", lr.cpu_period),
                     ("cpu_shares", lr.cpu_shares)):
            if v:
                c.resources[k] = v
        if self.isolation == "namespaces" and c.state == C.CONTAINER_RUNNING:
            cg = self._cgroup_of(c)
            for fname, val in (("memory.max", lr.memory_limit_in_bytes),
                               ("cpu.max", f"{lr.cpu_quota} {lr.cpu_period}" if lr.cpu_quota and lr.cpu_period else 0),
                               ("cpu.weight", _shares_to_weight(lr.cpu_shares) if lr.cpu_shares else 0)):
                if val:
                    try:
                        with open(os.path.join(cg, fname), "w") as f:
                            f.write(str(val))
                    except OSError:
                        pass
        self._ckpt("containers", c)

    async def exec_sync(self, cid: str, cmd: list[str], timeout: int):
        c = self.containers.get(cid)
        if c is None or c.state != C.CONTAINER_RUNNING:
            raise LookupError(f"container {cid} is not running")
        p = await asyncio.create_subprocess_exec(*self.exec_argv(c, cmd), env=c.env, cwd=self.exec_cwd(c),
                                                 stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE)
        try:
            out, err = await asyncio.wait_for(p.communicate(), timeout or None)
        except asyncio.TimeoutError:
            p.kill()
            return b"", b"timeout", 124
        return out, err, p.returncode


def _shares_to_weight(shares: int) -> int:
    """cgroup v1 cpu.shares → v2 cpu.weight (the runc/systemd conversion)."""
    return max(1, min(10000, 1 + ((shares - 2) * 9999) // 262142))


def _set_oom_score_adj(pid: int, adj: int):
    """Best effort without privileges: raising a score is always allowed, lowering it needs
    CAP_SYS_RESOURCE (then the kernel refuses and the container keeps the inherited value)."""
    try:
        with open(f"/proc/{pid}/oom_score_adj", "w") as f:
            f.write(str(adj))
    except OSError:
        pass


async def _wait_ns(pid: int, proc, timeout: float = 5.0):
    """The pause launcher execs pause only after unsharing: wait until its net namespace is
    not the launcher's parent's (or the process died)."""
    mine = os.path.realpath("/proc/self/ns/net")
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        try:
            if os.readlink(f"/proc/{pid}/ns/net") != os.readlink("/proc/self/ns/net") and \
                    os.readlink(f"/proc/{pid}/exe").endswith("/pause"):
                return
        except OSError:
            raise RuntimeError(f"pod sandbox process {pid} died while setting up its namespaces")
        if proc.returncode is not None:
            raise RuntimeError(f"pod sandbox process exited with {proc.returncode} while setting up its namespaces")
        await asyncio.sleep(0.005)
    raise RuntimeError(f"pod sandbox {pid} did not enter its own namespaces within {timeout}s (mine={mine})")


def sandbox_meta(s) -> "C.PodSandboxMetadata":
    return C.PodSandboxMetadata(name=s.meta["name"], uid=s.meta["uid"], namespace=s.meta["namespace"],
                                attempt=s.meta.get("attempt", 0))


def sandbox_status_msg(s, node_ip: str) -> "C.PodSandboxStatus":
    return C.PodSandboxStatus(id=s.id, metadata=sandbox_meta(s), state=s.state, created_at=s.created_at,
                              network=C.PodSandboxNetworkStatus(ip=s.ip or node_ip), labels=s.labels, annotations=s.annotations)


def container_status_msg(c) -> "C.ContainerStatus":
    return C.ContainerStatus(id=c.id, metadata=C.ContainerMetadata(name=c.name, attempt=c.attempt), state=c.state,
                             created_at=c.created_at, started_at=c.started_at, finished_at=c.finished_at,
                             exit_code=c.exit_code, image=C.ImageSpec(image=c.image), image_ref=c.image_ref,
                             reason=c.reason, message=c.message, labels=c.labels, annotations=c.annotations,
                             mounts=[C.Mount(container_path=m["container_path"], host_path=m["host_path"], readonly=m["readonly"])
                                     for m in c.mounts], log_path=c.log_path)


def _killpg(pid, sig) -> None:
    """Signal a container's process group. Never signal pid/pgid 0 or 1, our own group, or our
    own process: killpg(0) would hit the runtime (and whatever launched it)."""
    if not pid or pid <= 1 or pid == os.getpid() or pid == os.getpgrp():
        return
    try:
        os.killpg(pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _kill(pid, sig) -> None:
    if not pid or pid <= 1 or pid == os.getpid():
        return
    try:
        os.kill(pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _alive(pid: int) -> bool:
    if not pid:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:  # zombies count as dead
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


def _pgid_map() -> dict[int, list[int]]:
    """Process group → its pids, from one /proc pass (a container is a process group)."""
    out: dict[int, list[int]] = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
            out.setdefault(int(parts[2]), []).append(int(d))
        except (OSError, IndexError, ValueError):
            continue
    return out


def _group_pids(pgid: int) -> list[int]:
    """Every task of a container: the members of its process group (rocshim starts each
    container in its own session)."""
    out = []
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
            if int(parts[2]) == pgid:
                out.append(int(d))
        except (OSError, IndexError, ValueError):
            continue
    return out


def _abort(ctx, e):
    code = grpc.StatusCode.NOT_FOUND if isinstance(e, LookupError) else (
        grpc.StatusCode.FAILED_PRECONDITION if isinstance(e, (ValueError, FileNotFoundError)) else grpc.StatusCode.UNKNOWN)
    return ctx.abort(code, str(e))


class _Runtime:
    def __init__(self, r: RocShim):
        self.r = r

    async def Version(self, req, ctx):
        return C.VersionResponse(version=API_VERSION, runtime_name=RUNTIME_NAME, runtime_version=RUNTIME_VERSION,
                                 runtime_api_version="v1alpha1")

    async def Status(self, req, ctx):
        net_ok, net_msg = self.r.network.status()
        conds = [C.RuntimeCondition(type="RuntimeReady", status=True),
                 C.RuntimeCondition(type="NetworkReady", status=net_ok, reason="" if net_ok else "NetworkPluginNotReady",
                                    message=net_msg)]
        return C.StatusResponse(status=C.RuntimeStatus(conditions=conds),
                                info={"isolation": self.r.isolation, "handlers": ",".join(sorted(HANDLERS)),
                                      "cgroupDriver": self.r.cgroup_driver} if req.verbose else {})

    def _mark(self, ctx, sid):
        ctx.set_trailing_metadata(((EVENT_TRAILER, self.r.event_mark(sid)),))

    async def RunPodSandbox(self, req, ctx):
        try:
            sid = await self.r.run_sandbox(req.config)
        except Exception as e:
            await _abort(ctx, e)
        self._mark(ctx, sid)
        return C.RunPodSandboxResponse(pod_sandbox_id=sid)

    async def StopPodSandbox(self, req, ctx):
        await self.r.stop_sandbox(req.pod_sandbox_id)
        self._mark(ctx, req.pod_sandbox_id)
        return C.StopPodSandboxResponse()

    async def RemovePodSandbox(self, req, ctx):
        await self.r.remove_sandbox(req.pod_sandbox_id)
        self._mark(ctx, req.pod_sandbox_id)
        return C.RemovePodSandboxResponse()

    def _sb_meta(self, s):
        return sandbox_meta(s)

    async def PodSandboxStatus(self, req, ctx):
        s = self.r.sandboxes.get(req.pod_sandbox_id)
        if s is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"sandbox {req.pod_sandbox_id} not found")
        if s.state == C.SANDBOX_READY and not _alive(s.pid):
            s.state = C.SANDBOX_NOTREADY
        st = sandbox_status_msg(s, self.r.network.node_ip)
        return C.PodSandboxStatusResponse(status=st, info={"pid": str(s.pid)} if req.verbose else {})

    async def ListPodSandbox(self, req, ctx):
        f = req.filter if req.HasField("filter") else None
        out = []
        for s in self.r.sandboxes.values():
            if f is not None:
                if f.id and f.id != s.id:
                    continue
                if f.HasField("state") and f.state.state != s.state:
                    continue
                if any(s.labels.get(k) != v for k, v in f.label_selector.items()):
                    continue
            out.append(C.PodSandbox(id=s.id, metadata=self._sb_meta(s), state=s.state, created_at=s.created_at,
                                    labels=s.labels, annotations=s.annotations))
        return C.ListPodSandboxResponse(items=out)

    async def CreateContainer(self, req, ctx):
        try:
            cid = await self.r.create_container(req.pod_sandbox_id, req.config, req.sandbox_config)
        except Exception as e:
            await _abort(ctx, e)
        self._mark(ctx, req.pod_sandbox_id)
        return C.CreateContainerResponse(container_id=cid)

    def _sid_of(self, cid):
        c = self.r.containers.get(cid)
        return c.sandbox_id if c is not None else None

    async def StartContainer(self, req, ctx):
        sid = self._sid_of(req.container_id)
        try:
            await self.r.start_container(req.container_id)
        except Exception as e:
            await _abort(ctx, e)
        self._mark(ctx, sid)
        return C.StartContainerResponse()

    async def StopContainer(self, req, ctx):
        sid = self._sid_of(req.container_id)
        await self.r.stop_container(req.container_id, req.timeout)
        self._mark(ctx, sid)
        return C.StopContainerResponse()

    async def UpdateContainerResources(self, req, ctx):
        try:
            self.r.update_resources(req.container_id, req.linux)
        except Exception as e:
            await _abort(ctx, e)
        return C.UpdateContainerResourcesResponse()

    async def RemoveContainer(self, req, ctx):
        sid = self._sid_of(req.container_id)
        await self.r.remove_container(req.container_id)
        self._mark(ctx, sid)
        return C.RemoveContainerResponse()

    def _c(self, c):
        return C.Container(id=c.id, pod_sandbox_id=c.sandbox_id, metadata=C.ContainerMetadata(name=c.name, attempt=c.attempt),
                           image=C.ImageSpec(image=c.image), image_ref=c.image_ref, state=c.state, created_at=c.created_at,
                           labels=c.labels, annotations=c.annotations)

    async def ListContainers(self, req, ctx):
        f = req.filter if req.HasField("filter") else None
        out = []
        for c in self.r.containers.values():
            if f is not None:
                if f.id and f.id != c.id:
                    continue
                if f.pod_sandbox_id and f.pod_sandbox_id != c.sandbox_id:
                    continue
                if f.HasField("state") and f.state.state != c.state:
                    continue
                if any(c.labels.get(k) != v for k, v in f.label_selector.items()):
                    continue
            out.append(self._c(c))
        return C.ListContainersResponse(containers=out)

    async def ContainerStatus(self, req, ctx):
        c = self.r.containers.get(req.container_id)
        if c is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} not found")
        st = container_status_msg(c)
        info = {"pid": str(c.pid), "handler": c.handler, "devices": json.dumps(c.devices)} if req.verbose else {}
        return C.ContainerStatusResponse(status=st, info=info)

    async def Exec(self, req, ctx):
        c = self.r.containers.get(req.container_id)
        if c is None or c.state != C.CONTAINER_RUNNING:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} is not running")
        if not req.cmd:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "cmd is required")
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

    def _stats(self, c, pgmap=None):
        """cAdvisor-equivalent container stats: the container's cgroup-v2 leaf when it has one
        (namespaces isolation), else its process group; the writable layer is the container's
        root directory (du, cached)."""
        from ..monitoring.cadvisor import cgroup_stats, process_stats
        st = None
        if c.state == C.CONTAINER_RUNNING:
            if self.r.isolation == "namespaces":
                st = cgroup_stats(self.r._cgroup_of(c))
            if st is None:
                st = process_stats((pgmap or {}).get(c.pid) or [c.pid])
        st = st or {}
        ts = now_ns()
        u = lambda k: C.UInt64Value(value=int(st.get(k, 0)))    # noqa: E731
        root = os.path.join(self.r.state_dir, "rootfs", c.sandbox_id, c.name)
        used, inodes = self.r.du.get(root) if os.path.isdir(root) else (0, 0)
        return C.ContainerStats(
            attributes=C.ContainerAttributes(id=c.id, metadata=C.ContainerMetadata(name=c.name, attempt=c.attempt),
                                             labels=c.labels, annotations=c.annotations),
            cpu=C.CpuUsage(timestamp=ts, usage_core_nano_seconds=u("cpu_ns")),
            memory=C.MemoryUsage(timestamp=ts, working_set_bytes=u("working_set_bytes"), usage_bytes=u("usage_bytes"),
                                 rss_bytes=u("rss_bytes"), page_faults=u("page_faults"), major_page_faults=u("major_page_faults")),
            writable_layer=C.FilesystemUsage(timestamp=ts, storage_id=C.StorageIdentifier(uuid=root),
                                             used_bytes=C.UInt64Value(value=used), inodes_used=C.UInt64Value(value=inodes)))

    async def ContainerStats(self, req, ctx):
        c = self.r.containers.get(req.container_id)
        if c is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "not found")
        pgmap = await asyncio.to_thread(_pgid_map) if self.r.isolation != "namespaces" else None
        return C.ContainerStatsResponse(stats=await asyncio.to_thread(self._stats, c, pgmap))

    async def ListContainerStats(self, req, ctx):
        f = req.filter if req.HasField("filter") else None
        sel = [c for c in self.r.containers.values()
               if c.state == C.CONTAINER_RUNNING and (f is None or ((not f.id or f.id == c.id) and
                                                                    (not f.pod_sandbox_id or f.pod_sandbox_id == c.sandbox_id)))]

        def collect():    # /proc and cgroup reads block: one pass off the event loop
            pgmap = _pgid_map() if self.r.isolation != "namespaces" else None
            return [self._stats(c, pgmap) for c in sel]
        return C.ListContainerStatsResponse(stats=await asyncio.to_thread(collect) if sel else [])

    async def UpdateRuntimeConfig(self, req, ctx):
        cidr = req.runtime_config.network_config.pod_cidr
        if cidr:
            self.r.network.set_pod_cidr(cidr)
        return C.UpdateRuntimeConfigResponse()

    async def GetContainerEvents(self, req, ctx):
        q: asyncio.Queue = asyncio.Queue()
        self.r._event_streams.add(q)
        try:
            while True:
                yield await q.get()
        finally:
            self.r._event_streams.discard(q)


class _Images:
    def __init__(self, r: RocShim):
        self.r = r

    def _img(self, name, iid):
        return C.Image(id=iid, repo_tags=[name], size=self.r.images.size(name))

    async def ListImages(self, req, ctx):
        return C.ListImagesResponse(images=[self._img(n, i) for n, i, _ in self.r.images.list()])

    async def ImageStatus(self, req, ctx):
        res = self.r.images.resolve(req.image.image)
        if res is None:
            return C.ImageStatusResponse()
        return C.ImageStatusResponse(image=self._img(res[0], self.r.images.image_id(res[0])))

    async def PullImage(self, req, ctx):
        auth = None
        if req.HasField("auth"):
            auth = {"username": req.auth.username, "password": req.auth.password, "auth": req.auth.auth}
        try:
            ref = await asyncio.to_thread(self.r.images.pull, req.image.image, auth)
            return C.PullImageResponse(image_ref=ref)
        except PermissionError as e:
            await ctx.abort(grpc.StatusCode.UNAUTHENTICATED, str(e))
        except KeyError as e:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, str(e))
        except ValueError as e:            # oci.ImageFormatError: a bad manifest, a blob failing its digest
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, f"pulling {req.image.image}: {e}")
        except Exception as e:             # registry.RegistryError: transport / protocol
            await ctx.abort(grpc.StatusCode.UNAVAILABLE, f"pulling {req.image.image}: {e}")

    async def RemoveImage(self, req, ctx):
        ref = req.image.image
        name = next((n for n, i, _ in self.r.images.list() if i == ref), None) if ref.startswith("sha256:") else \
            (self.r.images.resolve(ref) or (None,))[0]
        if name is not None and not self.r.images.removable(name):
            await ctx.abort(grpc.StatusCode.FAILED_PRECONDITION, f"image {name} is preloaded and cannot be removed")
        if name is not None and any(c.image_ref == self.r.images.image_id(name) for c in self.r.containers.values()):
            await ctx.abort(grpc.StatusCode.FAILED_PRECONDITION, f"image {name} is in use by a container")
        self.r.images.remove(ref)
        return C.RemoveImageResponse()

    async def ImageFsInfo(self, req, ctx):
        """The image filesystem: bytes held by pulled images; storage_id names the directory
        (the kubelet statvfs()es it for capacity, as cAdvisor does for the runtime's root)."""
        root = self.r.images.blob_root
        used = await asyncio.to_thread(self.r.images.used_bytes)
        n = sum(1 for _ in os.scandir(root))
        return C.ImageFsInfoResponse(image_filesystems=[C.FilesystemUsage(
            timestamp=now_ns(), storage_id=C.StorageIdentifier(uuid=os.path.abspath(root)), used_bytes=C.UInt64Value(value=used),
            inodes_used=C.UInt64Value(value=n))])
