"""kuberuntime: pod lifecycle against a CRI runtime.

Reference pkg/kubelet/kuberuntime: SyncPod (kuberuntime_manager.go:568) driven by
computePodActions (:441) — create a sandbox when none is ready (killing stragglers), run
init containers one at a time, start/restart app containers per restartPolicy with
CrashLoopBackOff, kill containers whose spec hash changed; createPodSandbox +
generatePodSandboxConfig (kuberuntime_sandbox.go:35,62) whose annotations carry the device
plugins' AdmitPod annotations (:93, fork); startContainer + generateContainerConfig
(kuberuntime_container.go:88,180-231) whose devices/envs/mounts/annotations come from the
DeviceManager's merged InitContainer responses (makeDevices :277, labels.go:108-114).
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import os
import shutil
import time

import grpc

from ..security.apparmor import profile_name as apparmor_profile_name
from ..utils.flowcontrol import Backoff
from ..utils.trace import POD_TRACE
from .sysctl import pod_sysctls
from .qos import cgroup_parent
from ..grpcdesc.cri import CRI as C
from .cri_client import CRIClient

log = logging.getLogger("amdkube.kuberuntime")

L_POD_NAME, L_POD_NS, L_POD_UID = "io.kubernetes.pod.name", "io.kubernetes.pod.namespace", "io.kubernetes.pod.uid"
L_CONTAINER = "io.kubernetes.container.name"
A_HASH, A_RESTARTS, A_INIT = "io.kubernetes.container.hash", "io.kubernetes.container.restartCount", "io.amdkube.container.init"
A_TERM_PATH = "io.kubernetes.container.terminationMessagePath"       # labels.go
A_TERM_POLICY = "io.kubernetes.container.terminationMessagePolicy"

BACKOFF_BASE, BACKOFF_MAX = 10.0, 300.0


SECCOMP_POD_ANN = "seccomp.security.alpha.kubernetes.io/pod"
SECCOMP_CONTAINER_ANN = "container.seccomp.security.alpha.kubernetes.io/"


def seccomp_profile(pod: dict, container: str, root: str = "/var/lib/kubelet/seccomp") -> str:
    """kuberuntime_sandbox.go getSeccompProfileFromAnnotations: the container annotation wins
    over the pod one; docker/default means runtime/default; localhost/<p> is relative to
    --seccomp-profile-root; unconfined (or nothing) means no filter."""
    ann = (pod.get("metadata") or {}).get("annotations") or {}
    p = ann.get(SECCOMP_CONTAINER_ANN + container) or ann.get(SECCOMP_POD_ANN) or ""
    if p in ("", "unconfined"):
        return ""
    if p in ("docker/default", "runtime/default"):
        return "runtime/default"
    if p.startswith("localhost/"):
        rel = p[len("localhost/"):]
        return "localhost/" + (rel if os.path.isabs(rel) else os.path.join(root, rel))
    return p


def container_hash(c: dict) -> str:
    return hashlib.sha1(json.dumps(c, sort_keys=True).encode()).hexdigest()[:16]



def _container_files(hosts, tm_host: str):
    from .podcontext import atomic_write
    if hosts is not None:
        atomic_write(hosts[0], hosts[1], 0o644)
    os.makedirs(os.path.dirname(tm_host), exist_ok=True)
    open(tm_host, "w").close()

class ContainerRuntimeStatus:
    __slots__ = ("id", "name", "state", "exit_code", "reason", "message", "created_at", "started_at", "finished_at",
                 "restart_count", "hash", "image", "image_ref", "init", "log_path", "sandbox_id")

    @classmethod
    def from_cri(cls, st, ann, sandbox_id: str = ""):
        s = cls()
        s.sandbox_id = sandbox_id
        s.id, s.name, s.state = st.id, st.metadata.name, st.state
        s.exit_code, s.reason, s.message = st.exit_code, st.reason, st.message
        s.created_at, s.started_at, s.finished_at = st.created_at, st.started_at, st.finished_at
        s.restart_count = int(ann.get(A_RESTARTS, "0") or 0)
        s.hash = ann.get(A_HASH, "")
        s.init = ann.get(A_INIT) == "true"
        s.image, s.image_ref, s.log_path = st.image.image, st.image_ref, st.log_path
        return s


class PodRuntimeStatus:
    def __init__(self, uid):
        self.uid = uid
        self.sandboxes = []  # newest first: (id, state, attempt, created_at)
        self.ip = None      # the ready sandbox's pod IP (network plugin / CNI result); None = not known
        self.containers: dict[str, list[ContainerRuntimeStatus]] = {}  # name -> newest first

    def ready_sandbox(self):
        for s in self.sandboxes:
            if s[1] == C.SANDBOX_READY:
                return s
        return None

    def latest(self, name) -> ContainerRuntimeStatus | None:
        lst = self.containers.get(name)
        return lst[0] if lst else None

    def running(self):
        return [c for lst in self.containers.values() for c in lst if c.state == C.CONTAINER_RUNNING]

    def container_state(self, cid: str):
        for lst in self.containers.values():
            for c in lst:
                if c.id == cid:
                    return c.state
        return None


class SandboxRef:
    """(id, state) of a sandbox, enough for kill_pod/remove_pod without a ListPodSandbox."""
    __slots__ = ("id", "state")

    def __init__(self, sid, state):
        self.id, self.state = sid, state


def apply_event(rt: PodRuntimeStatus, ev, sandbox_ips: dict) -> PodRuntimeStatus:
    """A new PodRuntimeStatus = rt with one sandbox (and all its containers) replaced by the
    full state an evented-PLEG event carries (KEP-3386 ContainerEventResponse). rt itself is
    never mutated: a pod sync may still hold it."""
    sst = ev.pod_sandbox_status
    sid = sst.id
    gone = ev.container_event_type == C.CONTAINER_DELETED_EVENT and ev.container_id == sid
    new = PodRuntimeStatus(rt.uid)
    sbs = [x for x in rt.sandboxes if x[0] != sid]
    if not gone:
        sbs.append((sid, sst.state, sst.metadata.attempt, sst.created_at))
    new.sandboxes = sorted(sbs, key=lambda x: x[3], reverse=True)
    for name, lst in rt.containers.items():
        keep = [c for c in lst if c.sandbox_id != sid]
        if keep:
            new.containers[name] = keep
    if not gone:
        for cs in ev.containers_statuses:
            new.containers.setdefault(cs.metadata.name, []).append(ContainerRuntimeStatus.from_cri(cs, dict(cs.annotations), sid))
    for lst in new.containers.values():
        lst.sort(key=lambda x: x.created_at, reverse=True)
    if not gone and sst.state == C.SANDBOX_READY and sst.network.ip:
        sandbox_ips.setdefault(sid, sst.network.ip)
    ready = new.ready_sandbox()
    new.ip = sandbox_ips.get(ready[0]) if ready is not None else ""
    return new


def _go_duration(sec: float) -> str:
    """time.Duration.String() for whole seconds: 10s, 1m20s, 5m0s."""
    s = int(round(sec))
    if s < 60:
        return f"{s}s"
    h, rem = divmod(s, 3600)
    mnt, s = divmod(rem, 60)
    return (f"{h}h" if h else "") + f"{mnt}m{s}s"


def stable_key(pod: dict, c: dict) -> str:
    """kuberuntime_manager.go getStableKey: the back-off key of one container spec of one pod
    (a spec change starts a fresh back-off)."""
    md = pod["metadata"]
    return f"{md['name']}_{md.get('namespace', '')}_{md['uid']}_{c['name']}_{container_hash(c)}"


class PodActions:
    """kuberuntime_manager.go podActions (:356-379)."""
    __slots__ = ("kill_pod", "create_sandbox", "sandbox_id", "attempt", "next_init", "to_start", "to_kill")

    def __init__(self, kill_pod=False, create_sandbox=False, sandbox_id="", attempt=0, next_init=None,
                 to_start=None, to_kill=None):
        self.kill_pod, self.create_sandbox, self.sandbox_id, self.attempt = kill_pod, create_sandbox, sandbox_id, attempt
        self.next_init = next_init                  # the init container (spec dict) to start next
        self.to_start: list[int] = to_start if to_start is not None else []   # indexes into spec.containers
        self.to_kill: dict[str, tuple] = to_kill if to_kill is not None else {}   # cid -> (name, spec, message)

    def key(self, with_messages: bool = False):
        kill = {cid: (v[0], v[1]["name"] if v[1] else None) + ((v[2],) if with_messages else ())
                for cid, v in self.to_kill.items()}
        return (self.kill_pod, self.create_sandbox, self.sandbox_id, self.attempt,
                self.next_init["name"] if self.next_init else None, list(self.to_start), kill)

    def __eq__(self, other):
        return isinstance(other, PodActions) and self.key() == other.key()

    def __repr__(self):
        return "PodActions(kill_pod=%r, create_sandbox=%r, sandbox_id=%r, attempt=%r, next_init=%r, to_start=%r, to_kill=%r)" % self.key(True)


def should_restart_on_failure(pod: dict) -> bool:
    return ((pod.get("spec") or {}).get("restartPolicy") or "Always") != "Never"


def _failed(cs) -> bool:
    return cs.state == C.CONTAINER_EXITED and cs.exit_code != 0


def should_container_be_restarted(c: dict, pod: dict, st: PodRuntimeStatus) -> bool:
    """kubelet/container/helpers.go ShouldContainerBeRestarted (:65-94)."""
    cs = st.latest(c["name"])
    if cs is None:
        return True
    if cs.state == C.CONTAINER_RUNNING:
        return False
    if cs.state in (C.CONTAINER_UNKNOWN, C.CONTAINER_CREATED):
        return True
    policy = (pod.get("spec") or {}).get("restartPolicy") or "Always"
    if policy == "Never":
        return False
    if policy == "OnFailure" and cs.exit_code == 0:
        return False
    return True


def find_next_init_container(pod: dict, st: PodRuntimeStatus):
    """kuberuntime_container.go findNextInitContainerToRun (:720-759): (status of the last
    failed init container, next init container to run, done)."""
    inits = (pod.get("spec") or {}).get("initContainers") or []
    if not inits:
        return None, None, True
    for ic in reversed(inits):
        cs = st.latest(ic["name"])
        if cs is not None and _failed(cs):
            return cs, ic, False
    for i in range(len(inits) - 1, -1, -1):
        cs = st.latest(inits[i]["name"])
        if cs is None:
            continue
        if cs.state == C.CONTAINER_RUNNING:
            return None, None, False
        if cs.state == C.CONTAINER_EXITED:
            if i == len(inits) - 1:
                return None, None, True
            return None, inits[i + 1], False
    return None, inits[0], False


def pod_sandbox_changed(pod: dict, st: PodRuntimeStatus):
    """kuberuntime_manager.go podSandboxChanged (:383-421): (create, attempt, sandbox id).
    A newest sandbox that is not ready, more than one ready sandbox, or a non-host-network
    sandbox without an IP means a new sandbox."""
    if not st.sandboxes:
        return True, 0, ""
    sid, state, attempt = st.sandboxes[0][0], st.sandboxes[0][1], st.sandboxes[0][2]
    if sum(1 for s in st.sandboxes if s[1] == C.SANDBOX_READY) > 1:
        return True, attempt + 1, sid
    if state != C.SANDBOX_READY:
        return True, attempt + 1, sid
    if not (pod.get("spec") or {}).get("hostNetwork") and st.ip == "":
        return True, attempt + 1, sid
    return False, attempt, sid


def compute_pod_actions(pod: dict, st: PodRuntimeStatus, liveness_failed=None) -> PodActions:
    """kuberuntime_manager.go computePodActions (:441-558).

    * a changed sandbox kills and recreates the pod (init containers from the first; under
      OnFailure the succeeded containers stay done) — unless the policy is Never and the pod
      already ran once, then it is only killed;
    * init containers run one at a time; a failed one under Never kills the pod;
    * a dead container is started when ShouldContainerBeRestarted says so;
    * a running container whose spec hash changed is killed and always recreated; one that
      failed its liveness probe is killed and recreated only when restartPolicy != Never;
    * with nothing left running and nothing to start, the pod is killed.

    `liveness_failed`: container ids (or a predicate over them) whose liveness is Failure."""
    is_failed = (liveness_failed if callable(liveness_failed)
                 else (lambda cid, s=liveness_failed or (): cid in s))
    spec = pod.get("spec") or {}
    create, attempt, sid = pod_sandbox_changed(pod, st)
    acts = PodActions(kill_pod=create, create_sandbox=create, sandbox_id=sid, attempt=attempt)
    conts = spec.get("containers") or []
    if create:
        if not should_restart_on_failure(pod) and attempt != 0:
            # a Never pod that already ran is not restarted; the reference returns with
            # CreateSandbox still set and relies on syncPod never reaching here for a finished
            # pod — amdkube does not recreate a sandbox it will not use (later upstream fix)
            acts.create_sandbox = False
            return acts
        inits = spec.get("initContainers") or []
        if inits:
            acts.next_init = inits[0]
            return acts
        onfail = spec.get("restartPolicy") == "OnFailure"
        for i, c in enumerate(conts):
            cs = st.latest(c["name"])
            if onfail and cs is not None and cs.state != C.CONTAINER_RUNNING and cs.exit_code == 0:
                continue
            acts.to_start.append(i)
        return acts
    last, nxt, done = find_next_init_container(pod, st)
    if not done:
        if nxt is not None:
            if last is not None and _failed(last) and not should_restart_on_failure(pod):
                acts.kill_pod = True
            else:
                acts.next_init = nxt
        return acts
    keep = 0
    for i, c in enumerate(conts):
        cs = st.latest(c["name"])
        if cs is None or cs.state != C.CONTAINER_RUNNING:
            if should_container_be_restarted(c, pod, st):
                acts.to_start.append(i)
            continue
        restart = should_restart_on_failure(pod)
        if cs.hash and cs.hash != container_hash(c):
            reason = f"Container spec hash changed ({cs.hash} vs {container_hash(c)})."
            restart = True
        elif is_failed(cs.id):
            reason = "Container failed liveness probe."
        else:
            keep += 1
            continue
        message = reason
        if restart:
            message = f"{message}. Container will be killed and recreated."
            acts.to_start.append(i)
        acts.to_kill[cs.id] = (cs.name, c, message)
    if keep == 0 and not acts.to_start:
        acts.kill_pod = True
    return acts


IMAGE_BACKOFF_BASE, IMAGE_BACKOFF_MAX = 10.0, 300.0


class StartError(RuntimeError):
    """A container start failure with its kubelet waiting reason (kubecontainer errors:
    ErrImagePull, ImagePullBackOff, ErrImageNeverPull, CreateContainerConfigError,
    CreateContainerError, RunContainerError, PostStartHookError)."""

    def __init__(self, reason: str, message: str):
        super().__init__(f"{reason}: {message}")
        self.reason, self.message = reason, message


def start_error_reason(e: BaseException) -> tuple[str, str]:
    if isinstance(e, StartError):
        return e.reason, e.message
    if isinstance(e, grpc.RpcError):
        return "RunContainerError", e.details() or str(e.code())
    return "CreateContainerConfigError", str(e)


class RuntimeManager:
    cgroup_driver = "cgroupfs"      # --cgroup-driver
    legacy_logs_dir = ""            # /var/log/containers symlinks (cluster logging); "" = none

    def __init__(self, cri: CRIClient, device_manager, root_dir: str, recorder=None, image_pull_qps: float = 0,
                 image_pull_burst: int = 10, serialize_image_pulls: bool = True):
        self.cri = cri
        # images/image_manager.go: --serialize-image-pulls (one pull at a time) and
        # --registry-qps/--registry-burst (a token bucket in front of the puller)
        from ..client.rest import TokenBucket
        self._pull_sem = asyncio.Semaphore(1) if serialize_image_pulls else None
        self._pull_limiter = TokenBucket(image_pull_qps, image_pull_burst or 1) if image_pull_qps else None
        self.cpu_cfs_quota = True   # --cpu-cfs-quota
        self.dm = device_manager
        self.root = root_dir
        self.recorder = recorder
        # kubelet.go:859 the container restart back-off (10 s doubling to 300 s), keyed by
        # stable_key; (uid, name) -> (key, event time) of a start it is holding back
        self.backoff = Backoff(BACKOFF_BASE, BACKOFF_MAX)
        self._backoff_due: dict[tuple[str, str], tuple[str, float]] = {}
        self.sandbox_ips: dict[str, str] = {}   # sandbox id -> IP (PodSandboxStatus is asked once per sandbox)
        self.seccomp_root = os.path.join(root_dir, "seccomp")   # --seccomp-profile-root
        self._image_seen: dict[str, float] = {}
        # reason_cache.go: the last start failure per (pod uid, container) → (reason, message),
        # shown as the waiting state of a container that has not been created
        self.reasons: dict[str, dict[str, tuple[str, str]]] = {}
        # images/puller.go: pull back-off per (pod uid, image) (10 s doubling to 300 s) → ImagePullBackOff
        self.pull_backoff: dict[tuple[str, str], tuple[float, float]] = {}
        self.legacy = None          # gpu_legacy.AMDGPUManager when the Accelerators gate is on
        self.cpu_manager = None     # cpumanager.CPUManager
        self.node_ip = "127.0.0.1"
        self.cluster_domain = ""
        self.gpu_numa = None        # (pod, container) -> NUMA nodes of its GPUs
        self.dns = None             # dns.DNSConfigurer (pod resolv.conf)
        self.memory_capacity = 1 << 40   # node memory (burstable OOM score scaling), set by the kubelet
        self.active_pods = None

    # ----------------------------------------------------------------- status
    async def pod_status(self, uid: str, sandboxes=None) -> PodRuntimeStatus:
        st = PodRuntimeStatus(uid)
        sbs = sandboxes if sandboxes is not None else await self.cri.list_pod_sandbox(uid)
        sbs = sorted(sbs, key=lambda s: s.created_at, reverse=True)
        st.sandboxes = [(s.id, s.state, s.metadata.attempt, s.created_at) for s in sbs]
        ready = st.ready_sandbox()
        if ready is not None:
            ip = self.sandbox_ips.get(ready[0])
            if ip is None:
                try:
                    ip = (await self.cri.pod_sandbox_status(ready[0])).network.ip
                except grpc.RpcError:
                    ip = None       # unknown: not a reason to recreate the sandbox
                if ip:
                    self.sandbox_ips[ready[0]] = ip
            st.ip = ip
        if len(self.cri._cid_sid) > 100000:
            self.cri._cid_sid.clear()
        for s in sbs:
            for c in await self.cri.list_containers(s.id):
                self.cri._cid_sid[c.id] = s.id
                try:
                    cs, _ = await self.cri.container_status(c.id)
                except grpc.RpcError:
                    continue
                st.containers.setdefault(c.metadata.name, []).append(ContainerRuntimeStatus.from_cri(cs, dict(c.annotations), s.id))
        for lst in st.containers.values():
            lst.sort(key=lambda x: x.created_at, reverse=True)
        return st

    # ---------------------------------------------------------------- sandbox
    def sandbox_config(self, pod: dict, attempt: int, annotations: dict) -> "C.PodSandboxConfig":
        md, spec = pod["metadata"], pod.get("spec") or {}
        log_dir = os.path.join(self.root, "pods", md["uid"], "logs")
        made = self.__dict__.setdefault("_made_dirs", set())
        if log_dir not in made:            # the config is rebuilt on every sync; the directory once
            os.makedirs(log_dir, exist_ok=True)
            made.add(log_dir)
            if len(made) > 4096:
                made.clear()
        ports = [C.PortMapping(container_port=p.get("containerPort", 0), host_port=p.get("hostPort", 0),
                               protocol=C.UDP if p.get("protocol") == "UDP" else C.TCP)
                 for c in spec.get("containers") or [] for p in c.get("ports") or []]
        ann = dict(md.get("annotations") or {})
        ann.update(annotations or {})
        return C.PodSandboxConfig(
            metadata=C.PodSandboxMetadata(name=md["name"], uid=md["uid"], namespace=md.get("namespace", ""), attempt=attempt),
            hostname=spec.get("hostname") or md["name"], log_directory=log_dir, port_mappings=ports,
            labels={**(md.get("labels") or {}), L_POD_NAME: md["name"], L_POD_NS: md.get("namespace", ""), L_POD_UID: md["uid"]},
            annotations=ann, dns_config=self.dns.cri_config(pod) if self.dns is not None else None,
            linux=C.LinuxPodSandboxConfig(cgroup_parent=cgroup_parent(pod, self.cgroup_driver), sysctls=pod_sysctls(pod),
                                          security_context=C.LinuxSandboxSecurityContext(
                namespace_options=C.NamespaceOption(host_network=bool(spec.get("hostNetwork")), host_pid=bool(spec.get("hostPID")),
                                                    host_ipc=bool(spec.get("hostIPC"))))))

    # -------------------------------------------------------------- containers
    async def _pull(self, image: str, keyring):
        """kuberuntime_image.go PullImage: every matching credential in order, first success
        wins; anonymous when none matches."""
        creds = keyring.lookup(image) if keyring is not None else []
        if not creds:
            await self.cri.pull_image(image)
            return
        err = None
        for a in creds:
            try:
                await self.cri.pull_image(image, a.to_cri(C))
                return
            except grpc.RpcError as e:
                err = e
        raise err

    async def ensure_image(self, c: dict, keyring=None, uid: str = ""):
        image = c["image"]
        bkey = (uid, image)        # puller.go: back-off per pod and image
        policy = c.get("imagePullPolicy", "IfNotPresent")
        if policy != "Always" and self._image_seen.get(image, 0.0) > time.monotonic():
            return   # present a moment ago (image GC runs on minutes, not per pod)
        present = await self.cri.image_status(image)
        if present is not None:
            self._image_seen[image] = time.monotonic() + 30.0
        if policy == "Never" and present is None:
            raise StartError("ErrImageNeverPull", f'Container image "{image}" is not present with pull policy of Never')
        if present is None or policy == "Always":
            # image_manager.go:121-141: a pull that fails is ErrImagePull (and backs off) even
            # when an older copy is present — Always means the registry must agree
            until, _ = self.pull_backoff.get(bkey, (0.0, 0.0))
            if time.monotonic() < until:
                raise StartError("ImagePullBackOff", f'Back-off pulling image "{image}"')
            try:
                if self._pull_limiter is not None:
                    await self._pull_limiter.wait()
                if self._pull_sem is not None:
                    async with self._pull_sem:
                        await self._pull(image, keyring)
                else:
                    await self._pull(image, keyring)
                self.pull_backoff.pop(bkey, None)
            except grpc.RpcError as e:
                _, last = self.pull_backoff.get(bkey, (0.0, 0.0))
                delay = min(IMAGE_BACKOFF_MAX, last * 2 if last else IMAGE_BACKOFF_BASE)
                self.pull_backoff[bkey] = (time.monotonic() + delay, delay)
                raise StartError("ErrImagePull", e.details() or str(e.code()))

    async def start_container(self, pod: dict, c: dict, sid: str, sandbox_cfg, ctx: dict, restart_count: int, init: bool):
        await self.ensure_image(c, ctx.get("keyring"), pod["metadata"]["uid"])
        POD_TRACE(pod["metadata"]["uid"], "image_ready")
        opts = await self.dm.init_container(pod, c)
        POD_TRACE(pod["metadata"]["uid"], "devices_ready")
        if self.legacy is not None:   # Accelerators gate: kubelet_pods.go:486-490 AllocateGPU
            la = self.legacy.allocate(pod, c, self.active_pods() if self.active_pods else [])
            if la["devices"]:
                opts = dict(opts, devices=list(opts["devices"]) + [d for d in la["devices"] if d not in opts["devices"]],
                            envs={**opts["envs"], **la["envs"]}, annotations={**opts["annotations"], **la["annotations"]})
        from .podcontext import POD_IP, expand, hosts_file, atomic_write
        pod_ip = self.sandbox_ips.get(sid) or self.node_ip
        cenv = {k: v.replace(POD_IP, pod_ip) for k, v in (ctx.get("env", {}).get(c["name"]) or {}).items()}
        envs = [C.KeyValue(key=k, value=v) for k, v in cenv.items()]
        envs += [C.KeyValue(key=k, value=v) for k, v in opts["envs"].items()]
        extra_mounts = []
        spec = pod.get("spec") or {}
        pdir = os.path.join(self.root, "pods", pod["metadata"]["uid"])
        hosts = None
        if not spec.get("hostNetwork"):
            # kubelet_pods.go makeHostsMount: the kubelet-managed /etc/hosts (pod IP, hostname, hostAliases)
            hp = os.path.join(pdir, "etc-hosts")
            hosts = (hp, hosts_file(pod, pod_ip, self.cluster_domain).encode())
            extra_mounts.append({"container_path": "/etc/hosts", "host_path": hp, "read_only": False})
        tm_path = c.get("terminationMessagePath") or "/dev/termination-log"
        tm_host = os.path.join(pdir, "containers", c["name"], f"{restart_count}-termination-log")
        _container_files(hosts, tm_host)
        extra_mounts.append({"container_path": tm_path, "host_path": tm_host, "read_only": False})
        mounts = [C.Mount(container_path=m["container_path"], host_path=m["host_path"], readonly=bool(m.get("read_only")))
                  for m in (ctx.get("mounts", {}).get(c["name"]) or []) + opts["mounts"] + extra_mounts]
        devices = [C.Device(container_path=d["container_path"], host_path=d["host_path"], permissions=d.get("permissions", "rw"))
                   for d in opts["devices"]]
        ann = dict(opts["annotations"])
        ann.update({A_HASH: container_hash(c), A_RESTARTS: str(restart_count), A_INIT: "true" if init else "false",
                    A_TERM_PATH: tm_path, A_TERM_POLICY: c.get("terminationMessagePolicy") or "File"})
        res = (c.get("resources") or {}).get("limits") or {}
        from ..api.quantity import Quantity
        from .qos import oom_score_adj
        lres = C.LinuxContainerResources(oom_score_adj=oom_score_adj(pod, c, self.memory_capacity))
        if "memory" in res:
            lres.memory_limit_in_bytes = Quantity(res["memory"]).value()
        if "cpu" in res and self.cpu_cfs_quota:
            lres.cpu_period = 100000
            lres.cpu_quota = max(1000, Quantity(res["cpu"]).milli_value() * 100)
        req_cpu = ((c.get("resources") or {}).get("requests") or {}).get("cpu") or res.get("cpu")
        lres.cpu_shares = max(2, Quantity(req_cpu).milli_value() * 1024 // 1000) if req_cpu else 2   # MilliCPUToShares
        if self.cpu_manager is not None and self.cpu_manager.policy != "none":
            # cpu_manager.go AddContainer: exclusive CPUs (near the container's GPUs) or the shared pool
            lres.cpuset_cpus = self.cpu_manager.allocate(pod, c, self.gpu_numa(pod, c) if self.gpu_numa else None)
        md = pod["metadata"]
        cfg = C.ContainerConfig(
            metadata=C.ContainerMetadata(name=c["name"], attempt=restart_count), image=C.ImageSpec(image=c["image"]),
            command=[expand(x, cenv) for x in c.get("command") or []], args=[expand(x, cenv) for x in c.get("args") or []],
            working_dir=c.get("workingDir") or "",
            envs=envs, mounts=mounts, devices=devices,
            labels={L_POD_NAME: md["name"], L_POD_NS: md.get("namespace", ""), L_POD_UID: md["uid"], L_CONTAINER: c["name"]},
            annotations=ann, log_path=f"{c['name']}/{restart_count}.log",
            linux=C.LinuxContainerConfig(resources=lres, security_context=C.LinuxContainerSecurityContext(
                seccomp_profile_path=seccomp_profile(pod, c["name"], self.seccomp_root),
                apparmor_profile=apparmor_profile_name(pod, c["name"]),     # security_context.go:40
                no_new_privs=not bool(((c.get("securityContext") or {}).get("allowPrivilegeEscalation", True))))))
        cid = await self.cri.create_container(sid, cfg, sandbox_cfg)
        POD_TRACE(pod["metadata"]["uid"], "container_created")
        await self.cri.start_container(cid)
        POD_TRACE(pod["metadata"]["uid"], "container_started")
        if self.legacy_logs_dir:
            self._legacy_log_link(md, c["name"], cid, os.path.join(sandbox_cfg.log_directory, cfg.log_path))
        post = ((c.get("lifecycle") or {}).get("postStart"))
        if post:
            # kuberuntime_container.go startContainer step 4: a failing postStart hook kills the container
            err = await self.run_handler(pod, c, cid, post, pod_ip)
            if err:
                if self.recorder:
                    self.recorder.event(pod, "Warning", "FailedPostStartHook", err)
                await self.cri.stop_container(cid, 0)
                raise StartError("PostStartHookError", str(err))
        return cid

    def legacy_log_symlink(self, pod_name: str, namespace: str, container: str, cid: str) -> str:
        """kuberuntime_container.go legacyLogSymlink / logSymlink: `<pod>_<ns>_<container>-<id>.log`,
        cut to ext4's 255-byte file name limit."""
        name = f"{pod_name}_{namespace}_{container}-{cid}"[:255 - len(".log")]
        return os.path.join(self.legacy_logs_dir, name + ".log")

    def _legacy_log_link(self, md: dict, container: str, cid: str, target: str):
        """startContainer: symlink the container's log into the legacy directory the cluster
        logging agent tails (a failure is logged, never fatal — as the reference)."""
        link = self.legacy_log_symlink(md["name"], md.get("namespace", ""), container, cid)
        try:
            os.makedirs(self.legacy_logs_dir, exist_ok=True)
            if os.path.lexists(link):
                os.unlink(link)
            os.symlink(target, link)
        except OSError as e:
            log.warning("failed to create legacy symbolic link %s to container %s log %s: %r", link, cid, target, e)

    def remove_legacy_log_links(self, cid: str | None = None) -> int:
        """The container's symlink (removeContainerLog), or — cid None — every dangling one
        (container_gc.go: dead symlinks left by containers removed elsewhere)."""
        if not self.legacy_logs_dir or not os.path.isdir(self.legacy_logs_dir):
            return 0
        n = 0
        for f in os.listdir(self.legacy_logs_dir):
            p = os.path.join(self.legacy_logs_dir, f)
            if not f.endswith(".log") or not os.path.islink(p):
                continue
            if (cid is not None and f.endswith(f"-{cid}.log")) or (cid is None and not os.path.exists(p)):
                try:
                    os.unlink(p)
                    n += 1
                except OSError:
                    pass
        return n

    async def run_handler(self, pod, c, cid, handler: dict, pod_ip: str, timeout: int = 30) -> str:
        """lifecycle/handlers.go HandlerRunner: exec in the container or HTTP GET; '' on success."""
        if "exec" in handler:
            try:
                _out, err, code = await self.cri.exec_sync(cid, handler["exec"].get("command") or [], timeout)
            except grpc.RpcError as e:
                return f"Exec lifecycle hook ({handler['exec'].get('command')}) for Container {c['name']!r} failed - error: {e.details()}"
            return "" if code == 0 else (f"Exec lifecycle hook ({handler['exec'].get('command')}) for Container {c['name']!r} "
                                         f"failed - error: command exited with {code}, message: {err[-256:]!r}")
        if "httpGet" in handler:
            h = handler["httpGet"]
            port = h.get("port")
            if isinstance(port, str) and not port.isdigit():
                port = next((p["containerPort"] for p in c.get("ports") or [] if p.get("name") == port), None)
            url = f"{(h.get('scheme') or 'HTTP').lower()}://{h.get('host') or pod_ip}:{port}{h.get('path') or '/'}"
            import aiohttp
            try:
                async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout)) as s:
                    async with s.get(url, headers={x["name"]: x["value"] for x in h.get("httpHeaders") or []}, ssl=False) as r:
                        if r.status >= 400:
                            return f"Http lifecycle hook ({url}) for Container {c['name']!r} failed - HTTP {r.status}"
            except Exception as e:
                return f"Http lifecycle hook ({url}) for Container {c['name']!r} failed - error: {e!r}"
            return ""
        return "a lifecycle handler needs exec or httpGet"

    # ------------------------------------------------------------------ sync
    async def sync_pod(self, pod: dict, st: PodRuntimeStatus, ctx: dict, liveness_failed=None) -> list[str]:
        """kuberuntime_manager.go SyncPod (:568-741): compute the actions, then (2) kill the
        pod when the sandbox changed or nothing is left to run, (3) kill the containers that
        must not keep running, (4) create the sandbox, (5) start the next init container,
        (6) start the containers to start — each start behind doBackOff. Returns pod-level
        error messages. `liveness_failed`: the container ids whose liveness result is Failure
        (the probe manager's results cache)."""
        errors: list[str] = []
        spec = pod.get("spec") or {}
        uid = pod["metadata"]["uid"]
        acts = compute_pod_actions(pod, st, liveness_failed)
        if acts.create_sandbox and acts.sandbox_id and self.recorder is not None:
            self.recorder.event(pod, "Normal", "SandboxChanged", "Pod sandbox changed, it will be killed and re-created.")
        if acts.kill_pod and not acts.create_sandbox:
            # nothing left to run: the pod is finished. Its containers are stopped here; the
            # sandbox goes with the kubelet's terminal-phase release right after the status
            # (which still reports the sandbox's IP) is generated
            for cs in st.running():
                c = next((x for x in spec.get("containers") or [] if x["name"] == cs.name), None)
                msg = acts.to_kill.get(cs.id, (None, None, ""))[2]
                try:
                    await self.kill_container(pod, cs.id, c, msg)
                except grpc.RpcError as e:
                    errors.append(f"kill {cs.name}: {e.details()}")
            return errors
        if acts.kill_pod:
            if st.sandboxes or st.running():
                grace = int(spec.get("terminationGracePeriodSeconds", 30))
                await self.kill_pod(uid, grace, pod, [SandboxRef(x[0], x[1]) for x in st.sandboxes], clear_backoff=False)
                for c in st.running():     # containers whose sandbox is already gone
                    if all(c.sandbox_id != x[0] or x[1] != C.SANDBOX_READY for x in st.sandboxes):
                        await self.cri.stop_container(c.id, 0)
            if acts.create_sandbox:
                await self._purge_init_containers(pod, st)
        else:
            for cid, (name, c, message) in acts.to_kill.items():
                try:
                    await self.kill_container(pod, cid, c, message)
                except grpc.RpcError as e:
                    errors.append(f"kill {name}: {e.details()}")
                    return errors
        if not acts.create_sandbox and acts.next_init is None and not acts.to_start:
            return errors
        sid = acts.sandbox_id
        if acts.create_sandbox:
            sandbox_cfg = self.sandbox_config(pod, acts.attempt, self.dm.pod_resources(pod))
            POD_TRACE(uid, "sandbox_start")
            try:
                sid = await self.cri.run_pod_sandbox(sandbox_cfg)
            except grpc.RpcError as e:
                # createPodSandbox failed: FailedCreatePodSandBox event; the pod stays Pending and
                # the next sync retries
                msg = f"Failed create pod sandbox: {e.details() if hasattr(e, 'details') else e}"
                if self.recorder is not None:
                    self.recorder.event(pod, "Warning", "FailedCreatePodSandBox", msg)
                errors.append(msg)
                return errors
            POD_TRACE(uid, "sandbox_ready")
        else:
            sandbox_cfg = self.sandbox_config(pod, acts.attempt, self.dm.pod_resources(pod))
        conts = spec.get("containers") or []
        targets = ([(acts.next_init, True)] if acts.next_init is not None else []) + [(conts[i], False) for i in acts.to_start]
        for c, init in targets:
            if self.do_backoff(pod, c, st):
                if init:
                    return errors
                continue
            # startContainer: the attempt carries over from the newest instance of this container
            cur = st.latest(c["name"])
            rc = (cur.restart_count + 1) if cur is not None else 0
            try:
                await self.start_container(pod, c, sid, sandbox_cfg, ctx, rc, init)
                self._clear_reason(uid, c["name"])
            except grpc.RpcError as e:
                self.reasons.setdefault(uid, {})[c["name"]] = start_error_reason(e)
                errors.append(f"{'init container' if init else 'container'} {c['name']}: {e.details()}")
            except Exception as e:
                self.reasons.setdefault(uid, {})[c["name"]] = start_error_reason(e)
                errors.append(f"{'init container' if init else 'container'} {c['name']}: {e}")
            if init:
                break
        return errors

    async def _purge_init_containers(self, pod: dict, st: PodRuntimeStatus):
        """kuberuntime_container.go purgeInitContainers: a new sandbox runs its init containers
        again from the first, so the old instances must not count as done."""
        names = {ic["name"] for ic in (pod.get("spec") or {}).get("initContainers") or []}
        for n in names:
            for cs in st.containers.get(n) or []:
                if cs.state != C.CONTAINER_RUNNING:
                    try:
                        await self.cri.remove_container(cs.id)
                    except grpc.RpcError as e:
                        log.debug("purge init container %s: %s", cs.id, e.details())

    async def kill_container(self, pod: dict, cid: str, c: dict | None, reason: str = "", grace: int | None = None):
        """kuberuntime_container.go killContainer: preStop hook bounded by the grace period,
        then StopContainer, with a Killing event naming the reason."""
        spec = pod.get("spec") or {}
        if grace is None:
            grace = int(spec.get("terminationGracePeriodSeconds", 30))
        if self.recorder is not None:
            msg = f"Killing container with id rocshim://{cid}" + (f":{reason}" if reason else "")
            self.recorder.event(pod, "Normal", "Killing", msg)
        pre = ((c or {}).get("lifecycle") or {}).get("preStop")
        if pre:
            ip = self.sandbox_ips.get(self.cri._cid_sid.get(cid, "")) or self.node_ip
            err = await self.run_handler(pod, c, cid, pre, ip, min(grace, 30) or 1)
            if err and self.recorder:
                self.recorder.event(pod, "Warning", "FailedPreStopHook", err)
        await self.cri.stop_container(cid, grace)

    def _clear_reason(self, uid: str, name: str):
        r = self.reasons.get(uid)
        if r and r.pop(name, None) is not None and not r:
            del self.reasons[uid]

    def do_backoff(self, pod: dict, c: dict, st: PodRuntimeStatus) -> bool:
        """kuberuntime_manager.go doBackOff (:745-774): with the finish time of the newest
        exited instance as the event time, a container still inside its back-off is not
        started (BackOff event, CrashLoopBackOff waiting reason); otherwise the back-off
        advances (Next) and the start goes ahead."""
        last = next((x for x in st.containers.get(c["name"]) or [] if x.state == C.CONTAINER_EXITED), None)
        if last is None:
            return False
        ts = last.finished_at / 1e9 if last.finished_at else time.time()
        key = stable_key(pod, c)
        md = pod["metadata"]
        if self.backoff.is_in_backoff_since(key, ts):
            if self.recorder is not None:
                self.recorder.event(pod, "Warning", "BackOff", "Back-off restarting failed container")
            msg = (f"Back-off {_go_duration(self.backoff.get(key))} restarting failed container={c['name']} "
                   f"pod={md['name']}_{md.get('namespace', '')}({md['uid']})")
            self.reasons.setdefault(md["uid"], {})[c["name"]] = ("CrashLoopBackOff", msg)
            self._backoff_due[(md["uid"], c["name"])] = (key, ts)
            return True
        self.backoff.next(key, ts)
        self._backoff_due.pop((md["uid"], c["name"]), None)
        return False

    def backoff_remaining(self, uid, name) -> float:
        """Seconds until a container held back by do_backoff may start (0 when none is held)."""
        due = self._backoff_due.get((uid, name))
        return self.backoff.remaining(*due) if due else 0.0

    async def kill_pod(self, uid: str, grace: int = 30, pod: dict | None = None, sandboxes=None, clear_backoff: bool = True):
        sbs = sandboxes if sandboxes is not None else await self.cri.list_pod_sandbox(uid)
        hooks = pod is not None and any(((sc.get("lifecycle") or {}).get("preStop"))
                                        for sc in (pod.get("spec") or {}).get("containers") or [])
        for s in sbs:
            if s.state != C.SANDBOX_READY:
                continue   # already stopped: its containers are gone with it
            if grace or hooks:
                conts = await self.cri.list_containers(s.id)
                await asyncio.gather(*(self._kill_container(pod, c, grace) for c in conts if c.state == C.CONTAINER_RUNNING))
            # grace 0 and no preStop hook: StopPodSandbox kills the containers itself (one RPC, not 2 + N)
            await self.cri.stop_pod_sandbox(s.id)
        if clear_backoff:
            self.backoff.drop_prefix_containing(f"_{uid}_")
            for k in [k for k in self._backoff_due if k[0] == uid]:
                del self._backoff_due[k]

    async def kill_and_remove(self, uid: str, sandboxes=None):
        """The pod is gone from the API: one list, stop what still runs, remove everything."""
        sbs = sandboxes if sandboxes is not None else await self.cri.list_pod_sandbox(uid)
        await self.kill_pod(uid, 0, None, sbs)
        await self.remove_pod(uid, sbs)

    async def _kill_container(self, pod, c, grace):
        if pod is not None:
            for sc in (pod.get("spec") or {}).get("containers") or []:
                if sc["name"] == c.metadata.name:
                    pre = (sc.get("lifecycle") or {}).get("preStop")
                    if pre:   # kuberuntime_container.go executePreStopHook, bounded by the grace period
                        ip = self.sandbox_ips.get(c.pod_sandbox_id) or self.node_ip
                        err = await self.run_handler(pod, sc, c.id, pre, ip, min(grace, 30) or 1)
                        if err and self.recorder:
                            self.recorder.event(pod, "Warning", "FailedPreStopHook", err)
        await self.cri.stop_container(c.id, grace)

    # ------------------------------------------------------------ garbage collection
    async def garbage_collect(self, is_active, max_per_pod_container: int = 1, max_containers: int = -1,
                              min_age: float = 0.0, now_ns: int | None = None, sources_ready: bool = True,
                              has_volumes=None) -> dict:
        """kuberuntime_gc.go GarbageCollect: dead containers older than min_age are evictable,
        grouped in (pod, container name) units. Only when all pod sources are ready
        (allSourcesReady, :212-219) does a pod unknown to the kubelet count as deleted, and then
        all its units go; every other unit keeps its newest max_per_pod_container (<0: no limit).
        With max_containers ≥ 0 the units are first cut to an equal share (min 1, :227-234) and
        then the oldest go until the node is under it. Sandboxes (evictSandboxes, :256-311):
        not ready and without containers; a deleted pod loses all of them, others keep their
        newest. Container logs go with their containers; a deleted pod's directory (logs and
        volumes) goes once nothing of it is left (evictPodLogsDirectories, sources ready only) and
        no volume is still mounted in it (cleanupOrphanedPodDirs: `has_volumes(uid)`; deleting a
        directory with a live network mount would delete the remote data)."""
        now_ns = now_ns or time.time_ns()
        deleted = (lambda uid: not is_active(uid)) if sources_ready else (lambda uid: False)   # noqa: E731
        sbs = await self.cri.list_pod_sandbox()
        conts = await self.cri.list_containers()
        sb_uid = {s.id: s.labels.get(L_POD_UID, "") for s in sbs}
        groups: dict[tuple[str, str], list] = {}
        for c in conts:
            if c.state == C.CONTAINER_RUNNING or c.state == C.CONTAINER_CREATED:
                continue
            if now_ns - c.created_at < min_age * 1e9:
                continue
            uid = sb_uid.get(c.pod_sandbox_id) or c.labels.get(L_POD_UID, "")
            groups.setdefault((uid, c.metadata.name), []).append(c)
        evict = []
        for key, lst in list(groups.items()):
            lst.sort(key=lambda c: c.created_at, reverse=True)
            if deleted(key[0]):
                evict += lst
                del groups[key]
            elif max_per_pod_container >= 0:
                evict += lst[max_per_pod_container:]
                groups[key] = lst[:max_per_pod_container]
        if max_containers >= 0 and groups and sum(map(len, groups.values())) > max_containers:
            share = max(1, max_containers // len(groups))
            for key, lst in groups.items():
                evict += lst[share:]
                groups[key] = lst[:share]
            rest = sorted((c for lst in groups.values() for c in lst), key=lambda c: c.created_at)
            evict += rest[:max(0, len(rest) - max_containers)]
        removed = 0
        gone = set()
        for c in evict:
            try:
                st, _ = await self.cri.container_status(c.id)
                log_path = st.log_path
            except grpc.RpcError:
                log_path = ""
            try:
                await self.cri.remove_container(c.id)
                removed += 1
                gone.add(c.id)
            except grpc.RpcError:
                continue
            if log_path:
                try:
                    os.unlink(log_path)
                except OSError:
                    pass
            self.remove_legacy_log_links(c.id)
        self.remove_legacy_log_links()
        left = {c.pod_sandbox_id for c in conts if c.id not in gone}
        by_uid: dict[str, list] = {}
        for s in sbs:
            by_uid.setdefault(sb_uid[s.id], []).append(s)
        sb_removed = 0
        remaining = {u for u in by_uid if u}
        for uid, lst in by_uid.items():
            lst.sort(key=lambda s: s.created_at, reverse=True)
            candidates = lst if (uid and deleted(uid)) else lst[1:]
            kept = len(lst) - len(candidates)
            for s in candidates:
                if s.state == C.SANDBOX_READY or s.id in left:
                    kept += 1
                    continue
                try:
                    await self.cri.remove_pod_sandbox(s.id)
                    self.sandbox_ips.pop(s.id, None)
                    sb_removed += 1
                except grpc.RpcError:
                    kept += 1
            if not kept:
                remaining.discard(uid)
        dirs = 0
        if sources_ready:
            root = os.path.join(self.root, "pods")
            try:
                names = os.listdir(root)
            except OSError:
                names = []
            for uid in names:
                if uid not in remaining and deleted(uid):
                    if has_volumes is not None and has_volumes(uid):
                        continue
                    shutil.rmtree(os.path.join(root, uid), ignore_errors=True)
                    dirs += 1
        return {"containers": removed, "sandboxes": sb_removed, "pod_dirs": dirs}

    async def remove_pod(self, uid: str, sandboxes=None):
        for s in sandboxes if sandboxes is not None else await self.cri.list_pod_sandbox(uid):
            await self.cri.remove_pod_sandbox(s.id)
            self.sandbox_ips.pop(s.id, None)
