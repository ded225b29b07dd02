"""The kubelet: node agent that admits, runs and reports pods on one MI355X node.

Reference pkg/kubelet: NewMainKubelet/Run (kubelet.go:340,1361), syncLoop/syncLoopIteration
(:1772,1839), HandlePodAdditions with canAdmitPod (:1990-2023, :1729-1743) — predicate
admission (lifecycle/predicate.go:56-80) including the fork's DeviceManager.AdmitPod via
UpdatePluginResources (cm/container_manager_linux.go:619-621); per-pod workers
(pod_workers.go:153,195); PLEG relist (pleg/generic.go:182); node status every 10 s
(kubelet_node_status.go:380,393) with the fork's per-resource Capacity + full
Status.ExtendedResources and removal of vanished resources (:552-553,608-622); status
manager; prober (prober/prober_manager.go:98); eviction (eviction/eviction_manager.go:214).

amdkube differences (latency-driven, SURVEY §6 north star):
  * evented PLEG (CRI GetContainerEvents) with relist as the backstop;
  * node status is pushed immediately when device capacity/health changes (the reference
    waits for the next 10 s tick: SURVEY §3.2 latency note);
  * GPU assignment is read from the API object on every (re)start, so a kubelet restart
    never reshuffles devices (reference e2e test/e2e_node/gpu_device_plugin.go:90-103).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import socket
import time
from dataclasses import dataclass, field

import aiohttp

from .. import GIT_VERSION
from ..api import meta as m
from ..api.helpers import (is_pod_terminal, node_allocatable, pod_host_ports, pod_requests, find_untolerated_taint)
from ..api.labels import node_requirements_as_selector
from ..client import Client, EventRecorder, Informer
from ..deviceplugin.amd import TOPOLOGY_LABEL
from ..grpcdesc.cri import CRI as C
from ..utils.features import FeatureGate
from ..utils.metrics import Counter, Gauge, new_registry
from ..utils.quantiles import QuantileSummary as Summary
from .cm import enforce_pods_cgroup, node_allocatable as reserved_allocatable, parse_reserved
from .cri_client import CURRENT_POD, CRIClient
from .devicemanager import AdmissionError, ManagerImpl, ManagerStub
from ..utils.trace import POD_TRACE
from ..volume import VolumeError
from .kuberuntime import L_POD_UID, RuntimeManager, SandboxRef, apply_event
from .qos import CRITICAL_ANNOTATION
from .status import StatusManager, generate_status
from ..utils import wait_event

log = logging.getLogger("amdkube.kubelet")

# pkg/kubelet/types/pod_update.go
SOURCE_ANNOTATION = "kubernetes.io/config.source"
HASH_ANNOTATION = "kubernetes.io/config.hash"
MIRROR_ANNOTATION = "kubernetes.io/config.mirror"


def _atomic_write(path: str, data: bytes):
    """pkg/volume/util/atomic_writer.go: a running container never sees a half-written volume
    file; unchanged content is not rewritten (every pod sync resolves the volumes again)."""
    try:
        with open(path, "rb") as f:
            if f.read() == data:
                return
    except OSError:
        pass
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


MAX_IMAGES_IN_NODE_STATUS, MAX_NAMES_PER_IMAGE = 50, 5     # kubelet_node_status.go:52-57


@dataclass
class KubeletConfig:
    node_name: str = field(default_factory=socket.gethostname)
    root_dir: str = "/var/lib/kubelet"
    # legacy container log symlinks for cluster logging (kuberuntime legacyContainerLogsDir):
    # "" = /var/log/containers for the default root dir, <root_dir>/containers-logs otherwise
    container_logs_dir: str = ""
    plugins_dir: str = "/var/lib/kubelet/device-plugin/plugins"
    v1beta1_socket: str | None = None
    cri_socket: str = "/var/run/amdkube/rocshim.sock"
    address: str = "127.0.0.1"
    port: int = 10250
    node_ip: str = "127.0.0.1"
    node_status_update_frequency: float = 10.0     # kubeletconfig defaults.go:147-148
    relist_period: float = 1.0                      # pleg/generic.go relist period
    sync_frequency: float = 60.0
    max_pods: int = 110
    node_labels: dict = field(default_factory=dict)
    register_with_taints: list = field(default_factory=list)
    feature_gates: str = ""
    evented_pleg: bool = True
    prioritize_device_pods: bool = True              # start pods that hold accelerators before the rest of a burst
    device_pod_start_window: float = 0.25            # the longest a device-less pod waits for them (s)
    eviction_memory_available_bytes: int = 100 * 2 ** 20
    eviction_interval: float = 10.0
    eviction_hard: str | None = None                # --eviction-hard (default: memory.available<eviction_memory_available_bytes)
    eviction_soft: str = ""                         # --eviction-soft
    eviction_soft_grace_period: str = ""            # --eviction-soft-grace-period
    eviction_minimum_reclaim: str = ""              # --eviction-minimum-reclaim
    eviction_pressure_transition_period: float = 300.0
    eviction_max_pod_grace_period: int = 0
    chaos_chance: float = 0.0
    gpu_stats_backend: str = "none"                 # amdsmi|sysfs|fake|auto|none (per-container accelerator stats)
    oom_watcher: bool = True                        # SystemOOM node events (oom_watcher.go)
    oom_vmstat_path: str = "/proc/vmstat"
    oom_kmsg_path: str | None = "/dev/kmsg"
    cpu_capacity: int | None = None
    memory_capacity: int | None = None
    pod_manifest_path: str | None = None            # static pods (--pod-manifest-path)
    bootstrap_checkpoint_path: str | None = None    # --bootstrap-checkpoint-path (checkpoint.py)
    file_check_frequency: float = 20.0              # kubeletconfig FileCheckFrequency
    apparmor_fs: str | None = None                  # securityfs apparmor dir (None: discover from /proc/mounts)
    cluster_dns: list = field(default_factory=list)   # --cluster-dns
    cluster_domain: str = ""                          # --cluster-domain
    resolv_conf: str = "/etc/resolv.conf"             # --resolv-conf
    gc_period: float = 60.0                           # container GC cadence (kubelet.go ContainerGCPeriod)
    maximum_dead_containers_per_container: int = 1    # --maximum-dead-containers-per-container
    maximum_dead_containers: int = -1                 # --maximum-dead-containers
    minimum_container_ttl_duration: float = 0.0       # --minimum-container-ttl-duration (s)
    kube_reserved: str = ""                           # --kube-reserved cpu=…,memory=…,ephemeral-storage=…
    system_reserved: str = ""                         # --system-reserved
    enforce_node_allocatable: str = "pods"            # --enforce-node-allocatable (pods | none)
    cgroup_root: str = ""                             # cgroup v2 dir holding kubepods (empty: no enforcement)
    allowed_unsafe_sysctls: list = field(default_factory=list)   # --experimental-allowed-unsafe-sysctls
    cpu_manager_policy: str = "none"                  # --cpu-manager-policy (none | static)
    cpu_manager_reconcile_period: float = 10.0        # --cpu-manager-reconcile-period (s)
    cpu_topology: object = None                       # cpumanager.CPUTopology (None: discover from sysfs)
    image_gc_high_threshold: int = 85                 # --image-gc-high-threshold (%)
    image_gc_low_threshold: int = 80                  # --image-gc-low-threshold (%)
    minimum_image_ttl_duration: float = 120.0         # --minimum-image-ttl-duration (s)
    image_gc_period: float = 300.0                    # ImageGCPeriod
    tls_cert_file: str | None = None                  # --tls-cert-file (serve HTTPS)
    tls_private_key_file: str | None = None           # --tls-private-key-file
    client_ca_file: str | None = None                 # --client-ca-file (x509 client authentication)
    anonymous_auth: bool = True                       # --anonymous-auth
    authentication_token_webhook: bool = False        # --authentication-token-webhook (TokenReview)
    authorization_mode: str = "AlwaysAllow"           # --authorization-mode (AlwaysAllow | Webhook)
    cert_dir: str | None = None                       # --cert-dir (rotated certificates)
    rotate_certificates: bool = False                 # --rotate-certificates (client certificate rotation)
    rotate_server_certificates: bool = False          # RotateKubeletServerCertificate: serving cert via CSR
    config_file: str | None = None                    # --config (KubeletConfiguration file)
    dynamic_config_dir: str | None = None             # --dynamic-config-dir
    volume_plugin_dir: str | None = None              # --volume-plugin-dir (FlexVolume drivers; default <root>/volumeplugins)
    enable_controller_attach_detach: bool = True      # --enable-controller-attach-detach
    volume_mounter: str = "auto"                      # auto (system when root, else none) | system | none | fake
    volume_mount_timeout: float = 120.0               # WaitForAttachAndMount timeout (s)
    volume_reconcile_period: float = 2.0              # reconciler loop period (s)
    volume_remount_period: float = 60.0               # re-render secret/configMap/downwardAPI/projected content (s)
    cloud_provider: str = ""                          # --cloud-provider ("external": cloud-controller-manager initialises the node)
    cloud_config: str = ""                            # --cloud-config (in-tree providers: aws, gce, azure, openstack, vsphere, cloudstack, ovirt, photon, baremetal)
    enable_server: bool = True                        # --enable-server (the authenticated API on --port)
    enable_debugging_handlers: bool = True            # --enable-debugging-handlers (logs, exec, attach, portForward, run, pprof)
    read_only_port: int = -1                          # --read-only-port (unauthenticated read-only API; -1/0: off; CLI default 10255)
    healthz_port: int = -1                            # --healthz-port (-1/0: off; CLI default 10248)
    healthz_bind_address: str = "127.0.0.1"           # --healthz-bind-address
    manifest_url: str | None = None                   # --manifest-url (HTTP static pod source)
    manifest_url_header: dict = field(default_factory=dict)   # --manifest-url-header
    http_check_frequency: float = 20.0                # --http-check-frequency (s)
    register_node: bool = True                        # --register-node
    register_schedulable: bool = True                 # --register-schedulable (false: registers unschedulable)
    pod_cidr: str = ""                                # --pod-cidr (standalone; the controller's CIDR wins)
    provider_id: str = ""                             # --provider-id
    allow_privileged: bool = True                     # --allow-privileged
    host_network_sources: list = field(default_factory=lambda: ["*"])   # --host-network-sources (api, file, http, *)
    host_pid_sources: list = field(default_factory=lambda: ["*"])       # --host-pid-sources
    host_ipc_sources: list = field(default_factory=lambda: ["*"])       # --host-ipc-sources
    pods_per_core: int = 0                            # --pods-per-core (0: only --max-pods)
    serialize_image_pulls: bool = True                # --serialize-image-pulls
    registry_qps: float = 5.0                         # --registry-qps (image pulls per second; 0: unlimited)
    registry_burst: int = 10                          # --registry-burst
    event_qps: float = 5.0                            # --event-qps (0: unlimited)
    event_burst: int = 10                             # --event-burst
    runtime_request_timeout: float = 10.0             # --runtime-request-timeout (s, per CRI call; CLI default 2m)
    image_service_endpoint: str | None = None         # --image-service-endpoint (separate CRI image service)
    keep_terminated_pod_volumes: bool = False         # --keep-terminated-pod-volumes
    volume_stats_agg_period: float = 60.0             # --volume-stats-agg-period (du cache TTL, s)
    cpu_cfs_quota: bool = True                        # --cpu-cfs-quota (CPU limits become CFS quota)
    cgroup_driver: str = "cgroupfs"                   # --cgroup-driver: cgroupfs | systemd (slices and scopes)
    protect_kernel_defaults: bool = False             # --protect-kernel-defaults
    seccomp_profile_root: str | None = None           # --seccomp-profile-root (default <root-dir>/seccomp)


class PodWorker:
    __slots__ = ("uid", "pending", "task", "last_sync")

    def __init__(self, uid):
        self.uid = uid
        self.pending = asyncio.Event()
        self.task: asyncio.Task | None = None
        self.last_sync = 0.0


def _semantic(pod: dict):
    md = pod.get("metadata") or {}
    return (pod.get("spec"), md.get("labels"), md.get("annotations"), md.get("deletionTimestamp"),
            md.get("deletionGracePeriodSeconds"))


class _ImageGCAdapter:
    """eviction.ImageGC over the kubelet's image garbage collector."""
    def __init__(self, k):
        self.k = k

    async def delete_unused_images(self) -> int:
        return int(await self.k.image_gc.delete_unused() or 0)


class _ContainerGCAdapter:
    """eviction.ContainerGC: remove every dead container."""
    def __init__(self, k):
        self.k = k

    async def delete_all_unused_containers(self):
        await self.k.container_gc()


class Kubelet:
    def __init__(self, client: Client, config: KubeletConfig, smi_backend=None):
        from . import kubeletconfig as kcfg
        self.dynamic = None
        gates = FeatureGate(config.feature_gates)
        if config.config_file:        # --config: a KubeletConfiguration file over the flags
            config = kcfg.apply(config, kcfg.load_file(config.config_file))
        if config.dynamic_config_dir and gates("DynamicKubeletConfig"):
            self.dynamic = kcfg.DynamicConfig(config.dynamic_config_dir)
            config = self.dynamic.bootstrap(config)
        self.restart_requested = asyncio.Event()
        self.client = client
        self.cfg = config
        self.node_name = config.node_name
        # an in-tree cloud provider (kubelet_node_status.go setNodeAddress / initialNode): the node's
        # addresses, providerID, zone and instance type come from the cloud
        self.cloud, self._cloud_addrs = None, None
        if config.cloud_provider and config.cloud_provider != "external":
            from ..cloudprovider import get_cloud_provider, load_config
            self.cloud = get_cloud_provider(config.cloud_provider, load_config(config.cloud_config or None))
        self.gates = FeatureGate(config.feature_gates)
        self.metrics = new_registry()
        self._init_metrics()
        self.cri = CRIClient(config.cri_socket, metrics=(self.m_rt_ops, self.m_rt_errs, self.m_rt_lat),
                             timeout=config.runtime_request_timeout or 10.0,
                             image_socket=config.image_service_endpoint)
        self.pods: dict[str, dict] = {}
        self.admitted: set[str] = set()
        self.rejected: dict[str, tuple[str, str]] = {}
        self.workers: dict[str, PodWorker] = {}
        self._device_starting: set[str] = set()      # device-holding pods in their first start
        self._device_started: set[str] = set()       # … and those past it (pruned in _cleanup)
        self._device_idle = asyncio.Event()
        self._device_idle.set()
        self.terminated_deleted: set[str] = set()
        if self.gates("DevicePlugins"):
            self.dm = ManagerImpl(config.plugins_dir, active_pods=self.active_pods, registry=self.metrics,
                                  v1beta1_socket=config.v1beta1_socket)
        else:
            self.dm = ManagerStub()
        self.recorder = EventRecorder(client, "kubelet", self.node_name, qps=config.event_qps, burst=config.event_burst)
        self.runtime = RuntimeManager(self.cri, self.dm, config.root_dir, self.recorder, image_pull_qps=config.registry_qps,
                                      image_pull_burst=config.registry_burst, serialize_image_pulls=config.serialize_image_pulls)
        self.runtime.cpu_cfs_quota = config.cpu_cfs_quota
        self.runtime.cgroup_driver = config.cgroup_driver
        if config.cgroup_driver == "systemd" and config.cgroup_root:
            from .cgroups import systemd_cgroup_root
            config.cgroup_root = systemd_cgroup_root(config.cgroup_root)
        self.runtime.legacy_logs_dir = config.container_logs_dir or (
            "/var/log/containers" if os.path.abspath(config.root_dir) == "/var/lib/kubelet"
            else os.path.join(config.root_dir, "containers-logs"))
        self._node_keyring = None     # credentialprovider.node_keyring, read on first use
        from .checkpoint import PodCheckpointManager
        self.pod_checkpoints = PodCheckpointManager(config.bootstrap_checkpoint_path) \
            if config.bootstrap_checkpoint_path else None
        self.restored: set[str] = set()   # UIDs started from checkpoints, not yet confirmed by the API
        self._ckpt_chain = None           # the newest queued bootstrap-checkpoint write
        if config.seccomp_profile_root:
            self.runtime.seccomp_root = config.seccomp_profile_root
        self.runtime.node_ip, self.runtime.cluster_domain = config.node_ip, config.cluster_domain
        import psutil as _ps
        self.runtime.memory_capacity = config.memory_capacity or _ps.virtual_memory().total
        from .dns import DNSConfigurer
        self.runtime.dns = DNSConfigurer(config.cluster_dns, config.cluster_domain, config.resolv_conf, config.node_ip,
                                         self.recorder)
        self.gpu_legacy = None
        if self.gates("Accelerators"):   # legacy whole-GPU path (kubelet.go:907-919), alpha
            from .gpu_legacy import AMDGPUManager
            self.gpu_legacy = AMDGPUManager(smi_backend).start()
            self.runtime.legacy, self.runtime.active_pods = self.gpu_legacy, self.active_pods
        from ..security.apparmor import Validator as AppArmorValidator
        self.apparmor = AppArmorValidator(self.gates("AppArmor"), apparmor_fs=config.apparmor_fs)
        from .eviction import Config as EvictionConfig, EvictionManager, parse_thresholds
        hard = config.eviction_hard if config.eviction_hard is not None else f"memory.available<{config.eviction_memory_available_bytes}"
        # cmd/kubelet/app/server.go: ParseThresholdConfig(enforceNodeAllocatable, evictionHard, ...)
        thresholds = parse_thresholds(hard, config.eviction_soft, config.eviction_soft_grace_period,
                                      config.eviction_minimum_reclaim,
                                      [x.strip() for x in (config.enforce_node_allocatable or "").split(",")])
        self.eviction = EvictionManager(
            EvictionConfig(thresholds, config.eviction_pressure_transition_period, config.eviction_max_pod_grace_period),
            kill_pod=self._evict_kill, summary=lambda: self.stats.summary(), image_gc=_ImageGCAdapter(self),
            container_gc=_ContainerGCAdapter(self), recorder=self.recorder,
            node_ref={"kind": "Node", "name": self.node_name, "uid": self.node_name, "namespace": ""},
            clock=time.monotonic, gates=self.gates)
        self.eviction.on_eviction = lambda what: self.m_evictions.labels(what).inc()
        from .sysctl import SAFE, SAFE_ANNOTATION, UNSAFE_ANNOTATION, Whitelist
        self._sysctl_admit = (Whitelist(SAFE, SAFE_ANNOTATION), Whitelist(config.allowed_unsafe_sysctls, UNSAFE_ANNOTATION))
        self._kube_reserved = parse_reserved(config.kube_reserved)
        self._system_reserved = parse_reserved(config.system_reserved)
        from .cpumanager import CPUManager
        self.cpu_manager = CPUManager(config.cpu_manager_policy, config.cpu_topology,
                                      self._kube_reserved.get("cpu", 0) + self._system_reserved.get("cpu", 0),
                                      os.path.join(config.root_dir, "cpu_manager_state"))
        self.runtime.cpu_manager = self.cpu_manager
        from .auth import KubeletAuth
        self.auth = KubeletAuth(self.node_name, client, config.anonymous_auth, config.authentication_token_webhook,
                                config.authorization_mode)
        self.cert_managers = []
        cert_dir = config.cert_dir or os.path.join(config.root_dir, "pki")
        if config.rotate_certificates and self.gates("RotateKubeletClientCertificate"):
            from .certificate import CertManager
            cmc = CertManager(client, cert_dir, self.node_name, "client")
            cmc.listeners.append(lambda p: client.set_client_cert(p, p))
            if cmc.current():
                client.set_client_cert(cmc.current_path, cmc.current_path)
            self.cert_managers.append(cmc)
        self.server_cert_manager = None
        if config.rotate_server_certificates and self.gates("RotateKubeletServerCertificate"):
            from .certificate import CertManager
            self.server_cert_manager = CertManager(client, cert_dir, self.node_name, "server",
                                                   addresses=[config.node_ip, self.node_name])
            self.server_cert_manager.listeners.append(lambda p: self.server and self.server.reload_cert(p))
            self.cert_managers.append(self.server_cert_manager)
        from .images import ImageGCManager
        self.image_gc = ImageGCManager(self.cri, config.image_gc_high_threshold, config.image_gc_low_threshold,
                                       config.minimum_image_ttl_duration, recorder=self.recorder,
                                       node_ref=lambda: {"kind": "Node", "metadata": {"name": self.node_name, "uid": self.node_name}})
        self.runtime.gpu_numa = self._gpu_numa
        self.volume_manager = self._volume_manager(config)
        from .stats import StatsProvider
        self.stats = StatsProvider(self, du_ttl=config.volume_stats_agg_period)
        self._cpuset_applied: dict[str, str] = {}
        self._pods_cgroup_enforced = None
        self._cgroup_task: asyncio.Task | None = None
        self._cgroup_manager = None         # cgroups.CgroupManager for --cgroup-driver
        self.pressure: set[str] = set()
        self.status = StatusManager(client, on_terminal=self._on_terminal)
        self.node: dict | None = None
        self.informer: Informer | None = None
        self.svc_informer: Informer | None = None
        # prober_manager.go: one worker task per (pod, container, probe type)
        from .prober import ProbeManager
        self.probes = ProbeManager(self.status.get, runner=self._probe_exec, recorder=self.recorder,
                                   on_change=self.dispatch)
        self._tasks: list[asyncio.Task] = []
        self._node_dirty = asyncio.Event()
        self._sandbox_uid: dict[str, str] = {}
        self._pleg_snapshot: dict[str, int] = {}
        self._pleg_owner: dict[str, str] = {}
        # runtime pod-status cache (reference kubecontainer.Cache fed by PLEG, GetNewerThan): the
        # status observed after a sync stays valid until a PLEG event for the pod (generation bump)
        # or any mutating CRI call by this kubelet
        self._rt_gen: dict[str, int] = {}
        self._rt_cache: dict[str, tuple] = {}     # uid -> ((gen, mutations), PodRuntimeStatus, fetch start ns)
        self._rt_pending: dict[str, list] = {}    # uid -> full-status events that arrived while the cache was stale
        self._pending_waiters: dict[str, asyncio.Event] = {}
        self._full_events = False                 # the runtime's events carry complete pod state
        self.smi = smi_backend
        self.server = None
        self.first_seen: dict[str, float] = {}
        self.started_at = time.time()
        self._runtime_uids: set[str] = set()
        self._deadline_timers: set[str] = set()
        self._static_read = False
        self.last_sync_loop = time.time()
        self.sync_errors: dict[str, str] = {}
        self.static: dict[str, dict] = {}      # uid -> static pod from --pod-manifest-path
        self.mirrors: dict[tuple, dict] = {}   # (ns, name) -> mirror pod in the API
        self._static_dirty = asyncio.Event()

    def _volume_manager(self, config):
        from ..volume import FakeMounter, NoopMounter, PluginMgr, SysMounter, VolumeHost, default_plugins
        from .podcontext import PodContext
        from .volumemanager import VolumeManager
        kind = config.volume_mounter
        if kind == "auto":
            kind = "system" if os.geteuid() == 0 else "none"
        mounter = {"system": SysMounter, "none": NoopMounter, "fake": FakeMounter}[kind]()
        host = VolumeHost(config.root_dir, self.node_name, self.client, mounter, pod_context=PodContext(self),
                          node_ip=config.node_ip, plugins_dir=config.volume_plugin_dir)
        return VolumeManager(self, PluginMgr(default_plugins(), host), config.enable_controller_attach_detach,
                             config.volume_reconcile_period, config.volume_mount_timeout, config.volume_remount_period)

    def _init_metrics(self):
        r = self.metrics
        self.m_pod_start = Summary("kubelet_pod_start_latency_microseconds", "Latency in microseconds for a single pod to go from pending to running.", registry=r)
        self.m_worker = Summary("kubelet_pod_worker_latency_microseconds", "Latency in microseconds to sync a single pod. Broken down by operation type: create, update, or sync", ["operation_type"], registry=r)
        self.m_pleg = Summary("kubelet_pleg_relist_latency_microseconds", "Latency in microseconds for relisting pods in PLEG.", registry=r)
        self.m_pleg_interval = Summary("kubelet_pleg_relist_interval_microseconds", "Interval in microseconds between relisting in PLEG.", registry=r)
        self.m_containers_per_pod = Summary("kubelet_containers_per_pod_count", "The number of containers per pod.", registry=r)
        self.m_rt_ops = Counter("kubelet_runtime_operations", "Cumulative number of runtime operations by operation type.", ["operation_type"], registry=r)
        self.m_rt_errs = Counter("kubelet_runtime_operations_errors", "Cumulative number of runtime operation errors by operation type.", ["operation_type"], registry=r)
        self.m_rt_lat = Summary("kubelet_runtime_operations_latency_microseconds", "Latency in microseconds of runtime operations.", ["operation_type"], registry=r)
        self.m_running_pods = Gauge("kubelet_running_pod_count", "Number of pods currently running", registry=r)
        self.m_running_containers = Gauge("kubelet_running_container_count", "Number of containers currently running", registry=r)
        self.m_evictions = Counter("kubelet_evictions", "Cumulative number of pod evictions by eviction signal", ["eviction_signal"], registry=r)

    # ================================================================ lifecycle
    async def _check_cgroup_driver(self):
        """dockershim NewDockerService (docker_service.go:237-253): the kubelet and its runtime
        must agree on the cgroup driver, or pods would land in cgroups nobody enforces. A runtime
        that does not report one (CRI Status info `cgroupDriver`) is not checked."""
        try:
            st = await self.cri.status()
            rt = dict(getattr(st, "info", {}) or {}).get("cgroupDriver", "")
        except Exception as e:
            log.debug("runtime status for the cgroup driver check: %r", e)
            return
        if rt and rt != self.cfg.cgroup_driver:
            raise RuntimeError(f"misconfiguration: kubelet cgroup driver: {self.cfg.cgroup_driver!r} is different from "
                               f"the container runtime's cgroup driver: {rt!r}")

    async def start(self):
        os.makedirs(os.path.join(self.cfg.root_dir, "pods"), exist_ok=True)
        await self.cri.connect()
        await self._check_cgroup_driver()
        # pods the runtime already holds anything of (a previous kubelet incarnation): decided
        # from runtime state, never from creation timestamps (static pods get a fresh
        # creationTimestamp on every manifest read; API clocks may run ahead of the node's)
        self._runtime_uids = {s.labels.get(L_POD_UID, "") for s in await self.cri.list_pod_sandbox()} - {""}
        if self.gpu_legacy is not None:   # in-use GPUs survive a kubelet restart (the reference inspects docker)
            self.gpu_legacy.rebuild([(c.labels.get(L_POD_UID, ""), c.metadata.name, dict(c.annotations))
                                     for c in await self.cri.list_containers() if c.state == C.CONTAINER_RUNNING])
        await self.dm.start()
        self.recorder.start()
        self.status.start()
        if hasattr(self.dm, "store"):
            self.dm.store.listeners.append(lambda rname: self._node_dirty.set())
        scm = self.server_cert_manager
        if scm is not None and scm.current() is None:
            try:   # the first serving certificate before the listener starts (needs an approved CSR)
                await asyncio.wait_for(scm.rotate(), 30)
            except Exception as e:
                log.warning("no kubelet serving certificate yet (%r); serving without TLS until one is issued", e)
        if self.cfg.protect_kernel_defaults:
            from .node_setup import kernel_tunables
            kernel_tunables(True)
        from .server import KubeletServer
        if self.cfg.enable_server:
            self.server = await KubeletServer(self).start(self.cfg.address, self.cfg.port)
        self.extra_servers = []
        if self.cfg.read_only_port > 0:     # server.go ListenAndServeKubeletReadOnlyServer
            self.extra_servers.append(await KubeletServer(self, mode="readonly").start(self.cfg.address, self.cfg.read_only_port))
        if self.cfg.healthz_port > 0:       # cmd/kubelet/app/server.go healthz listener
            self.extra_servers.append(await KubeletServer(self, mode="healthz").start(self.cfg.healthz_bind_address,
                                                                                       self.cfg.healthz_port))
        for cmgr in self.cert_managers:
            self._tasks.append(asyncio.create_task(cmgr.run(), name=f"cert-rotation-{cmgr.kind}"))
        self._tasks += [asyncio.create_task(self._relist_loop(), name="pleg-relist"),
                        asyncio.create_task(self._housekeeping(), name="housekeeping"),
                        asyncio.create_task(self._gc_loop(), name="container-gc"),
                        asyncio.create_task(self._eviction_loop(), name="eviction")]
        if self.cfg.evented_pleg:
            self._tasks.append(asyncio.create_task(self._evented_pleg(), name="pleg-events"))
        if self.cfg.oom_watcher:    # kubelet.go: oomWatcher.Start(nodeRef)
            from .oom_watcher import OOMWatcher
            self.oom_watcher = OOMWatcher(self.recorder, lambda: {"kind": "Node", "metadata": {"name": self.node_name,
                                                                                               "uid": self.node_name}},
                                          vmstat=self.cfg.oom_vmstat_path, kmsg=self.cfg.oom_kmsg_path)
            self._tasks.append(asyncio.create_task(self.oom_watcher.run(), name="oom-watcher"))
        self.volume_manager.start()
        if self.cpu_manager.policy != "none":
            self._tasks.append(asyncio.create_task(self._cpu_reconcile_loop(), name="cpu-manager"))
        restored = self._restore_checkpoints() if self.pod_checkpoints is not None else 0
        if self.cfg.pod_manifest_path or self.cfg.manifest_url or restored:
            # static pods run with or without an apiserver (kubeadm: the apiserver IS a static
            # pod), so registration is retried in the background (kubelet_node_status.go
            # registerWithAPIServer: exponential back-off up to 7 s)
            self._tasks.append(asyncio.create_task(self._static_pods_loop(), name="static-pods"))
            self._tasks.append(asyncio.create_task(self._connect_api(), name="api-connect"))
        else:
            await self._connect_api()
        log.info("kubelet %s started (cri=%s, devicePlugins=%s)", self.node_name, self.cfg.cri_socket, self.gates("DevicePlugins"))
        return self

    async def _connect_api(self):
        delay = 0.1
        while True:
            try:
                await self.register_node()
                break
            except (aiohttp.ClientError, OSError, asyncio.TimeoutError) as e:
                log.info("unable to register node %s with the API server: %r; retrying in %.1fs", self.node_name, e, delay)
                await asyncio.sleep(delay)
                delay = min(7.0, delay * 2)
        await self.dm.wait_initial_registration(5.0)
        # service environment variables (kubelet.go serviceLister)
        self.svc_informer = Informer(self.client, "services")
        self.svc_informer.start()
        # this node's own object, as the reference's node lister (kubelet.go nodeInfo): labels a
        # controller sets (the master label, a DaemonSet's nodeSelector target) reach admission
        # at once instead of at the next status update
        self.node_informer = Informer(self.client, "nodes", field_selector=f"metadata.name={self.node_name}")
        self.node_informer.add_handler(on_add=self._on_node, on_update=lambda old, new: self._on_node(new))
        self.node_informer.start()
        self.informer = Informer(self.client, "pods", field_selector=f"spec.nodeName={self.node_name}")
        self.informer.add_handler(on_add=self._on_pod_add, on_update=self._on_pod_update, on_delete=self._on_pod_delete)
        self.informer.start()
        await self.informer.wait_synced(30)
        if self.restored:
            self._reconcile_restored()
        self._tasks.append(asyncio.create_task(self._node_status_loop(), name="node-status"))
        self._static_dirty.set()   # create mirror pods now that the API is there

    def _on_node(self, node: dict):
        cur = self.node or {}
        try:
            newer = int(m.rv_of(node) or 0) >= int(m.rv_of(cur) or 0)
        except ValueError:
            newer = True
        if newer:
            self.node = node

    async def stop(self):
        from ..utils import cancel_and_wait
        await cancel_and_wait(self._tasks)
        await self.volume_manager.stop()
        if self.informer:
            await self.informer.stop()
        if self.svc_informer is not None:
            await self.svc_informer.stop()
        if getattr(self, "node_informer", None) is not None:
            await self.node_informer.stop()
        await cancel_and_wait([w.task for w in self.workers.values()])
        await self.probes.stop()
        if self._ckpt_chain is not None:
            await asyncio.wait({self._ckpt_chain}, timeout=5)     # queued bootstrap-checkpoint writes land
        await self.status.stop()
        await self.recorder.stop()
        await self.dm.stop()
        if self.server:
            await self.server.stop()
        for srv in getattr(self, "extra_servers", []):
            await srv.stop()
        await self.cri.close()
        await self.client.close()

    # ================================================================ node
    def _capacity(self) -> dict:
        import psutil
        cpu = self.cfg.cpu_capacity or psutil.cpu_count() or 1
        mem = self.cfg.memory_capacity or psutil.virtual_memory().total
        pods = self.cfg.max_pods
        if self.cfg.pods_per_core > 0:      # kubelet_node_status.go: min(max-pods, cores × pods-per-core)
            pods = min(pods, cpu * self.cfg.pods_per_core)
        cap = {"cpu": str(cpu), "memory": f"{mem // 1024}Ki", "pods": str(pods)}
        if self.gpu_legacy is not None:   # kubelet_node_status.go:557-562
            from .gpu_legacy import RESOURCE
            cap[RESOURCE] = str(self.gpu_legacy.capacity())
        if self.gates("LocalStorageCapacityIsolation"):
            # kubelet_node_status.go:599-606: the root filesystem's size (container manager capacity)
            import shutil
            try:
                cap["ephemeral-storage"] = str(shutil.disk_usage(
                    self.cfg.root_dir if os.path.isdir(self.cfg.root_dir) else "/").total)
            except OSError:
                cap["ephemeral-storage"] = "0"
        return cap

    async def register_node(self):
        if not self.cfg.register_node:
            # --register-node=false: the node object is someone else's; wait for it to exist
            while (node := await self.client.get_or_none("nodes", self.node_name)) is None:
                await asyncio.sleep(1.0)
            self.node = node
            await self.update_node_status()
            return
        labels = {"kubernetes.io/hostname": self.node_name, "beta.kubernetes.io/os": "linux",
                  "beta.kubernetes.io/arch": "amd64", **self.cfg.node_labels}
        taints = list(self.cfg.register_with_taints)
        ann = {}
        if self.cfg.cloud_provider == "external":
            # kubelet_node_status.go: an external cloud provider initialises the node (providerID,
            # addresses, zone) — register tainted until the cloud-controller-manager has done so,
            # and tell it which address the operator chose
            taints.append({"key": "node.cloudprovider.kubernetes.io/uninitialized", "value": "true", "effect": "NoSchedule"})
            if self.cfg.node_ip:
                ann["alpha.kubernetes.io/provided-node-ip"] = self.cfg.node_ip
        spec = {"taints": taints} if taints else {}
        if self.cloud is not None and self.cloud.instances() is not None:
            inst = self.cloud.instances()
            if not self.cfg.provider_id:
                # cloudprovider.GetInstanceProviderID: "<provider>://<instance id>"
                iid = await inst.instance_id(self.node_name)
                self.cfg.provider_id = iid if "://" in iid else f"{self.cloud.name}://{iid}"
            itype = await inst.instance_type(self.node_name)
            if itype:
                labels["beta.kubernetes.io/instance-type"] = itype
            zone = await asyncio.to_thread(self.cloud.zone_for_node, self.node_name) if hasattr(self.cloud, "zone_for_node") \
                else self.cloud.zones()
            if zone is not None and zone.failure_domain:
                labels["failure-domain.beta.kubernetes.io/zone"] = zone.failure_domain
            if zone is not None and zone.region:
                labels["failure-domain.beta.kubernetes.io/region"] = zone.region
            await self.refresh_cloud_addresses()
        if not self.cfg.register_schedulable:
            spec["unschedulable"] = True
        if self.cfg.pod_cidr:
            spec["podCIDR"] = self.cfg.pod_cidr
        if self.cfg.provider_id:
            spec["providerID"] = self.cfg.provider_id
        node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": self.node_name, "labels": labels,
                                                                "annotations": ann},
                "spec": spec, "status": self._node_status_body({})}
        node["status"].pop("_removed", None)
        try:
            self.node = await self.client.create(node)
        except m.StatusError as e:
            if not m.is_already_exists(e):
                raise
            self.node = await self.client.get("nodes", self.node_name)
        await self.update_node_status()

    async def refresh_cloud_addresses(self):
        """The cloud's view of this node's addresses; with --node-ip that address must be one of
        them and is listed first (kubelet_node_status.go setNodeAddress)."""
        if self.cloud is None or self.cloud.instances() is None:
            return
        try:
            addrs = await self.cloud.instances().node_addresses(self.node_name)
        except Exception as e:
            log.warning("cloud node addresses for %s: %r", self.node_name, e)
            return
        ip = self.cfg.node_ip
        if ip and ip not in ("127.0.0.1", "0.0.0.0"):
            hit = [a for a in addrs if a.get("address") == ip]
            if not hit:
                log.warning("--node-ip %s is not one of the cloud's addresses for %s", ip, self.node_name)
                return
            addrs = hit + [a for a in addrs if a.get("address") != ip]
        self._cloud_addrs = addrs + [{"type": "Hostname", "address": self.node_name}]

    def _node_status_body(self, prev: dict) -> dict:
        cap = self._capacity()
        ext = {}
        if hasattr(self.dm, "store"):
            ext, removed = self.dm.get_capacity()
        else:
            removed = []
        for rname, dom in ext.items():
            cap[rname] = str(len(dom["resources"]))
        alloc = reserved_allocatable(cap, self._kube_reserved, self._system_reserved, self.eviction.thresholds)
        for rname, dom in ext.items():  # allocatable counts only healthy devices (fix #6 for node capacity)
            alloc[rname] = str(sum(1 for d in dom["resources"].values() if d.get("health") == "Healthy"))
        now = m.now_rfc3339()
        prev_conds = {c["type"]: c for c in (prev.get("conditions") or [])}

        def cond(t, ok, reason, msg):
            st = "True" if ok else "False"
            p = prev_conds.get(t)
            return {"type": t, "status": st, "reason": reason, "message": msg, "lastHeartbeatTime": now,
                    "lastTransitionTime": p["lastTransitionTime"] if p and p.get("status") == st else now}
        mem_pressure, disk_pressure = "MemoryPressure" in self.pressure, "DiskPressure" in self.pressure
        conds = [cond("Ready", True, "KubeletReady", "kubelet is posting ready status"),
                 cond("MemoryPressure", mem_pressure, "KubeletHasSufficientMemory" if not mem_pressure else "KubeletHasInsufficientMemory",
                      "kubelet has sufficient memory available" if not mem_pressure else "kubelet has insufficient memory available"),
                 cond("DiskPressure", disk_pressure, "KubeletHasNoDiskPressure" if not disk_pressure else "KubeletHasDiskPressure",
                      "kubelet has no disk pressure" if not disk_pressure else "kubelet has disk pressure"),
                 cond("OutOfDisk", False, "KubeletHasSufficientDisk", "kubelet has sufficient disk space available")]
        if self.dynamic is not None:
            dc = self.dynamic.condition
            conds.append(cond("ConfigOK", dc["status"] == "True", dc["reason"], dc["message"]))
        st = {"capacity": cap, "allocatable": alloc, "conditions": conds,
              "addresses": [{"type": "InternalIP", "address": self.cfg.node_ip}, {"type": "Hostname", "address": self.node_name}],
              "daemonEndpoints": {"kubeletEndpoint": {"Port": self.server.port if self.server else self.cfg.port}},
              "nodeInfo": {"kubeletVersion": GIT_VERSION, "kubeProxyVersion": GIT_VERSION, "operatingSystem": "linux",
                           "architecture": "amd64", "containerRuntimeVersion": "rocshim://0.1.0", "osImage": "Linux",
                           "machineID": "", "systemUUID": "", "bootID": "", "kernelVersion": os.uname().release},
              "extendedResources": ext}
        in_use = self.volume_manager.volumes_in_use()
        if in_use or prev.get("volumesInUse"):
            st["volumesInUse"] = in_use or None     # attachable volumes mounted or about to be (safe detach)
        if self.cfg.cloud_provider == "external":
            del st["addresses"]          # the cloud-controller-manager owns them
        elif self._cloud_addrs:
            st["addresses"] = list(self._cloud_addrs)
        st["_removed"] = removed
        return st

    def _enforce_pods_cgroup(self, alloc: dict):
        """enforceNodeAllocatableCgroups (node_container_manager_linux.go): the pods cgroup capped
        at allocatable, once per allocatable value. Creating it under the systemd driver is a
        D-Bus round trip plus a wait for systemd's directory, so it runs in a worker thread,
        one at a time, and never holds up the node-status update (or the pod workers and PLEG
        sharing its event loop); a failed attempt is retried on a later update."""
        if not self.cfg.cgroup_root or "pods" not in self.cfg.enforce_node_allocatable.split(","):
            return None
        want = (alloc.get("cpu"), alloc.get("memory"))
        if self._pods_cgroup_enforced == want or (self._cgroup_task is not None and not self._cgroup_task.done()):
            return None
        if self._cgroup_manager is None:
            from .cgroups import CgroupManager
            self._cgroup_manager = CgroupManager(self.cfg.cgroup_driver, self.cfg.cgroup_root)

        async def enforce():
            if await asyncio.to_thread(enforce_pods_cgroup, self.cfg.cgroup_root, dict(alloc), manager=self._cgroup_manager):
                self._pods_cgroup_enforced = want
        self._cgroup_task = asyncio.get_running_loop().create_task(enforce(), name="kubelet-pods-cgroup")
        return self._cgroup_task

    async def _node_images(self):
        """setNodeStatusImages (kubelet_node_status.go:692-720): the runtime's images, largest
        first, at most 50, each named by up to 5 of its digests and tags; what the scheduler's
        ImageLocalityPriority scores. None when the runtime cannot list them."""
        try:
            imgs = await self.cri.list_images()
        except Exception as e:
            log.debug("image list for node status failed: %r", e)
            return None
        imgs = sorted(imgs, key=lambda i: -int(i.size))[:MAX_IMAGES_IN_NODE_STATUS]
        return [{"names": (list(i.repo_digests) + list(i.repo_tags))[:MAX_NAMES_PER_IMAGE] or [i.id],
                 "sizeBytes": int(i.size)} for i in imgs]

    async def update_node_status(self):
        prev = (self.node or {}).get("status") or {}
        body = self._node_status_body(prev)
        self._enforce_pods_cgroup(body["allocatable"])
        images = await self._node_images()
        if images is not None:
            body["images"] = images
        removed = body.pop("_removed", [])
        patch = {"status": body}
        # resources that vanished must be deleted explicitly (merge patch: null removes the key)
        for r in removed:
            patch["status"]["capacity"][r] = None
            patch["status"]["allocatable"][r] = None
            patch["status"]["extendedResources"][r] = None
        for r in list(((prev.get("extendedResources") or {}).keys())):
            if r not in body["extendedResources"]:
                patch["status"]["extendedResources"][r] = None
                patch["status"]["capacity"].setdefault(r, None)
                patch["status"]["allocatable"].setdefault(r, None)
        ann = {}
        labels = getattr(self.dm, "plugin_labels", {}) or {}
        if labels.get(TOPOLOGY_LABEL):
            ann[TOPOLOGY_LABEL] = labels[TOPOLOGY_LABEL]
        try:
            # strategic merge (nodeutil.PatchNodeStatus): conditions and addresses merge by
            # `type`, so conditions other components own (node-problem-detector) survive
            self.node = await self.client.patch("nodes", self.node_name, patch, sub="status",
                                                patch_type="application/strategic-merge-patch+json")
            cidr = (self.node.get("spec") or {}).get("podCIDR") or self.cfg.pod_cidr or ""
            if cidr and cidr != getattr(self, "_pod_cidr", ""):
                # kubelet_network.go updatePodCIDR → CRI UpdateRuntimeConfig
                await self.cri.update_runtime_config(cidr)
                self._pod_cidr = cidr
            if ann and any(m.annotations_of(self.node).get(k) != v for k, v in ann.items()):
                self.node = await self.client.patch("nodes", self.node_name, {"metadata": {"annotations": ann}})
        except m.StatusError as e:
            if m.is_not_found(e):
                await self.register_node()
            else:
                raise

    async def _node_status_loop(self):
        while True:
            await wait_event(self._node_dirty, self.cfg.node_status_update_frequency)
            self._node_dirty.clear()
            try:
                if self.cloud is not None:
                    await self.refresh_cloud_addresses()
                await self.update_node_status()
            except Exception as e:
                log.warning("node status update failed: %r", e)
                await asyncio.sleep(0.5)
            if self.dynamic is not None and self.node is not None:
                try:
                    if await self.dynamic.sync(self.client, self.node):
                        self.restart_requested.set()
                except Exception as e:
                    log.warning("dynamic config sync failed: %r", e)

    # ============================================================= pod sources
    def active_pods(self) -> list[dict]:
        return [p for uid, p in self.pods.items() if uid in self.admitted and not is_pod_terminal(p)
                and (self.status.get(uid) or {}).get("phase") not in ("Succeeded", "Failed")]

    def _on_pod_add(self, pod):
        if MIRROR_ANNOTATION in m.annotations_of(pod):
            self.mirrors[(m.namespace_of(pod), m.name_of(pod))] = pod
            return
        uid = m.uid_of(pod)
        self.pods[uid] = pod
        self.restored.discard(uid)
        if self.pod_checkpoints is not None:
            self._checkpoint_io(self.pod_checkpoints.write_pod, pod)
        self.first_seen.setdefault(uid, time.time())
        POD_TRACE(uid, "kubelet_seen")
        self.dispatch(uid)

    def _on_pod_update(self, old, pod):
        if MIRROR_ANNOTATION in m.annotations_of(pod):
            self.mirrors[(m.namespace_of(pod), m.name_of(pod))] = pod
            return
        self.pods[m.uid_of(pod)] = pod
        if self.pod_checkpoints is not None and (old is None or _semantic(old) != _semantic(pod)):
            self._checkpoint_io(self.pod_checkpoints.write_pod, pod)   # removes it when the annotation went away
        # only semantic changes wake the pod worker (reference pkg/kubelet/config/config.go
        # checkAndUpdatePod / podsDifferSemantically): the kubelet's own status writes echo back
        # through the watch and must not trigger another runtime sync
        if old is None or _semantic(old) != _semantic(pod):
            self.dispatch(m.uid_of(pod))

    def _on_pod_delete(self, pod):
        if MIRROR_ANNOTATION in m.annotations_of(pod):
            key = (m.namespace_of(pod), m.name_of(pod))
            if self.mirrors.get(key, {}).get("metadata", {}).get("uid") == m.uid_of(pod):
                self.mirrors.pop(key, None)
            self._static_dirty.set()   # a deleted mirror pod is recreated (mirror_client.go)
            return
        uid = m.uid_of(pod)
        self.pods.pop(uid, None)
        if self.pod_checkpoints is not None:
            self._checkpoint_io(self.pod_checkpoints.delete_pod, pod)
        self.dispatch(uid)

    def _checkpoint_io(self, fn, pod):
        """Bootstrap-checkpoint writes run off the event loop, in order per kubelet (one chain of
        executor jobs), so informer handlers never block on the disk."""
        prev = self._ckpt_chain
        loop = asyncio.get_running_loop()

        async def step():
            if prev is not None:
                await prev
            await loop.run_in_executor(None, fn, pod)
        self._ckpt_chain = loop.create_task(step())

    def _restore_checkpoints(self) -> int:
        """Checkpointed pods run before the API server is reachable (treated as new pods)."""
        n = 0
        for pod in self.pod_checkpoints.load_pods():
            uid = m.uid_of(pod)
            if uid in self.pods:
                continue
            self.restored.add(uid)
            self.pods[uid] = pod
            self.first_seen.setdefault(uid, time.time())
            self.dispatch(uid)
            n += 1
        if n:
            log.info("restored %d pod(s) from bootstrap checkpoints in %s", n, self.pod_checkpoints.path)
        return n

    def _reconcile_restored(self):
        """The API server's pod list is the truth once synced: restored pods it does not know
        were deleted while the kubelet was away."""
        for uid in list(self.restored):
            pod = self.pods.get(uid)
            self.restored.discard(uid)
            if pod is not None:
                self._on_pod_delete(pod)

    # ============================================================= static pods
    def _read_manifests(self) -> dict[str, dict]:
        """pkg/kubelet/config/file.go: every *.yaml/*.yml/*.json in --pod-manifest-path is a pod;
        it is named <name>-<node>, defaults to namespace `default`, and gets a UID derived from
        the node name and the file content (config/common.go applyDefaults)."""
        import hashlib
        import uuid as _uuid

        from ..api.defaults import default_pod
        out = {}
        for doc, fallback, source in self._file_docs() + self._http_docs():
            md = doc.setdefault("metadata", {})
            md["name"] = f"{md.get('name', fallback)}-{self.node_name}"
            md["namespace"] = md.get("namespace") or "default"
            h = hashlib.md5((self.node_name + json.dumps(doc, sort_keys=True)).encode()).hexdigest()
            md["uid"] = str(_uuid.UUID(h))
            md.setdefault("annotations", {}).update({HASH_ANNOTATION: h, SOURCE_ANNOTATION: source})
            md.setdefault("creationTimestamp", m.now_rfc3339())
            doc["apiVersion"], doc["kind"] = "v1", "Pod"
            doc.setdefault("spec", {})["nodeName"] = self.node_name
            doc["spec"].setdefault("restartPolicy", "Always")
            doc.setdefault("status", {"phase": "Pending"})
            default_pod(doc)            # decoded through the scheme: SetDefaults_Pod, as the apiserver would
            out[md["uid"]] = doc
        return out

    def _file_docs(self) -> list[tuple[dict, str, str]]:
        from ..api.scheme import load_manifests
        d = self.cfg.pod_manifest_path
        if not d:
            return []
        try:
            files = sorted(f for f in os.listdir(d) if f.endswith((".yaml", ".yml", ".json")) and not f.startswith("."))
        except OSError:
            return []
        out = []
        for f in files:
            try:
                with open(os.path.join(d, f)) as fh:
                    text = fh.read()
                out += [(x, os.path.splitext(f)[0], "file") for x in load_manifests(text) if x.get("kind", "Pod") == "Pod"]
            except Exception as e:
                log.warning("static pod manifest %s is invalid: %r", f, e)
        return out

    def _http_docs(self) -> list[tuple[dict, str, str]]:
        """config/http.go: --manifest-url returns one Pod, a PodList or a v1 List of pods (with
        --manifest-url-header sent); fetched at most every --http-check-frequency, and a failed
        fetch keeps the last good answer."""
        url = self.cfg.manifest_url
        if not url:
            return []
        now = time.monotonic()
        cached = getattr(self, "_http_cache", None)
        if cached is not None and now - cached[0] < self.cfg.http_check_frequency:
            return json.loads(cached[1])
        import urllib.request
        from ..api.scheme import load_manifests
        try:
            req = urllib.request.Request(url, headers=dict(self.cfg.manifest_url_header))
            with urllib.request.urlopen(req, timeout=10) as r:
                if r.status != 200:
                    raise OSError(f"HTTP {r.status}")
                text = r.read().decode()
            docs = []
            for d in load_manifests(text):
                if d.get("kind") in ("PodList", "List"):
                    docs += [x for x in d.get("items") or [] if x.get("kind", "Pod") == "Pod"]
                elif d.get("kind", "Pod") == "Pod":
                    docs.append(d)
            out = [(x, "http-pod", "http") for x in docs]
        except Exception as e:
            log.warning("static pods from %s: %r", url, e)
            return json.loads(cached[1]) if cached is not None else []
        self._http_cache = (now, json.dumps(out))
        return out

    async def _static_pods_loop(self):
        while True:
            want = await asyncio.to_thread(self._read_manifests)
            for uid in [u for u in self.static if u not in want]:   # manifest removed or changed
                old = self.static.pop(uid)
                self.pods.pop(uid, None)
                self.dispatch(uid)
                mirror = self.mirrors.get((m.namespace_of(old), m.name_of(old)))
                if mirror is not None and m.annotations_of(mirror).get(MIRROR_ANNOTATION) == uid.replace("-", "") \
                        and not any(m.name_of(p) == m.name_of(old) and m.namespace_of(p) == m.namespace_of(old)
                                    for p in want.values()):
                    await self._delete_mirror(mirror)
            for uid, pod in want.items():
                if uid not in self.static:
                    self.static[uid] = pod
                    self.pods[uid] = pod
                    self.first_seen.setdefault(uid, time.time())
                    self.dispatch(uid)
                try:
                    await self._ensure_mirror(pod)
                except Exception as e:
                    log.debug("mirror pod for %s: %r", m.name_of(pod), e)
            self._static_dirty.clear()
            self._static_read = True
            period = self.cfg.file_check_frequency if self.cfg.pod_manifest_path else self.cfg.http_check_frequency
            if self.cfg.pod_manifest_path and self.cfg.manifest_url:
                period = min(period, self.cfg.http_check_frequency)
            await wait_event(self._static_dirty, period)

    async def _ensure_mirror(self, pod):
        """pkg/kubelet/pod/mirror_client.go: the API object that stands for a static pod."""
        key = (m.namespace_of(pod), m.name_of(pod))
        h = m.annotations_of(pod)[HASH_ANNOTATION]
        cur = self.mirrors.get(key) or await self.client.get_or_none("pods", key[1], key[0])
        if cur is not None and m.annotations_of(cur).get(MIRROR_ANNOTATION) == h and \
                not (cur.get("metadata") or {}).get("deletionTimestamp"):
            self.mirrors[key] = cur
            return
        if cur is not None:
            await self._delete_mirror(cur)
        body = json.loads(json.dumps(pod))
        md = body["metadata"]
        md.pop("uid", None)
        md.pop("creationTimestamp", None)
        md["annotations"][MIRROR_ANNOTATION] = h
        body.pop("status", None)
        try:
            self.mirrors[key] = await self.client.create(body, key[0])
        except m.StatusError as e:
            if not m.is_already_exists(e):
                raise
        st = self.status.get(m.uid_of(pod))
        if st:
            self.status.forget(m.uid_of(pod))
            self.status.set(pod, st)     # the status written before the mirror existed

    async def _delete_mirror(self, mirror):
        try:
            await self.client.delete("pods", m.name_of(mirror), m.namespace_of(mirror), grace=0, uid=m.uid_of(mirror))
        except m.StatusError as e:
            if not (m.is_not_found(e) or m.is_conflict(e)):
                raise
        self.mirrors.pop((m.namespace_of(mirror), m.name_of(mirror)), None)

    def dispatch(self, uid: str):
        w = self.workers.get(uid)
        if w is None:
            w = self.workers[uid] = PodWorker(uid)
            pod = self.pods.get(uid)
            if pod is not None:        # kubelet.go dispatchWork on SyncPodCreate
                self.m_containers_per_pod.observe(len((pod.get("spec") or {}).get("containers") or []))
            w.task = asyncio.create_task(self._worker_loop(w), name=f"podworker-{uid[:8]}")
        w.pending.set()

    async def _worker_loop(self, w: PodWorker):
        CURRENT_POD.set(w.uid)   # task-local: CRI mutations are attributed to this pod
        while True:
            await w.pending.wait()
            w.pending.clear()
            t0 = time.perf_counter()
            try:
                done = await self.sync_pod(w.uid)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.exception("sync of pod %s failed: %r", w.uid, e)
                self.sync_errors[w.uid] = repr(e)
                done = False
                asyncio.get_running_loop().call_later(1.0, w.pending.set)
            self.m_worker.labels("sync").observe((time.perf_counter() - t0) * 1e6)
            w.last_sync = time.time()
            self.last_sync_loop = time.time()
            if done:
                self.workers.pop(w.uid, None)
                return

    # ============================================================= admission
    def can_admit(self, pod: dict) -> tuple[bool, str, str]:
        node = self.node or {}
        alloc = node_allocatable(node)
        others = self.active_pods()
        used: dict[str, int] = {}
        ports = set()
        for p in others:
            for k, v in pod_requests(p).items():
                used[k] = used.get(k, 0) + v
            ports.update(pod_host_ports(p))
        want = pod_requests(pod)
        if len(others) + 1 > alloc.get("pods", 110):
            return False, "OutOfpods", "Node didn't have enough resource: pods"
        for k, v in want.items():
            if k in alloc and used.get(k, 0) + v > alloc[k]:
                return False, f"OutOf{k}", f"Node didn't have enough resource: {k}, requested: {v}, used: {used.get(k, 0)}, capacity: {alloc[k]}"
        for hp in pod_host_ports(pod):
            if hp in ports:
                return False, "HostPortConflict", f"host port {hp[2]}/{hp[1]} is already in use"
        labels = m.labels_of(node)
        for k, v in ((pod.get("spec") or {}).get("nodeSelector") or {}).items():
            if labels.get(k) != v:
                return False, "NodeSelectorMismatching", "node labels do not match the pod's node selector"
        na = (((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}).get(
            "requiredDuringSchedulingIgnoredDuringExecution") or {}
        terms = na.get("nodeSelectorTerms") or []
        if terms and not any(node_requirements_as_selector(t.get("matchExpressions")).matches(labels) for t in terms):
            return False, "NodeAffinityMismatching", "node does not match the pod's required node affinity"
        taint = find_untolerated_taint((node.get("spec") or {}).get("taints"), (pod.get("spec") or {}).get("tolerations"),
                                       ("NoExecute",))
        if taint:
            return False, "Taint", f"pod does not tolerate taint {taint.get('key')}={taint.get('value', '')}:NoExecute"
        ok, reason, msg = self._can_run(pod)
        if not ok:
            return False, reason, msg
        ok, reason, msg = self.eviction.admit(pod)   # eviction_manager.go Admit
        if not ok:
            return False, reason, msg
        for wl in self._sysctl_admit:       # kubelet.go:838-848 sysctl whitelists as admit handlers
            ok, reason, msg = wl.admit(pod)
            if not ok:
                return False, reason, msg
        err = self.apparmor.validate(pod)   # lifecycle/handlers.go:142-165
        if err:
            return False, "AppArmor", f"Cannot enforce AppArmor: {err}"
        return True, "", ""

    def _can_run(self, pod: dict) -> tuple[bool, str, str]:
        """kubelet_pods.go canRunPod: --allow-privileged and the --host-{network,pid,ipc}-sources
        allow-lists (a pod's source is file, http or api)."""
        spec = pod.get("spec") or {}
        src = m.annotations_of(pod).get(SOURCE_ANNOTATION) or "api"
        for field_, allowed in (("hostNetwork", self.cfg.host_network_sources), ("hostPID", self.cfg.host_pid_sources),
                                ("hostIPC", self.cfg.host_ipc_sources)):
            if spec.get(field_) and "*" not in allowed and src not in allowed:
                return False, "Forbidden", f"pod with UID {m.uid_of(pod)} specified {field_}, but is disallowed for source {src}"
        if not self.cfg.allow_privileged:
            for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
                if ((c.get("securityContext") or {}).get("privileged")):
                    return False, "Forbidden", f"pod with UID {m.uid_of(pod)} specified privileged container, but is disallowed"
        return True, "", ""

    def _shortfall(self, pod: dict) -> dict[str, int]:
        """What the node lacks to admit `pod` (preemption.go admissionRequirementList)."""
        from .preemption import request
        alloc = node_allocatable(self.node or {})
        others = self.active_pods()
        want = dict(pod_requests(pod))
        want["pods"] = 1
        out = {}
        for k, v in want.items():
            if k in alloc:
                need = sum(request(p, k) for p in others) + v - alloc[k]
                if need > 0:
                    out[k] = need
        return out

    async def _preempt_for(self, pod: dict) -> bool:
        """CriticalPodAdmissionHandler.HandleAdmissionFailure: evict what the critical pod needs."""
        from .preemption import is_critical, pods_to_preempt
        if not self.gates("ExperimentalCriticalPodAnnotation") or not is_critical(pod):
            return False
        try:
            victims = pods_to_preempt(self.active_pods(), self._shortfall(pod))
        except ValueError as e:
            log.warning("cannot preempt for critical pod %s: %s", m.name_of(pod), e)
            return False
        msg = "Preempted in order to admit critical pod"
        for v in victims:
            self.recorder.event(v, "Warning", "Preempting", msg)
            # killPodNow through _evict_kill: terminal first, so a racing sync never restarts it
            await self._evict_kill(v, {"phase": "Failed", "reason": "Preempting", "message": msg},
                                   int((v.get("spec") or {}).get("terminationGracePeriodSeconds", 30)))
        return bool(victims)

    async def _admit(self, pod: dict) -> bool:
        uid = m.uid_of(pod)
        ok, reason, msg = self.can_admit(pod)
        if not ok and reason.startswith("OutOf") and await self._preempt_for(pod):
            ok, reason, msg = self.can_admit(pod)
        if ok:
            try:
                await self.dm.admit_pod(pod)
            except AdmissionError as e:
                ok, reason, msg = False, e.reason, e.message
            except Exception as e:
                ok, reason, msg = False, "UnexpectedAdmissionError", f"device admission failed: {e!r}"
        if ok:
            self.admitted.add(uid)
            self.probes.add_pod(pod)       # HandlePodAdditions: probeManager.AddPod after admission
            POD_TRACE(uid, "admitted")
            return True
        self.rejected[uid] = (reason, msg)
        log.warning("pod %s/%s rejected: %s %s", m.namespace_of(pod), m.name_of(pod), reason, msg)
        self.recorder.event(pod, "Warning", reason, msg)
        st = {"phase": "Failed", "reason": reason, "message": msg, "conditions": (pod.get("status") or {}).get("conditions") or [],
              "startTime": m.now_rfc3339()}
        self.status.set(pod, st)
        return False

    # ============================================================= sync
    def _device_start_done(self, uid: str):
        if uid in self._device_starting:
            self._device_starting.discard(uid)
            self._device_started.add(uid)
            if not self._device_starting:
                self._device_idle.set()

    def _device_start_pause(self, uid: str):
        """Out of the start window without counting as started (the gate re-adds it later)."""
        if uid in self._device_starting:
            self._device_starting.discard(uid)
            if not self._device_starting:
                self._device_idle.set()

    async def _context_holding_device_window(self, uid: str, pod: dict) -> dict:
        """The pod's volumes/env context. A device pod whose volumes take longer than the start
        window (a missing ConfigMap waits up to the mount timeout) stops holding device-less
        pods behind it; the start gate takes it back once its volumes are there."""
        if uid not in self._device_starting:
            return await self._pod_context(pod)
        task = asyncio.ensure_future(self._pod_context(pod))
        try:
            try:
                return await asyncio.wait_for(asyncio.shield(task), self.cfg.device_pod_start_window)
            except asyncio.TimeoutError:
                self._device_start_pause(uid)
                return await task
        finally:
            if not task.done():
                task.cancel()

    @staticmethod
    def _holds_devices(pod: dict) -> bool:
        spec = pod.get("spec") or {}
        if any(er.get("assigned") for er in spec.get("extendedResources") or []):
            return True
        return any("/" in k and not k.startswith(("kubernetes.io/", "hugepages-"))
                   for c in spec.get("containers") or [] for k in ((c.get("resources") or {}).get("limits") or {}))

    async def sync_pod(self, uid: str) -> bool:
        """Returns True when the worker for this pod is finished (pod gone from the node).

        Whatever path a sync takes (rejected, deleted, terminal, waiting on a volume, started),
        it ends the pod's device-start window, so a GPU pod that waits on a missing Secret does
        not hold every device-less pod's first start behind `device_pod_start_window`."""
        try:
            return await self._sync_pod(uid)
        finally:
            self._device_start_done(uid)

    async def _sync_pod(self, uid: str) -> bool:
        pod = self.pods.get(uid)
        if pod is None:
            await self.runtime.kill_and_remove(uid, self._cached_sandboxes(uid))
            self._cleanup(uid)
            return True
        md = pod.get("metadata") or {}
        if uid in self.rejected:
            self._device_start_done(uid)
            if md.get("deletionTimestamp"):
                await self._finalize_delete(pod)
            return False
        if (self.cfg.prioritize_device_pods and uid not in self.admitted and uid not in self._device_started
                and not md.get("deletionTimestamp") and not is_pod_terminal(pod) and self._holds_devices(pod)):
            self._device_starting.add(uid)      # from first sight: its admission counts as its start
            self._device_idle.clear()
        if uid not in self.admitted:
            if is_pod_terminal(pod):
                self.admitted.add(uid)  # e.g. kubelet restart: nothing to run
            elif uid in self._runtime_uids and await self._already_running(uid):
                # kubelet restart: the pod was admitted by the previous incarnation and is running;
                # never kill it because a device plugin has not re-registered yet
                self.admitted.add(uid)
                self.probes.add_pod(pod)
                try:
                    await self.dm.admit_pod(pod)  # refresh plugin annotations, best effort
                except Exception:
                    pass
            elif not await self._admit(pod):
                return False
        if md.get("deletionTimestamp"):
            grace = md.get("deletionGracePeriodSeconds")
            grace = (pod.get("spec") or {}).get("terminationGracePeriodSeconds", 30) if grace is None else grace
            await self.runtime.kill_pod(uid, int(grace), pod)
            self.volume_manager.remove_pod(uid)
            rt = await self.runtime.pod_status(uid)
            st = generate_status(pod, rt, self.cfg.node_ip, {}, [], m.now_rfc3339())
            if st["phase"] == "Running":
                st["phase"] = "Failed" if (pod.get("spec") or {}).get("restartPolicy") != "Always" else "Succeeded"
            self.status.set(pod, st)
            await self._finalize_delete(pod)
            return False
        sent_phase = (self.status.get(uid) or {}).get("phase") or (pod.get("status") or {}).get("phase")
        if sent_phase in ("Succeeded", "Failed"):
            # terminal phases are final (status_manager.go: a terminal pod never goes back); a
            # recomputation must not drop the reason of a kubelet-decided failure (deadline,
            # eviction) that may not be written yet
            await self.runtime.kill_pod(uid, 0, pod, self._cached_sandboxes(uid))
            if not self.cfg.keep_terminated_pod_volumes:
                self.volume_manager.remove_pod(uid)     # terminated: its volumes go (populator findAndRemoveDeletedPods)
            return False
        if sent_phase not in ("Succeeded", "Failed") and self._active_deadline_exceeded(pod):
            # active_deadline.go: the pod sync handler fails the pod once it has been active on
            # the node longer than spec.activeDeadlineSeconds (kubelet.go syncPod kills it)
            msg = "Pod was active on the node longer than the specified deadline"
            self.recorder.event(pod, "Normal", "DeadlineExceeded", msg)
            grace = int((pod.get("spec") or {}).get("terminationGracePeriodSeconds", 30))
            await self.runtime.kill_pod(uid, grace, pod, self._cached_sandboxes(uid))
            rt = await self._cached_status(uid, fresh=True)
            st = generate_status(pod, rt, self.cfg.node_ip, {}, [], m.now_rfc3339())
            st.update({"phase": "Failed", "reason": "DeadlineExceeded", "message": msg})
            self.status.set(pod, st)
            return False
        try:
            ctx = await self._context_holding_device_window(uid, pod)
        except VolumeError as e:
            # kubelet.go syncPod: "Unable to mount volumes for pod": the pod waits in
            # ContainerCreating and the sync is retried
            self.sync_errors[uid] = str(e)
            rt = await self._cached_status(uid)
            st = generate_status(pod, rt, self.cfg.node_ip, self.probes.readiness_of(uid, pod, rt), [], m.now_rfc3339())
            self.status.set(pod, st)
            asyncio.get_running_loop().call_later(2.0, self.dispatch, uid)
            return False
        POD_TRACE(uid, "sync_ctx")
        rt = await self._cached_status(uid)
        mut0 = self.cri.pod_mutations(uid)
        self.cri.take_touched(uid)
        gate = self.cfg.prioritize_device_pods and not rt.sandboxes
        if gate and self._holds_devices(pod):
            if uid not in self._device_started:
                self._device_starting.add(uid)
                self._device_idle.clear()
        elif gate and self._device_starting:
            # accelerator pods first: a pod that holds no device waits (bounded) while pods that
            # hold GPUs are being started, so a burst of mixed pods does not queue the GPU
            # containers behind pause containers in the runtime
            try:
                await asyncio.wait_for(self._device_idle.wait(), self.cfg.device_pod_start_window)
            except asyncio.TimeoutError:
                pass
        try:
            errors = await self.runtime.sync_pod(pod, rt, ctx, self.probes.liveness_failed)
        finally:
            self._device_start_done(uid)
        if self.cri.pod_mutations(uid) != mut0 or errors:
            touched = self.cri.take_touched(uid)
            new_rt = None
            if touched is not None and not errors and self._full_events:
                new_rt = await self._status_from_events(uid, touched)
            rt = new_rt if new_rt is not None else await self._cached_status(uid, fresh=True)
        for sb in rt.sandboxes:
            self._sandbox_uid[sb[0]] = uid
        st = generate_status(pod, rt, self.cfg.node_ip, self.probes.readiness_of(uid, pod, rt), errors, m.now_rfc3339(),
                             self.runtime.reasons.get(uid))
        prev_phase = (self.status.get(uid) or {}).get("phase")
        self.status.set(pod, st)
        if st["phase"] != prev_phase:
            POD_TRACE(uid, "status_" + st["phase"])
        if st["phase"] == "Running" and prev_phase != "Running" and uid in self.first_seen:
            ct = m.parse_time(md.get("creationTimestamp"))
            if ct:
                self.m_pod_start.observe(max(0.0, time.time() - ct) * 1e6)
        if st["phase"] in ("Succeeded", "Failed"):
            # release the sandbox (devices stay API-assigned)
            await self.runtime.kill_pod(uid, 0, pod, self._cached_sandboxes(uid))
            if not self.cfg.keep_terminated_pod_volumes:
                self.volume_manager.remove_pod(uid)
        ads = (pod.get("spec") or {}).get("activeDeadlineSeconds")
        if ads is not None and st["phase"] not in ("Succeeded", "Failed") and uid not in self._deadline_timers:
            start = m.parse_time(st.get("startTime"))
            if start:
                self._deadline_timers.add(uid)
                asyncio.get_running_loop().call_later(max(0.0, start + float(ads) - time.time()) + 0.01, self.dispatch, uid)
        if errors:
            # pod_workers.go: a failed sync is retried after the worker back-off (10 s, jittered)
            import random
            asyncio.get_running_loop().call_later(10.0 * (1 + 0.5 * random.random()), self.dispatch, uid)
        # container restarts waiting on back-off: re-sync when the back-off expires
        for c in (pod.get("spec") or {}).get("containers") or []:
            rem = self.runtime.backoff_remaining(uid, c["name"])
            if rem > 0:
                asyncio.get_running_loop().call_later(rem + 0.05, self.dispatch, uid)
                break
        return False

    def _active_deadline_exceeded(self, pod: dict) -> bool:
        ads = (pod.get("spec") or {}).get("activeDeadlineSeconds")
        if ads is None:
            return False
        start = m.parse_time((self.status.get(m.uid_of(pod)) or {}).get("startTime") or (pod.get("status") or {}).get("startTime"))
        return bool(start) and time.time() - start >= float(ads)

    async def _already_running(self, uid: str) -> bool:
        try:
            rt = await self.runtime.pod_status(uid)
        except Exception:
            return False
        return rt.ready_sandbox() is not None and bool(rt.running())

    async def _finalize_delete(self, pod):
        uid = m.uid_of(pod)
        if uid in self.terminated_deleted:
            return
        await self.status.flush(uid)
        try:
            await self.client.delete("pods", m.name_of(pod), m.namespace_of(pod), grace=0, uid=uid)
            self.terminated_deleted.add(uid)
        except m.StatusError as e:
            if m.is_not_found(e):
                self.terminated_deleted.add(uid)
            else:
                log.warning("final delete of %s failed: %s", m.name_of(pod), e)

    def _on_terminal(self, uid):
        pass

    def _cache_valid(self, uid: str):
        hit = self._rt_cache.get(uid)
        if hit is not None and hit[0] == (self._rt_gen.get(uid, 0), self.cri.pod_mutations(uid)):
            return hit
        return None

    async def _cached_status(self, uid: str, fresh: bool = False):
        """The pod's runtime status: the cache while no mutation/invalidation happened since it
        was filled (events keep it current), otherwise one fetch (1 + sandboxes + containers RPCs)
        with the full-status events newer than the fetch applied on top."""
        hit = self._cache_valid(uid)
        if not fresh and hit is not None:
            return hit[1]
        key = (self._rt_gen.get(uid, 0), self.cri.pod_mutations(uid))
        t0 = time.time_ns()
        pod = self.pods.get(uid)
        if not fresh and uid not in self._rt_cache and self._full_events and pod is not None and \
                uid not in self._runtime_uids:
            # absent from the runtime when this kubelet started and never synced since: the
            # runtime cannot hold anything of it (its sandboxes would come through the event stream)
            from .kuberuntime import PodRuntimeStatus
            rt = PodRuntimeStatus(uid)
        else:
            rt = await self.runtime.pod_status(uid)
        for ev in self._rt_pending.pop(uid, ()):
            if ev.created_at > t0:
                rt = apply_event(rt, ev, self.runtime.sandbox_ips)
        self._rt_cache[uid] = (key, rt, t0)  # key taken before the fetch: a concurrent invalidation wins
        return rt

    def _cached_sandboxes(self, uid: str):
        hit = self._cache_valid(uid)
        return [SandboxRef(x[0], x[1]) for x in hit[1].sandboxes] if hit is not None else None

    def _apply_full_event(self, uid: str, ev):
        for cs in ev.containers_statuses:
            self.cri._cid_sid[cs.id] = ev.pod_sandbox_status.id
        hit = self._cache_valid(uid)
        if hit is not None:
            if ev.created_at > hit[2]:
                self._rt_cache[uid] = (hit[0], apply_event(hit[1], ev, self.runtime.sandbox_ips), max(hit[2], ev.created_at))
        else:
            pend = self._rt_pending.setdefault(uid, [])
            pend.append(ev)
            del pend[:-64]
            w = self._pending_waiters.get(uid)
            if w is not None:
                w.set()

    async def _status_from_events(self, uid: str, touched: dict, timeout: float = 0.25):
        """The pod's status after its own mutations, from the runtime's events instead of a
        re-list. Every mutating CRI call returns (trailer) the created_at of the event that carries
        its sandbox's complete state as of the call's return; each touched sandbox's state is
        taken once that exact event (or a newer one) has arrived, so earlier events of the same
        call (e.g. StopPodSandbox's per-container events that still show the sandbox READY) never
        stand for the final state. Untouched sandboxes keep the cached state; calls that emitted
        nothing (no-ops) need no event. None → the caller re-lists (timeout)."""
        base = self._rt_cache.get(uid)
        if base is None:
            return None
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        while True:
            pend = self._rt_pending.get(uid, ())
            if all(t <= base[2] or any(e.pod_sandbox_status.id == sid and e.created_at >= t for e in pend)
                   for sid, t in touched.items()):
                break
            rem = deadline - loop.time()
            if rem <= 0:
                return None
            w = self._pending_waiters.setdefault(uid, asyncio.Event())
            w.clear()
            try:
                await asyncio.wait_for(w.wait(), rem)
            except asyncio.TimeoutError:
                return None
        key = (self._rt_gen.get(uid, 0), self.cri.pod_mutations(uid))
        rt, t_last = base[1], base[2]
        for e in self._rt_pending.pop(uid, ()):
            if e.created_at > base[2]:
                rt = apply_event(rt, e, self.runtime.sandbox_ips)
                t_last = max(t_last, e.created_at)
        self._pending_waiters.pop(uid, None)
        self._rt_cache[uid] = (key, rt, t_last)
        return rt

    def _pleg_event(self, uid: str):
        self._rt_gen[uid] = self._rt_gen.get(uid, 0) + 1
        self.dispatch(uid)

    def serving_cert(self) -> tuple[str | None, str | None]:
        """The kubelet's HTTPS identity: a rotated server certificate, else --tls-cert-file."""
        scm = self.server_cert_manager
        if scm is not None and scm.current():
            return scm.current_path, scm.current_path
        return self.cfg.tls_cert_file, self.cfg.tls_private_key_file

    def _gpu_numa(self, pod: dict, container: dict) -> set[int]:
        """NUMA nodes of the GPUs assigned to one container (the AMD plugin's amd.com/numa-node
        device attribute): where the CPU manager places its exclusive CPUs."""
        from ..api.helpers import pod_extended_resource_assigned
        out: set[int] = set()
        cap = self.dm.store.capacity if hasattr(self.dm, "store") else {}
        for rname, dom in cap.items():
            for did in pod_extended_resource_assigned(rname, container, pod):
                v = ((dom["resources"].get(did) or {}).get("attributes") or {}).get("amd.com/numa-node")
                if v is not None and str(v).lstrip("-").isdigit() and int(v) >= 0:
                    out.add(int(v))
        return out

    async def cpu_reconcile(self):
        """cpu_manager.go reconcileState: shared-pool containers follow the shared pool as
        exclusive assignments come and go (CRI UpdateContainerResources)."""
        cm = self.cpu_manager
        if self.sources_ready():
            cm.retain_only(set(self.pods) | set(self.workers))
        shared = cm.default_set()
        from .cpumanager import format_cpuset
        want = format_cpuset(shared)
        updated = 0
        for c in await self.cri.list_containers():
            if c.state != C.CONTAINER_RUNNING:
                continue
            uid, name = c.labels.get(L_POD_UID, ""), c.metadata.name
            if not uid or cm.exclusive(uid, name) or self._cpuset_applied.get(c.id) == want:
                continue
            try:
                await self.cri.update_container_resources(c.id, cpuset_cpus=want)
                self._cpuset_applied[c.id] = want
                updated += 1
            except Exception as e:
                log.debug("cpu manager: update of %s failed: %r", c.id, e)
        return updated

    async def _cpu_reconcile_loop(self):
        while True:
            await asyncio.sleep(self.cfg.cpu_manager_reconcile_period)
            try:
                await self.cpu_reconcile()
            except Exception as e:
                log.debug("cpu manager reconcile failed: %r", e)

    def _cleanup(self, uid):
        self._device_start_done(uid)
        self._device_started.discard(uid)
        self._runtime_uids.add(uid)   # the runtime may still hold leftovers: list before trusting the cache again
        self.cpu_manager.release_pod(uid)
        self.volume_manager.remove_pod(uid)
        self._rt_gen.pop(uid, None)
        self._rt_cache.pop(uid, None)
        self._rt_pending.pop(uid, None)
        self._pending_waiters.pop(uid, None)
        self.cri.forget_pod(uid)
        if self.gpu_legacy is not None:
            self.gpu_legacy.release(uid)
        self.admitted.discard(uid)
        self.rejected.pop(uid, None)
        self.status.forget(uid)
        self.probes.remove_pod(uid)
        self.runtime.reasons.pop(uid, None)
        for k in [k for k in self.runtime.pull_backoff if k[0] == uid]:
            del self.runtime.pull_backoff[k]
        self.first_seen.pop(uid, None)
        self.terminated_deleted.discard(uid)
        self.sync_errors.pop(uid, None)
        self._deadline_timers.discard(uid)

    # ---------------------------------------------------- volumes / env context
    async def _pod_context(self, pod: dict) -> dict:
        """Volumes and per-container env and mounts (podcontext.PodContext)."""
        from .podcontext import PodContext
        from .volumemanager import subpath
        pc = PodContext(self)
        vols = await self.volume_manager.wait_for_attach_and_mount(pod)
        spec = pod.get("spec") or {}
        ns = m.namespace_of(pod)
        services = []
        if self.svc_informer is not None:
            services = [s for s in self.svc_informer.list()
                        if m.namespace_of(s) == ns or (m.namespace_of(s) == "default" and m.name_of(s) == "kubernetes")]
        env, mounts = {}, {}
        for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
            env[c["name"]] = await pc.env(pod, c, services)
            mounts[c["name"]] = [{"container_path": vm["mountPath"],
                                  "host_path": subpath(vols[vm["name"]], vm.get("subPath", ""),
                                                       f"container {c['name']} mount {vm['name']}").rstrip("/"),
                                  "read_only": bool(vm.get("readOnly"))} for vm in c.get("volumeMounts") or [] if vm["name"] in vols]
        return {"env": env, "mounts": mounts, "keyring": await self._pull_keyring(pod)}

    async def _pull_keyring(self, pod: dict):
        """Pod imagePullSecrets before the node's docker config (credentialprovider
        MakeDockerKeyring); a missing secret only logs (kubelet_pods.go getPullSecretsForPod)."""
        from .credentialprovider import UnionKeyring, node_keyring, secrets_keyring
        if self._node_keyring is None:
            self._node_keyring = node_keyring(self.cfg.root_dir)
        secrets = []
        for ref in (pod.get("spec") or {}).get("imagePullSecrets") or []:
            s = await self.client.get_or_none("secrets", ref.get("name", ""), m.namespace_of(pod))
            if s is None:
                log.warning("unable to retrieve pull secret %s/%s for %s; the image pull may not succeed",
                            m.namespace_of(pod), ref.get("name"), m.name_of(pod))
            else:
                secrets.append(s)
        return UnionKeyring(secrets_keyring(secrets), self._node_keyring) if secrets else self._node_keyring

    async def _env_from(self, pod, vf) -> str:
        from .podcontext import PodContext
        if "fieldRef" in vf:
            return PodContext(self).field(pod, vf["fieldRef"].get("fieldPath", ""))
        return ""

    # ================================================================ PLEG
    async def _relist_loop(self):
        last = None
        while True:
            await asyncio.sleep(self.cfg.relist_period)
            t0 = time.perf_counter()
            if last is not None:
                self.m_pleg_interval.observe((t0 - last) * 1e6)
            last = t0
            try:
                await self.relist()
            except Exception as e:
                log.debug("relist failed: %r", e)
            self.m_pleg.observe((time.perf_counter() - t0) * 1e6)

    async def relist(self):
        sbs = await self.cri.list_pod_sandbox()
        cur: dict[str, int] = {}
        uids_changed = set()
        running_pods = 0
        for s in sbs:
            uid = s.labels.get(L_POD_UID, "")
            self._sandbox_uid[s.id] = uid
            if s.state == C.SANDBOX_READY:
                running_pods += 1
        conts = await self.cri.list_containers()
        running_c = 0
        owner = {}
        for c in conts:
            cur[c.id] = c.state
            uid = self._sandbox_uid.get(c.pod_sandbox_id) or c.labels.get(L_POD_UID, "")
            owner[c.id] = uid
            if c.state == C.CONTAINER_RUNNING:
                running_c += 1
            if self._pleg_snapshot.get(c.id) != c.state:
                hit = self._cache_valid(uid) if uid else None
                if hit is None or hit[1].container_state(c.id) != c.state:   # events already told us
                    uids_changed.add(uid)
        for cid in set(self._pleg_snapshot) - set(cur):
            uid = self._pleg_owner.get(cid)
            if uid is None:
                self._rt_cache.clear()  # a container vanished and its owner is unknown: drop every cached status
                break
            hit = self._cache_valid(uid)
            if hit is not None and hit[1].container_state(cid) is not None:
                self._rt_gen[uid] = self._rt_gen.get(uid, 0) + 1
        self._pleg_snapshot = cur
        self._pleg_owner = owner
        self.m_running_pods.set(running_pods)
        self.m_running_containers.set(running_c)
        for uid in uids_changed:
            if uid and (uid in self.pods or uid in self.workers):
                self._pleg_event(uid)
        # orphaned sandboxes (pod deleted while the kubelet was down)
        for s in sbs:
            uid = s.labels.get(L_POD_UID, "")
            if uid and uid not in self.pods and uid not in self.workers and self.sources_ready():
                self.dispatch(uid)

    async def _evented_pleg(self):
        backoff = 0.1
        while True:
            try:
                async for ev in self.cri.container_events():
                    backoff = 0.1
                    sst = ev.pod_sandbox_status
                    sid = sst.id
                    full = bool(sst.metadata.uid)   # the runtime sends complete pod state (KEP-3386)
                    if full:
                        self._sandbox_uid[sid] = sst.metadata.uid
                        self._full_events = True
                    uid = self._sandbox_uid.get(sid)
                    if uid is None:
                        for s in await self.cri.list_pod_sandbox():
                            self._sandbox_uid[s.id] = s.labels.get(L_POD_UID, "")
                        uid = self._sandbox_uid.get(sid)
                    if not uid:
                        continue
                    if full:
                        self._apply_full_event(uid, ev)
                    if ev.container_event_type in (C.CONTAINER_STOPPED_EVENT, C.CONTAINER_STARTED_EVENT) and ev.container_id != sid:
                        if uid in self.pods or uid in self.workers:
                            if full:
                                self.dispatch(uid)     # the cache already holds the new state
                            else:
                                self._pleg_event(uid)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.debug("container event stream ended: %r", e)
            await asyncio.sleep(backoff)
            backoff = min(2.0, backoff * 2)

    async def container_gc(self) -> dict:
        """One pass of the container/sandbox garbage collector (active pods keep their newest
        dead container per container name for logs and restart accounting)."""
        active = lambda uid: (uid in self.pods or uid in self.workers) and uid not in self.terminated_deleted   # noqa: E731
        return await self.runtime.garbage_collect(active, self.cfg.maximum_dead_containers_per_container,
                                                  self.cfg.maximum_dead_containers, self.cfg.minimum_container_ttl_duration,
                                                  sources_ready=self.sources_ready(),
                                                  has_volumes=self.volume_manager.has_mounts)

    def sources_ready(self) -> bool:
        """config.SourcesReady.AllReady: every configured pod source has delivered its first
        complete set (the API informer synced; --pod-manifest-path read once). Until then a pod
        the kubelet does not know may simply not have been seen yet."""
        api = self.informer is not None and self.informer.has_synced()
        return api and (not (self.cfg.pod_manifest_path or self.cfg.manifest_url) or self._static_read)

    async def _gc_loop(self):
        last_image_gc = time.monotonic()
        while True:
            await asyncio.sleep(min(self.cfg.gc_period, self.cfg.image_gc_period))
            try:
                await self.container_gc()
            except Exception as e:
                log.debug("container GC failed: %r", e)
            if time.monotonic() - last_image_gc >= self.cfg.image_gc_period:
                last_image_gc = time.monotonic()
                try:
                    await self.image_gc.garbage_collect()
                except Exception as e:
                    log.debug("image GC failed: %r", e)

    async def _housekeeping(self):
        """Periodic resync (syncFrequency) of every pod; keeps the sync loop health probe fresh."""
        while True:
            await asyncio.sleep(self.cfg.sync_frequency)
            for uid in list(self.pods):
                self._pleg_event(uid)  # periodic resync re-reads the runtime (never trusts the cache)
            self.last_sync_loop = time.time()

    # ================================================================ probes
    async def _probe_exec(self, cid: str, cmd: list, timeout: float):
        """The prober's exec runner (RunInContainer): combined output and exit status."""
        out, err, code = await self.cri.exec_sync(cid.split("://", 1)[-1], cmd, max(1, int(timeout)))
        text = b"".join(x if isinstance(x, bytes) else (x or "").encode() for x in (out, err))
        return text.decode(errors="replace"), code

    # ================================================================ eviction
    async def _eviction_loop(self):
        while True:
            await asyncio.sleep(self.cfg.eviction_interval)
            try:
                await self.eviction_pass()
            except Exception as e:
                log.debug("eviction pass failed: %r", e)

    async def eviction_pass(self):
        """One synchronize() of the eviction manager (eviction_manager.go:199-371); the node
        conditions it holds feed the next node status."""
        evicted = await self.eviction.synchronize(self._has_dedicated_image_fs, self.active_pods,
                                                  self._eviction_capacity())
        pressure = self.eviction.conditions
        if pressure != self.pressure:
            self.pressure = pressure
            self._node_dirty.set()
        return evicted[0] if evicted else None

    async def _evict_kill(self, pod: dict, status: dict, grace: int):
        """killPodNow: the pod turns Failed/Evicted first (a sync racing the kill sees a terminal
        pod and never restarts its containers), then its containers stop with `grace`."""
        self.status.set(pod, {**status, "conditions": (pod.get("status") or {}).get("conditions") or []})
        await self.runtime.kill_pod(m.uid_of(pod), grace, pod)

    async def _has_dedicated_image_fs(self) -> bool:
        """DiskInfoProvider.HasDedicatedImageFs: the runtime's image filesystem is a different
        device from the kubelet's root directory."""
        try:
            fsu = (await self.cri.image_fs_info())[0]
            path = fsu.storage_id.uuid
            root = self.cfg.root_dir if os.path.isdir(self.cfg.root_dir) else "/"
            return bool(path) and os.path.exists(path) and os.stat(path).st_dev != os.stat(root).st_dev
        except Exception:
            return False

    def _eviction_capacity(self):
        """CapacityProvider: node memory capacity and the node-allocatable reservation
        (kube + system reserved + hard eviction, cm GetNodeAllocatableReservation)."""
        from .cm import hard_eviction_reservation
        from .eviction import CapacityProvider
        from ..api.quantity import Quantity
        cap = {k: Quantity(v).value() for k, v in self._capacity().items() if k in ("memory", "ephemeral-storage")}
        ev = hard_eviction_reservation([t for t in self.eviction.thresholds if t.hard], cap)
        res = {k: self._kube_reserved.get(k, 0) + self._system_reserved.get(k, 0) + ev.get(k, 0) for k in cap}
        return CapacityProvider(cap, res)
