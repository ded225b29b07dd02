"""kube-controller-manager equivalent.

Reference cmd/kube-controller-manager/app/controllermanager.go:332-363
(NewControllerInitializers). Every controller the reference registers has a counterpart
here under the same name, except `nodelifecycle`, which is the reference's `node`:
  endpoint, replicationcontroller, podgc, resourcequota, namespace, serviceaccount,
  serviceaccount-token, garbagecollector, daemonset, job, deployment, replicaset,
  horizontalpodautoscaling, disruption, statefulset, cronjob, csrsigning, csrapproving,
  csrcleaner, ttl, bootstrapsigner, tokencleaner, service, nodelifecycle, nodeipam,
  route, persistentvolume-binder, attachdetach, persistentvolume-expander,
  clusterrole-aggregation, pvc-protection, pv-protection.
As in the reference, some are off by default:
  * bootstrapsigner and tokencleaner (`--controllers=*,bootstrapsigner,tokencleaner`);
  * nodeipam, which needs --allocate-node-cidrs;
  * service and route, which need a --cloud-provider (route also needs --configure-cloud-routes).
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass, field

from ..client import Client, EventRecorder, LeaderElector, SharedInformerFactory
from .accounts import (BootstrapSignerController, CSRApprovingController, CSRCleanerController, CSRSigningController,
                       GroupCSRApprovingController, WebhookSigningController,
                       ServiceAccountsController, TokenCleanerController, TokensController)
from .apps import CronJobController, ReplicationManager, StatefulSetController
from .autoscaling import HorizontalPodAutoscalerController
from .cloud import CloudNodeController, PersistentVolumeLabelController, RouteController, ServiceLBController
from .garbagecollector import GarbageCollector
from .lifecycle import NamespaceController, NodeLifecycleController, PodGCController
from .networking import EndpointsController, NodeIPAMController
from .policy import ClusterRoleAggregationController, DisruptionController, ResourceQuotaController, TTLController
from .volumes import (AttachDetachController, PersistentVolumeBinderController, PVCProtectionController,
                      PVProtectionController, VolumeExpandController)
from .daemonset import DaemonSetController
from .deployment import DeploymentController
from .job import JobController
from .replicaset import ReplicaSetController


@dataclass
class Options:
    """kube-controller-manager flags that shape individual controllers."""
    node_monitor_grace: float = 40.0
    pod_eviction_timeout: float = 300.0
    cluster_cidr: str = "10.244.0.0/16"
    node_cidr_mask_size: int = 24
    allocate_node_cidrs: bool = False
    configure_cloud_routes: bool = True
    cloud: object = None
    cluster_name: str = "kubernetes"
    service_account_key: bytes | None = None
    root_ca: bytes = b""
    cluster_signing_cert_file: str | None = None
    cluster_signing_key_file: str | None = None
    hostpath_pv_root: str = "/tmp/amdkube-hostpath-pv"
    hpa_sync_period: float = 30.0
    hpa_upscale_delay: float = 180.0
    hpa_downscale_delay: float = 300.0
    hpa_metrics: object = None
    node_monitor_period: float = 5.0              # --node-monitor-period
    node_startup_grace: float = 60.0              # --node-startup-grace-period
    node_eviction_rate: float = 0.1               # --node-eviction-rate (nodes/s per zone)
    secondary_node_eviction_rate: float = 0.01    # --secondary-node-eviction-rate
    unhealthy_zone_threshold: float = 0.55        # --unhealthy-zone-threshold
    large_cluster_size_threshold: int = 50        # --large-cluster-size-threshold
    enable_taint_manager: bool = True             # --enable-taint-manager
    taint_based_evictions: bool = True            # --feature-gates TaintBasedEvictions
    terminated_pod_gc_threshold: int = 12500      # --terminated-pod-gc-threshold
    extra: dict = field(default_factory=dict)


ALL = {
    "nodelifecycle": lambda mgr, o: NodeLifecycleController(
        mgr, grace=o.node_monitor_grace, eviction_timeout=o.pod_eviction_timeout, period=o.node_monitor_period,
        startup_grace=o.node_startup_grace, eviction_rate=o.node_eviction_rate,
        secondary_eviction_rate=o.secondary_node_eviction_rate, unhealthy_zone_threshold=o.unhealthy_zone_threshold,
        large_cluster_threshold=o.large_cluster_size_threshold, enable_taint_manager=o.enable_taint_manager,
        taint_based_evictions=o.taint_based_evictions),
    "replicaset": lambda mgr, o: ReplicaSetController(mgr),
    "deployment": lambda mgr, o: DeploymentController(mgr),
    "daemonset": lambda mgr, o: DaemonSetController(mgr),
    "job": lambda mgr, o: JobController(mgr),
    "namespace": lambda mgr, o: NamespaceController(mgr),
    "garbagecollector": lambda mgr, o: GarbageCollector(mgr, sync_period=o.extra.get("gc_discovery_period", 30.0)),
    "podgc": lambda mgr, o: PodGCController(mgr, threshold=o.terminated_pod_gc_threshold),
    "endpoint": lambda mgr, o: EndpointsController(mgr),
    "nodeipam": lambda mgr, o: NodeIPAMController(mgr, o.cluster_cidr, o.node_cidr_mask_size),
    "replicationcontroller": lambda mgr, o: ReplicationManager(mgr),
    "statefulset": lambda mgr, o: StatefulSetController(mgr),
    "cronjob": lambda mgr, o: CronJobController(mgr),
    "disruption": lambda mgr, o: DisruptionController(mgr),
    "resourcequota": lambda mgr, o: ResourceQuotaController(mgr),
    "ttl": lambda mgr, o: TTLController(mgr),
    "clusterrole-aggregation": lambda mgr, o: ClusterRoleAggregationController(mgr),
    "serviceaccount": lambda mgr, o: ServiceAccountsController(mgr),
    "serviceaccount-token": lambda mgr, o: TokensController(mgr, o.service_account_key, o.root_ca),
    "csrapproving": lambda mgr, o: CSRApprovingController(mgr),
    "csrsigning": lambda mgr, o: CSRSigningController(mgr, o.cluster_signing_cert_file, o.cluster_signing_key_file),
    "csrcleaner": lambda mgr, o: CSRCleanerController(mgr),
    "bootstrapsigner": lambda mgr, o: BootstrapSignerController(mgr),
    "tokencleaner": lambda mgr, o: TokenCleanerController(mgr),
    "horizontalpodautoscaling": lambda mgr, o: HorizontalPodAutoscalerController(
        mgr, o.hpa_metrics, o.hpa_sync_period, o.hpa_upscale_delay, o.hpa_downscale_delay),
    "persistentvolume-binder": lambda mgr, o: PersistentVolumeBinderController(mgr, o.hostpath_pv_root),
    "attachdetach": lambda mgr, o: AttachDetachController(mgr),
    "persistentvolume-expander": lambda mgr, o: VolumeExpandController(mgr),
    "pvc-protection": lambda mgr, o: PVCProtectionController(mgr),
    "pv-protection": lambda mgr, o: PVProtectionController(mgr),
    "service": lambda mgr, o: ServiceLBController(mgr, o.cloud, o.cluster_name),
    "route": lambda mgr, o: RouteController(mgr, o.cloud, o.cluster_name, o.cluster_cidr),
    # cloud-controller-manager only (cmd/cloud-controller-manager/app/controllermanager.go)
    "cloud-node": lambda mgr, o: CloudNodeController(mgr, o.cloud, o.extra.get("node_status_update_frequency", 300.0),
                                                     o.extra.get("node_monitor_period", 5.0)),
    "persistentvolume-labeler": lambda mgr, o: PersistentVolumeLabelController(mgr, o.cloud),
    # gke-certificates-controller only (cmd/gke-certificates-controller/app)
    "csrsigning-webhook": lambda mgr, o: WebhookSigningController(mgr, o.extra["signing_kubeconfig"],
                                                                  o.extra.get("signing_retry_backoff", 0.5)),
    "csrapproving-group": lambda mgr, o: GroupCSRApprovingController(mgr, o.extra["approve_group"]),
}
DISABLED_BY_DEFAULT = {"bootstrapsigner", "tokencleaner"}
CLOUD_CONTROLLERS = ["cloud-node", "service", "route", "persistentvolume-labeler"]
OPT_IN = DISABLED_BY_DEFAULT | {"nodeipam", "service", "route", "cloud-node", "persistentvolume-labeler",
                                "csrsigning-webhook", "csrapproving-group"}


def default_controllers(opts: Options) -> list[str]:
    names = [n for n in ALL if n not in OPT_IN]
    if opts.allocate_node_cidrs:
        names.append("nodeipam")
    if opts.cloud is not None:
        names.append("service")
        if opts.allocate_node_cidrs and opts.configure_cloud_routes:
            names.append("route")
    return names


def resolve_controllers(spec: str, opts: Options) -> list[str]:
    """--controllers: '*' enables the defaults, 'foo' enables foo, '-foo' disables foo."""
    items = [s.strip() for s in (spec or "*").split(",") if s.strip()]
    names = default_controllers(opts) if "*" in items else []
    for it in items:
        if it == "*":
            continue
        if it.startswith("-"):
            names = [n for n in names if n != it[1:]]
        elif it not in names:
            if it not in ALL:
                raise ValueError(f"unknown controller {it!r}")
            names.append(it)
    return names


class ControllerManager:
    def __init__(self, client: Client, controllers=None, leader_elect: bool = False, identity: str = "controller-manager",
                 node_monitor_grace: float = 40.0, pod_eviction_timeout: float = 300.0, cluster_cidr: str = "10.244.0.0/16",
                 node_cidr_mask_size: int = 24, allocate_node_cidrs: bool = False, options: Options | None = None, **kw):
        self.client = client
        self.opts = options or Options(node_monitor_grace=node_monitor_grace, pod_eviction_timeout=pod_eviction_timeout,
                                       cluster_cidr=cluster_cidr, node_cidr_mask_size=node_cidr_mask_size,
                                       allocate_node_cidrs=allocate_node_cidrs, **kw)
        if self.opts.cloud is not None and hasattr(self.opts.cloud, "initialize"):
            self.opts.cloud.initialize(client)
        self.factory = SharedInformerFactory(client)
        self.pods = self.factory.informer("pods")
        self.nodes = self.factory.informer("nodes")
        self.recorder = EventRecorder(client, "controller-manager")
        names = controllers or default_controllers(self.opts)
        self.controllers = [ALL[n](self, self.opts) for n in names]
        self.leader_elect = leader_elect
        self.identity = identity
        self._task = None

    async def _run(self):
        for c in self.controllers:
            c.setup()
        self.factory.start()
        self.recorder.start()
        await self.factory.wait_for_cache_sync(30)
        for c in self.controllers:
            await c.start()

    async def start(self):
        if self.leader_elect:
            le = LeaderElector(self.client, "kube-controller-manager", self.identity)

            async def hold():
                await self._run()
                await asyncio.Event().wait()
            self._task = asyncio.create_task(le.run(hold))
        else:
            await self._run()
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
        for c in self.controllers:
            await c.stop()
        await self.recorder.stop()
        await self.factory.stop()

    def get(self, name):
        for c in self.controllers:
            if c.name == name or c.name.replace("-", "") == name:
                return c
        return None
