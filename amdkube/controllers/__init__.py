"""kube-controller-manager equivalent (reference cmd/kube-controller-manager/app/
controllermanager.go:332-363 lists ~30 controllers; amdkube runs the ones the GPU-pod
path needs: node lifecycle, ReplicaSet, Deployment, DaemonSet, Job, Namespace, garbage
collector and pod GC — SURVEY U20/U21)."""
from __future__ import annotations

import asyncio

from ..client import Client, LeaderElector, SharedInformerFactory
from .lifecycle import GarbageCollector, NamespaceController, NodeLifecycleController, PodGCController
from .networking import EndpointsController, NodeIPAMController
from .workloads import DaemonSetController, DeploymentController, JobController, ReplicaSetController

ALL = {"nodelifecycle": NodeLifecycleController, "replicaset": ReplicaSetController, "deployment": DeploymentController,
       "daemonset": DaemonSetController, "job": JobController, "namespace": NamespaceController,
       "garbagecollector": GarbageCollector, "podgc": PodGCController, "endpoint": EndpointsController,
       "nodeipam": NodeIPAMController}
# controllers the reference starts only when asked (--allocate-node-cidrs for node IPAM)
OPT_IN = {"nodeipam"}


class ControllerManager:
    def __init__(self, client: Client, controllers=None, leader_elect: bool = False, identity: str = "controller-manager",
                 node_monitor_grace: float = 40.0, pod_eviction_timeout: float = 300.0, cluster_cidr: str = "10.244.0.0/16",
                 node_cidr_mask_size: int = 24, allocate_node_cidrs: bool = False):
        self.client = client
        self.factory = SharedInformerFactory(client)
        self.pods = self.factory.informer("pods")
        self.nodes = self.factory.informer("nodes")
        names = controllers or [n for n in ALL if n not in OPT_IN or (n == "nodeipam" and allocate_node_cidrs)]
        self.controllers = []
        for n in names:
            cls = ALL[n]
            if cls is NodeLifecycleController:
                self.controllers.append(cls(self, grace=node_monitor_grace, eviction_timeout=pod_eviction_timeout))
            elif cls is NodeIPAMController:
                self.controllers.append(cls(self, cluster_cidr, node_cidr_mask_size))
            else:
                self.controllers.append(cls(self))
        self.leader_elect = leader_elect
        self.identity = identity
        self._task = None

    async def _run(self):
        for c in self.controllers:
            c.setup()
        self.factory.start()
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
        await self.factory.stop()

    def get(self, name):
        for c in self.controllers:
            if c.name == name or c.name.replace("-", "") == name:
                return c
        return None
