"""cluster-proportional-autoscaler: scale a workload with the size of the cluster.

What cluster/addons/dns-horizontal-autoscaler/dns-horizontal-autoscaler.yaml runs against
kube-dns (the upstream kubernetes-incubator/cluster-proportional-autoscaler 1.1 image, flags
--namespace / --configmap / --target / --default-params). Every poll period:
* the cluster status: all nodes and cores (node capacity cpu, rounded up to whole cores), and
  the schedulable ones (spec.unschedulable unset) — the controllers size on the schedulable
  numbers unless `includeUnschedulableNodes`;
* the parameters: the ConfigMap's single `linear` or `ladder` key (JSON). A missing ConfigMap is
  created from --default-params; a ConfigMap that does not parse keeps the last good params;
* linear: max(ceil(cores / coresPerReplica), ceil(nodes / nodesPerReplica)), each clamped to
  [min, max] (a zero ratio gives 1), with at least 2 from the node term when
  `preventSinglePointFailure` and more than one node;
* ladder: for cores and for nodes the replicas of the last step whose threshold the count
  reaches (1 below the first step), the larger of the two;
* the target's scale subresource is read and, when it differs, updated.
MI355X extension: `gpusPerReplica` (linear) and `gpusToReplicas` (ladder) size on the cluster's
amd.com/gpu capacity as a third term, for services whose load follows accelerator count.
"""
from __future__ import annotations

import asyncio
import json
import logging
import math

from ..api import meta as m
from ..api.quantity import Quantity

log = logging.getLogger("amdkube.cluster-proportional-autoscaler")

GPU_RESOURCE = "amd.com/gpu"
TARGET_KINDS = {"deployment": "deployments", "replicationcontroller": "replicationcontrollers",
                "replicaset": "replicasets"}


class ParamsError(ValueError):
    pass


def cluster_status(nodes: list) -> dict:
    st = {"total_nodes": 0, "total_cores": 0, "total_gpus": 0,
          "schedulable_nodes": 0, "schedulable_cores": 0, "schedulable_gpus": 0}
    for n in nodes:
        cap = (n.get("status") or {}).get("capacity") or {}
        cores = math.ceil(Quantity(cap.get("cpu", "0")).as_fraction())
        gpus = int(Quantity(cap.get(GPU_RESOURCE, "0")).value())
        st["total_nodes"] += 1
        st["total_cores"] += cores
        st["total_gpus"] += gpus
        if not (n.get("spec") or {}).get("unschedulable"):
            st["schedulable_nodes"] += 1
            st["schedulable_cores"] += cores
            st["schedulable_gpus"] += gpus
    return st


def _counts(status: dict, include_unschedulable: bool):
    pre = "total" if include_unschedulable else "schedulable"
    return status[f"{pre}_cores"], status[f"{pre}_nodes"], status[f"{pre}_gpus"]


class Linear:
    def __init__(self, p: dict):
        self.cores = float(p.get("coresPerReplica", 0) or 0)
        self.nodes = float(p.get("nodesPerReplica", 0) or 0)
        self.gpus = float(p.get("gpusPerReplica", 0) or 0)
        self.min, self.max = int(p.get("min", 0) or 0), int(p.get("max", 0) or 0)
        self.spof = bool(p.get("preventSinglePointFailure", False))
        self.include_unschedulable = bool(p.get("includeUnschedulableNodes", False))
        if self.cores < 0 or self.nodes < 0 or self.gpus < 0:
            raise ParamsError("coresPerReplica, nodesPerReplica and gpusPerReplica may not be negative")
        if self.cores == 0 and self.nodes == 0 and self.gpus == 0:
            raise ParamsError("at least one of coresPerReplica and nodesPerReplica must be set")
        if self.min < 0 or self.max < 0 or (self.max and self.min > self.max):
            raise ParamsError(f"invalid min/max: {self.min}/{self.max}")

    def _from(self, amount: int, per: float) -> int:
        if per == 0:
            return 1
        res = math.ceil(amount / per)
        if self.max:
            res = min(self.max, res)
        return max(self.min, res)

    def replicas(self, status: dict) -> int:
        cores, nodes, gpus = _counts(status, self.include_unschedulable)
        from_cores, from_nodes = self._from(cores, self.cores), self._from(nodes, self.nodes)
        if self.spof and nodes > 1 and from_nodes < 2:
            from_nodes = 2
        out = max(from_cores, from_nodes)
        if self.gpus:
            out = max(out, self._from(gpus, self.gpus))
        return out


class Ladder:
    def __init__(self, p: dict):
        self.include_unschedulable = bool(p.get("includeUnschedulableNodes", False))
        self.maps = {}
        for key in ("coresToReplicas", "nodesToReplicas", "gpusToReplicas"):
            entries = p.get(key) or []
            norm = []
            for e in entries:
                if not isinstance(e, list) or len(e) != 2 or not all(isinstance(x, int) and x >= 0 for x in e):
                    raise ParamsError(f"{key}: every step is a [threshold, replicas] pair of non-negative integers")
                norm.append((e[0], e[1]))
            self.maps[key] = sorted(norm)
        if not self.maps["coresToReplicas"] and not self.maps["nodesToReplicas"]:
            raise ParamsError("either coresToReplicas or nodesToReplicas must be set")

    @staticmethod
    def _step(amount: int, steps) -> int:
        replicas = 1
        for threshold, r in steps:
            if amount < threshold:
                break
            replicas = r
        return replicas

    def replicas(self, status: dict) -> int:
        cores, nodes, gpus = _counts(status, self.include_unschedulable)
        out = max(self._step(cores, self.maps["coresToReplicas"]), self._step(nodes, self.maps["nodesToReplicas"]))
        if self.maps["gpusToReplicas"]:
            out = max(out, self._step(gpus, self.maps["gpusToReplicas"]))
        return out


def parse_params(data: dict):
    """The ConfigMap's data: exactly one of `linear` / `ladder`, a JSON object."""
    keys = [k for k in ("linear", "ladder") if k in (data or {})]
    if len(keys) != 1:
        raise ParamsError(f"the ConfigMap needs exactly one of linear, ladder (has {sorted(data or {})})")
    try:
        p = json.loads(data[keys[0]])
    except ValueError as e:
        raise ParamsError(f"{keys[0]}: {e}") from e
    if not isinstance(p, dict):
        raise ParamsError(f"{keys[0]}: not a JSON object")
    return (Linear if keys[0] == "linear" else Ladder)(p)


def parse_target(target: str) -> tuple[str, str]:
    kind, _, name = target.partition("/")
    resource = TARGET_KINDS.get(kind.lower())
    if resource is None or not name:
        raise ValueError(f"--target {target!r}: expected <Deployment|ReplicationController|ReplicaSet>/<name>")
    return resource, name


class ProportionalAutoscaler:
    def __init__(self, client, namespace: str, configmap: str, target: str, default_params: str = "",
                 poll_period: float = 10.0):
        self.client, self.namespace, self.configmap = client, namespace, configmap
        self.resource, self.target = parse_target(target)
        self.default_params = json.loads(default_params) if default_params else None
        if self.default_params is not None:
            parse_params({k: json.dumps(v) for k, v in self.default_params.items()})     # fail at start, not later
        self.poll_period = poll_period
        self.controller = None
        self._cm_version = None

    async def _params(self):
        cm = await self.client.get_or_none("configmaps", self.configmap, self.namespace)
        if cm is None:
            if self.default_params is None:
                raise ParamsError(f"ConfigMap {self.namespace}/{self.configmap} not found and no --default-params")
            cm = await self.client.create({"apiVersion": "v1", "kind": "ConfigMap",
                                           "metadata": {"name": self.configmap, "namespace": self.namespace},
                                           "data": {k: json.dumps(v) for k, v in self.default_params.items()}},
                                          self.namespace)
            log.info("created ConfigMap %s/%s from the default params", self.namespace, self.configmap)
        rv = (cm.get("metadata") or {}).get("resourceVersion")
        if rv != self._cm_version or self.controller is None:
            try:
                self.controller = parse_params(cm.get("data") or {})
                self._cm_version = rv
            except ParamsError as e:
                if self.controller is None:
                    raise
                log.warning("ConfigMap %s/%s: %s; keeping the previous params", self.namespace, self.configmap, e)
        return self.controller

    async def poll_once(self) -> int | None:
        """One poll; the replica count written, or None when the target already has it."""
        ctrl = await self._params()
        nodes, _ = await self.client.list("nodes")
        want = ctrl.replicas(cluster_status(nodes))
        ri = self.client.resource_info(self.resource)
        path = self.client.path(ri, self.namespace, self.target, "scale")
        scale = await self.client.request("GET", path)
        if int((scale.get("spec") or {}).get("replicas", 0)) == want:
            return None
        scale.setdefault("spec", {})["replicas"] = want
        await self.client.request("PUT", path, body=scale)
        log.info("scaled %s/%s/%s to %d replicas", self.resource, self.namespace, self.target, want)
        return want

    async def run(self, stop: asyncio.Event | None = None):
        stop = stop or asyncio.Event()
        while not stop.is_set():
            try:
                await self.poll_once()
            except (m.StatusError, ParamsError, OSError) as e:
                log.error("poll: %s", e)
            try:
                await asyncio.wait_for(stop.wait(), self.poll_period)
            except asyncio.TimeoutError:
                pass
