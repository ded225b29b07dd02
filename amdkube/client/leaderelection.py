"""Leader election on a resource lock (Endpoints / ConfigMap / Lease annotation).

Reference: staging/src/k8s.io/client-go/tools/leaderelection/leaderelection.go:138
(Run → acquire → renew), :152 (acquire loop with RetryPeriod jitter), the
LeaderElectionRecord JSON in the `control-plane.alpha.kubernetes.io/leader` annotation
(resourcelock/interface.go), used by scheduler/controller-manager
(plugin/cmd/kube-scheduler/app/server.go:600-626). Defaults: lease 15s, renew 10s, retry 2s.
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import time

from ..api import meta as m
from .rest import Client

log = logging.getLogger("amdkube.leaderelection")
ANNOTATION = "control-plane.alpha.kubernetes.io/leader"


def _ts(t: float) -> str:
    # microsecond resolution: every renew must change the record, or followers with a short
    # lease would mistake an unchanged (same-second) record for a dead leader
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + f".{int((t % 1) * 1e6):06d}Z"


class LeaderElector:
    def __init__(self, client: Client, name: str, identity: str, ns: str = "kube-system", lock_kind: str = "endpoints",
                 lease_duration: float = 15.0, renew_deadline: float = 10.0, retry_period: float = 2.0):
        self.client, self.name, self.identity, self.ns = client, name, identity, ns
        self.lock_kind = lock_kind
        self.lease, self.renew_deadline, self.retry = lease_duration, renew_deadline, retry_period
        self.observed: dict | None = None
        self.observed_time = 0.0
        self.is_leader = False

    async def _get(self):
        return await self.client.get_or_none(self.lock_kind, self.name, self.ns)

    async def try_acquire_or_renew(self) -> bool:
        now = time.time()
        rec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease), "acquireTime": _ts(now),
               "renewTime": _ts(now), "leaderTransitions": 0}
        obj = await self._get()
        if obj is None:
            kind = {"endpoints": "Endpoints", "configmaps": "ConfigMap", "leases": "Lease"}[self.lock_kind]
            api = "coordination.k8s.io/v1" if kind == "Lease" else "v1"
            try:
                await self.client.create({"apiVersion": api, "kind": kind,
                                          "metadata": {"name": self.name, "namespace": self.ns,
                                                       "annotations": {ANNOTATION: json.dumps(rec)}}})
            except m.StatusError:
                return False
            self.observed, self.observed_time = rec, now
            return True
        cur = json.loads(m.annotations_of(obj).get(ANNOTATION, "{}") or "{}")
        if cur != self.observed:
            self.observed, self.observed_time = cur, now
        holder = cur.get("holderIdentity")
        # like client-go, the observer's own LeaseDuration decides expiry (leaderelection.go:152+)
        if holder and holder != self.identity and self.observed_time + self.lease > now:
            return False
        if holder == self.identity:
            rec["acquireTime"] = cur.get("acquireTime", rec["acquireTime"])
            rec["leaderTransitions"] = cur.get("leaderTransitions", 0)
        else:
            rec["leaderTransitions"] = cur.get("leaderTransitions", 0) + 1
        obj.setdefault("metadata", {}).setdefault("annotations", {})[ANNOTATION] = json.dumps(rec)
        try:
            await self.client.update(obj)
        except m.StatusError:
            return False
        self.observed, self.observed_time = rec, now
        return True

    async def run(self, on_started, on_stopped=None):
        """Block until leadership is acquired, run on_started() (a coroutine) while renewing."""
        while not await self._safe_try():
            await asyncio.sleep(self.retry * (1 + random.random() * 0.2))
        self.is_leader = True
        log.info("%s became leader for %s/%s", self.identity, self.ns, self.name)
        work = asyncio.create_task(on_started())
        try:
            last_renew = time.time()
            while not work.done():
                await asyncio.sleep(self.retry)
                if await self._safe_try():
                    last_renew = time.time()
                elif time.time() - last_renew > self.renew_deadline:
                    log.warning("%s lost leadership", self.identity)
                    break
        finally:
            self.is_leader = False
            if not work.done():
                work.cancel()
            if on_stopped:
                on_stopped()

    async def _safe_try(self):
        try:
            return await self.try_acquire_or_renew()
        except Exception as e:
            log.debug("leader election attempt failed: %r", e)
            return False
