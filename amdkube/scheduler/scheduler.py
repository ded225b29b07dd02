"""kube-scheduler equivalent: watch → queue → schedule → assume (with devices) → async bind.

Reference: plugin/pkg/scheduler/scheduler.go:170-180 (Run: scheduleOne loop), :430-497
(scheduleOne: schedule, assume, bind in a goroutine; the fork puts the chosen device IDs into
Binding.Target.ExtendedResources at :483-491), :194/:425 (FailedScheduling / Scheduled
events); factory/factory.go:554-830 (informer handlers: unscheduled pods → queue, assigned
non-terminated pods → cache, node events → cache + MoveAllToActiveQueue); metrics
plugin/pkg/scheduler/metrics/metrics.go:34-50; policy file & algorithm providers
(plugin/cmd/kube-scheduler/app/server.go:218-290, algorithmprovider/defaults).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from aiohttp import web

from ..utils.trace import POD_TRACE
from ..api import meta as m
from ..api.helpers import is_pod_terminal
from ..client import Client, EventRecorder, Informer, LeaderElector
from ..utils import profiling
from ..utils.features import FeatureGate
from ..utils.metrics import CONTENT_TYPE, MICRO_BUCKETS, Counter, Histogram, new_registry, render
from .cache import SchedulerCache
from .extender import HTTPExtender
from .generic import FitError, GenericScheduler
from .predicates import DEFAULT_PREDICATES
from .priorities import DEFAULT_PRIORITIES
from .queue import NOMINATED_NODE_ANNOTATION, SchedulingQueue
log = logging.getLogger("amdkube.scheduler")

PROVIDERS = {
    "DefaultProvider": (DEFAULT_PREDICATES, DEFAULT_PRIORITIES),
    "ClusterAutoscalerProvider": (DEFAULT_PREDICATES, {**{k: v for k, v in DEFAULT_PRIORITIES.items() if k != "LeastRequestedPriority"},
                                                       "MostRequestedPriority": 1}),
}


def read_policy(path_or_dict) -> dict:
    if isinstance(path_or_dict, str):
        with open(path_or_dict) as f:
            return json.load(f)
    return path_or_dict


def load_policy(path_or_dict) -> tuple[list, dict, list]:
    from .policy_args import build
    pol = read_policy(path_or_dict)
    preds, prios, _, _ = build(pol)
    return preds, prios, list(pol.get("extenders") or [])


class Scheduler:
    def __init__(self, client: Client, scheduler_name: str = "default-scheduler", policy=None,
                 algorithm_provider: str = "DefaultProvider", feature_gates: str = "", leader_elect: bool = False,
                 identity: str | None = None, port: int | None = None, disable_preemption: bool = False,
                 bind_concurrency: int = 256, hard_pod_affinity_weight: int = 1, lock_object_name: str = "kube-scheduler",
                 lock_object_namespace: str = "kube-system", address: str = "127.0.0.1",
                 policy_configmap: tuple[str, str] | None = None):
        """policy: a Policy file path or dict (--policy-config-file); policy_configmap: (namespace,
        name) of a ConfigMap whose `policy.cfg` holds it (--policy-configmap), read at start."""
        self.client = client
        self.name = scheduler_name
        self.gates = FeatureGate(feature_gates)
        self.policy_configmap = policy_configmap
        self.hard_weight = hard_pod_affinity_weight
        cpreds, cprios = {}, {}
        if policy is not None:
            from .policy_args import build
            pol = read_policy(policy)
            preds, prios, cpreds, cprios = build(pol)
            exts = list(pol.get("extenders") or [])
            self.hard_weight = int(pol.get("hardPodAffinitySymmetricWeight", self.hard_weight))
        else:
            preds, prios = PROVIDERS[algorithm_provider]
            exts = []
        self.lock_object = (lock_object_namespace, lock_object_name)
        self.address = address
        self.extenders = [HTTPExtender(e) for e in exts]
        self.cache = SchedulerCache()
        from .volumes import VolumeLister
        self.volumes = VolumeLister()
        prios = self._gate_priorities(prios)
        self.svc_inf = None
        self.ctl_infs: dict[str, Informer] = {}     # replicationcontrollers/replicasets/statefulsets
        from .listers import ControllerListers
        listers = ControllerListers(services=lambda: self.svc_inf.list() if self.svc_inf is not None else [],
                                    rcs=lambda: self._ctl_list("replicationcontrollers"),
                                    rss=lambda: self._ctl_list("replicasets"),
                                    sss=lambda: self._ctl_list("statefulsets"))
        self.algo = GenericScheduler(self.cache, preds, prios, self.extenders, use_topology=self.gates("GPUTopologyScheduling"),
                                     volumes=self.volumes, volume_scheduling=self.gates("VolumeScheduling"),
                                     custom_predicates=cpreds, custom_priorities=cprios,
                                     services=listers.services, listers=listers,
                                     hard_affinity_weight=self.hard_weight)
        self._set_needs(cpreds, cprios, prios)
        self.queue = SchedulingQueue(self.gates("PodPriority"))
        self.algo.queue = self.queue
        self.pdb_inf = None             # PodDisruptionBudgets for preemption (cache.ListPDBs)
        self.recorder = EventRecorder(client, self.name)
        self.leader_elect = leader_elect
        self.identity = identity or f"{self.name}-{id(self):x}"
        self.port = port
        self.disable_preemption = disable_preemption
        self.bind_sem = asyncio.Semaphore(bind_concurrency)
        self.metrics = new_registry()
        r = self.metrics
        self.m_e2e = Histogram("scheduler_e2e_scheduling_latency_microseconds", "E2e scheduling latency (scheduling algorithm + binding)", buckets=MICRO_BUCKETS, registry=r)
        self.m_algo = Histogram("scheduler_scheduling_algorithm_latency_microseconds", "Scheduling algorithm latency", buckets=MICRO_BUCKETS, registry=r)
        self.m_bind = Histogram("scheduler_binding_latency_microseconds", "Binding latency", buckets=MICRO_BUCKETS, registry=r)
        self.m_attempts = Counter("scheduler_schedule_attempts", "Number of attempts to schedule pods, by the result.", ["result"], registry=r)
        self.m_preempt = Counter("scheduler_total_preemption_attempts", "Total preemption attempts in the cluster till now", registry=r)
        self.pod_inf = self.node_inf = None
        self._tasks: list[asyncio.Task] = []
        self._binds: set[asyncio.Task] = set()
        self.scheduled = 0
        self.failed = 0
        self.bind_errors = 0
        self._runner = None

    def _gate_priorities(self, prios: dict) -> dict:
        """Drop priorities whose gate is off: GPUTopologyPriority (GPUTopologyScheduling) and the
        reference's gated ResourceLimitsPriority (defaults.go:113-115); a policy that names a
        gated-off priority is refused, as the reference's registry would not know the name."""
        from .priorities import GATED_PRIORITIES
        out = {}
        for k, v in prios.items():
            if k == "GPUTopologyPriority" and not self.gates("GPUTopologyScheduling"):
                continue
            gate = GATED_PRIORITIES.get(k)
            if gate and not self.gates(gate):
                raise ValueError(f"priority {k!r} is registered only with feature gate {gate}=true")
            out[k] = v
        return out

    def _set_needs(self, cpreds, cprios, prios):
        # serviceAffinity/serviceAntiAffinity arguments read Services; the spreading priorities
        # read Services plus the controllers
        self._needs_controllers = "SelectorSpreadPriority" in prios
        self._needs_services = bool(cpreds or cprios) or self._needs_controllers or "ServiceSpreadingPriority" in prios

    def _ctl_list(self, resource: str) -> list:
        inf = self.ctl_infs.get(resource)
        return inf.list() if inf is not None else []

    # ----------------------------------------------------------- informers
    def _responsible(self, pod) -> bool:
        return (pod.get("spec") or {}).get("schedulerName", "default-scheduler") == self.name

    def _unassigned(self, pod) -> bool:
        return not (pod.get("spec") or {}).get("nodeName") and not is_pod_terminal(pod) and \
            not (pod.get("metadata") or {}).get("deletionTimestamp") and self._responsible(pod)

    @staticmethod
    def _assigned_live(pod) -> bool:
        return bool((pod.get("spec") or {}).get("nodeName")) and not is_pod_terminal(pod)

    def _on_pod_add(self, pod):
        if self._assigned_live(pod):
            self.cache.add_pod(pod)
            self.queue.assigned_pod_added(pod)
        elif self._unassigned(pod):
            POD_TRACE(m.uid_of(pod), "sched_queued")
            self.queue.add(pod)

    def _on_pod_update(self, old, pod):
        if self._assigned_live(pod):
            self.cache.update_pod(old, pod)
            self.queue.delete(pod)
            if m.labels_of(old) != m.labels_of(pod) or not self._assigned_live(old):
                self.queue.assigned_pod_updated(pod)
        elif (pod.get("spec") or {}).get("nodeName"):
            # bound pod went terminal → its resources (incl. GPUs) are free again
            if self._assigned_live(old) or self.cache.is_assumed(pod) or m.key_of(pod) in self.cache.pod_states:
                self.cache.remove_pod(pod)
                self.queue.move_all_to_active()
        elif self._unassigned(pod):
            self.queue.update(pod, old)
        else:
            self.queue.delete(pod)

    def _on_pod_delete(self, pod):
        if (pod.get("spec") or {}).get("nodeName"):
            self.cache.remove_pod(pod)
            self.queue.move_all_to_active()
        else:
            self.queue.delete(pod)

    def _on_volume_update(self, old, new):
        if new.get("kind") == "PersistentVolume" and ((new.get("spec") or {}).get("claimRef")):
            self.volumes.assumed.pop(m.name_of(new), None)     # our pre-binding is visible now
        self.queue.move_all_to_active()

    def _on_node(self, node):
        self.cache.add_node(node)
        self.queue.move_all_to_active()

    def _on_node_update(self, old, node):
        self.cache.update_node(node)
        if (old.get("status") or {}).get("extendedResources") != (node.get("status") or {}).get("extendedResources") or \
                (old.get("spec") or {}) != (node.get("spec") or {}) or \
                (old.get("status") or {}).get("allocatable") != (node.get("status") or {}).get("allocatable"):
            self.queue.move_all_to_active()

    # ------------------------------------------------------------ lifecycle
    async def _policy_from_configmap(self):
        """--policy-configmap: the Policy in a ConfigMap's `policy.cfg` (factory.go CreateFromConfig)."""
        from .policy_args import build
        ns, name = self.policy_configmap
        cm = await self.client.get("configmaps", name, ns)
        raw = (cm.get("data") or {}).get("policy.cfg")
        if not raw:
            raise ValueError(f"ConfigMap {ns}/{name} has no policy.cfg")
        pol = json.loads(raw)
        preds, prios, cpreds, cprios = build(pol)
        prios = self._gate_priorities(prios)
        self.extenders = [HTTPExtender(e) for e in pol.get("extenders") or []]
        self.hard_weight = int(pol.get("hardPodAffinitySymmetricWeight", self.hard_weight))
        self.algo.configure(preds, prios, cpreds, cprios, self.extenders, self.hard_weight)
        self._set_needs(cpreds, cprios, prios)

    async def start(self):
        self.recorder.start()
        if self.policy_configmap is not None:
            await self._policy_from_configmap()
        if self.port is not None:
            await self._serve()
        if self.leader_elect:
            le = LeaderElector(self.client, self.lock_object[1], self.identity, ns=self.lock_object[0])
            self._tasks.append(asyncio.create_task(le.run(self._run_informers_and_loop)))
        else:
            await self._start_informers()
            self._tasks.append(asyncio.create_task(self.run(), name="schedule-loop"))
            self._tasks.append(asyncio.create_task(self._housekeeping(), name="sched-housekeeping"))
        return self

    async def _run_informers_and_loop(self):
        await self._start_informers()
        self._tasks.append(asyncio.create_task(self._housekeeping()))
        await self.run()

    async def _start_informers(self):
        self.node_inf = Informer(self.client, "nodes")
        self.node_inf.add_handler(on_add=self._on_node, on_update=self._on_node_update,
                                  on_delete=lambda n: self.cache.remove_node(n))
        if self.gates("PodPriority") and not self.disable_preemption:
            self.pdb_inf = Informer(self.client, "poddisruptionbudgets")
            self.pdb_inf.start()
        self.pod_inf = Informer(self.client, "pods")
        self.pod_inf.add_handler(on_add=self._on_pod_add, on_update=self._on_pod_update, on_delete=self._on_pod_delete)
        # claims, volumes and classes for the volume predicates; a claim or volume change may make
        # an unschedulable pod schedulable
        self.vol_infs = [Informer(self.client, r) for r in ("persistentvolumeclaims", "persistentvolumes", "storageclasses")]
        self.volumes._pvcs, self.volumes._pvs, self.volumes._classes = self.vol_infs
        for inf in self.vol_infs[:2]:
            inf.add_handler(on_add=lambda o: self.queue.move_all_to_active(), on_update=self._on_volume_update)
        for inf in self.vol_infs:
            inf.start()
        if self._needs_services:
            self.svc_inf = Informer(self.client, "services")
            self.svc_inf.start()
        if self._needs_controllers:
            for r in ("replicationcontrollers", "replicasets", "statefulsets"):
                self.ctl_infs[r] = Informer(self.client, r)
                self.ctl_infs[r].start()
        self.node_inf.start()
        await self.node_inf.wait_synced(30)
        for inf in (*self.vol_infs, *([self.svc_inf] if self.svc_inf else []), *self.ctl_infs.values()):
            await inf.wait_synced(30)
        self.pod_inf.start()
        await self.pod_inf.wait_synced(30)

    async def stop(self):
        from ..utils import cancel_and_wait
        await cancel_and_wait(list(self._tasks) + list(self._binds))
        for inf in (self.pod_inf, self.node_inf, self.svc_inf, self.pdb_inf, *self.ctl_infs.values(),
                    *getattr(self, "vol_infs", [])):
            if inf:
                await inf.stop()
        await self.recorder.stop()
        for e in self.extenders:
            await e.close()
        if self._runner:
            await self._runner.cleanup()
        await self.client.close()

    async def _housekeeping(self):
        while True:
            await asyncio.sleep(1.0)
            self.cache.cleanup_expired()

    async def _serve(self):
        app = web.Application()

        async def healthz(r):
            return web.Response(text="ok")

        async def metrics(r):
            return web.Response(body=render(self.metrics), headers={"Content-Type": CONTENT_TYPE})
        app.router.add_get("/healthz", healthz)
        app.router.add_get("/metrics", metrics)
        profiling.add_routes(app)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.address, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]

    # ------------------------------------------------------------ main loop
    async def run(self):
        while True:
            pod = await self.queue.pop()
            try:
                await self.schedule_one(pod)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.exception("scheduling %s crashed: %r", m.key_of(pod), e)
                self.queue.add_unschedulable(pod, marked=True)

    async def schedule_one(self, pod: dict):
        key = m.key_of(pod)
        cur = self.pod_inf.get(key) if self.pod_inf else pod
        if cur is None or not self._unassigned(cur) or self.cache.is_assumed(cur):
            return
        pod = cur
        t0 = time.perf_counter()
        POD_TRACE(m.uid_of(pod), "sched_start")
        try:
            host, binding = await self.algo.schedule(pod)
        except FitError as e:
            self.failed += 1
            self.m_attempts.labels("unschedulable").inc()
            self.recorder.event(pod, "Warning", "FailedScheduling", str(e))
            asyncio.create_task(self._mark_unschedulable(pod, str(e)))
            if not self.disable_preemption and self.gates("PodPriority"):
                pod = await self._preempt(pod, e)
            self.queue.add_unschedulable(pod, marked=True)
            return
        self.m_algo.observe((time.perf_counter() - t0) * 1e6)
        # assume: nodeName + chosen devices (fix #1: devices are reserved before the bind)
        # a structural copy of only what assume changes (the informer's object is never mutated)
        spec = dict(pod.get("spec") or {}, nodeName=host)
        if binding and self.gates("ReserveDevicesOnAssume") and spec.get("extendedResources"):
            spec["extendedResources"] = [dict(pres, assigned=list(binding[pres["name"]]["resources"]))
                                         if pres.get("name") in binding else pres for pres in spec["extendedResources"]]
        assumed = dict(pod, spec=spec)
        try:
            self.cache.assume_pod(assumed)
        except KeyError:
            return
        vbinds = self.algo.volume_binds.pop(key, [])
        for pvc, pv in vbinds:
            self.volumes.assumed[m.name_of(pv)] = m.key_of(pvc)
        t = asyncio.create_task(self._bind(pod, assumed, host, binding, t0, vbinds))
        self._binds.add(t)
        t.add_done_callback(self._binds.discard)

    async def _bind(self, pod, assumed, host, binding, t0, vbinds=()):
        POD_TRACE(m.uid_of(pod), "sched_assumed")
        async with self.bind_sem:
            tb = time.perf_counter()
            try:
                # scheduler_binder.go BindPodVolumes: pre-bind the chosen PVs to their claims;
                # the PV controller completes the binding
                for pvc, pv in vbinds:
                    await self.client.patch("persistentvolumes", m.name_of(pv), {"spec": {"claimRef": {
                        "kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": m.namespace_of(pvc),
                        "name": m.name_of(pvc), "uid": m.uid_of(pvc)}}})
                bound_by_ext = False
                for ext in self.extenders:
                    if ext.bind_verb:
                        await ext.bind(pod, host, binding or None)
                        bound_by_ext = True
                        break
                if not bound_by_ext:
                    await self.client.bind(m.namespace_of(pod), m.name_of(pod), host, binding or None, uid=m.uid_of(pod))
            except Exception as e:
                self.bind_errors += 1
                self.m_attempts.labels("error").inc()
                self.cache.forget_pod(assumed)
                for _pvc, pv in vbinds:
                    self.volumes.assumed.pop(m.name_of(pv), None)
                log.info("binding %s to %s rejected: %s", m.key_of(pod), host, e)
                self.recorder.event(pod, "Warning", "FailedScheduling", f"Binding rejected: {e}")
                if not (isinstance(e, m.StatusError) and (m.is_not_found(e) or "already assigned" in e.message)):
                    self.queue.add_unschedulable(pod, marked=True)
                    self.queue.move_all_to_active()
                return
            self.cache.finish_binding(assumed)
            now = time.perf_counter()
            self.m_bind.observe((now - tb) * 1e6)
            self.m_e2e.observe((now - t0) * 1e6)
            POD_TRACE(m.uid_of(pod), "sched_bound")
            self.m_attempts.labels("scheduled").inc()
            self.scheduled += 1
            self.recorder.event(pod, "Normal", "Scheduled", f"Successfully assigned {m.name_of(pod)} to {host}")

    async def _mark_unschedulable(self, pod, msg):
        cond = {"type": "PodScheduled", "status": "False", "reason": "Unschedulable", "message": msg,
                "lastProbeTime": None, "lastTransitionTime": m.now_rfc3339()}
        for c in (pod.get("status") or {}).get("conditions") or []:
            if c.get("type") == "PodScheduled" and c.get("message") == msg:
                return
        try:
            await self.client.patch("pods", m.name_of(pod), {"status": {"conditions": [cond]}}, m.namespace_of(pod), sub="status")
        except Exception:
            pass

    async def _preempt(self, pod, fit_error) -> dict:
        """scheduler.go preempt (:209-253): nominate the preemptor to the chosen node (the
        NominatedNodeName annotation), delete the victims, clear the nominations the algorithm
        hands back. Returns the preemptor as the queue must now hold it (with its nomination,
        before the informer brings the patched object back)."""
        self.m_preempt.inc()
        pdbs = self.pdb_inf.list() if self.pdb_inf is not None else []
        node, victims, to_clear = await self.algo.preempt_async(pod, fit_error.failed, pdbs)
        if node:
            ann = dict(((pod.get("metadata") or {}).get("annotations")) or {}, **{NOMINATED_NODE_ANNOTATION: node})
            try:
                await self.client.patch("pods", m.name_of(pod), {"metadata": {"annotations": {NOMINATED_NODE_ANNOTATION: node}}},
                                        m.namespace_of(pod))
            except m.StatusError as e:
                log.info("nominating %s to %s: %s", m.key_of(pod), node, e)
                return pod
            pod = dict(pod, metadata=dict(pod.get("metadata") or {}, annotations=ann))
            for v in victims:
                try:
                    await self.client.delete("pods", m.name_of(v), m.namespace_of(v))
                except m.StatusError as e:
                    log.info("preempting %s: %s", m.key_of(v), e)
                    return pod
                self.recorder.event(v, "Normal", "Preempted", f"by {m.key_of(pod)} on node {node}")
        for p in to_clear:
            # RemoveNominatedNodeAnnotation: a JSON merge patch that deletes the key
            try:
                await self.client.patch("pods", m.name_of(p), {"metadata": {"annotations": {NOMINATED_NODE_ANNOTATION: None}}},
                                        m.namespace_of(p))
            except m.StatusError:
                pass
            if m.key_of(p) == m.key_of(pod):
                md = dict(pod.get("metadata") or {})
                md["annotations"] = {k: v for k, v in (md.get("annotations") or {}).items() if k != NOMINATED_NODE_ANNOTATION}
                pod = dict(pod, metadata=md)
        return pod
