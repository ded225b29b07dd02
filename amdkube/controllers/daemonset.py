"""DaemonSet controller (pkg/controller/daemon/{daemon_controller,update}.go, util/daemonset_util.go).

One pass of `sync` (syncDaemonSet :1082-1151):
  * a selector that selects everything is refused (SelectingAll event);
  * history (constructHistory): ControllerRevisions matching the selector are claimed; the one
    whose data is this template (getPatch) is current — renumbered past the old ones when it
    comes back, deduplicated when several match — or a new snapshot `<ds>-<hash>` (hash =
    ComputeHash(template, collisionCount), also the pods' controller-revision-hash label);
  * being deleted, or expectations unsatisfied: status only;
  * manage: per node, nodeShouldRunDaemonPod (a simulated scheduling of the would-be pod against
    the node's other pods: taints with the daemon tolerations for not-ready / unreachable /
    disk- and memory-pressure (+ out-of-disk for critical pods), GeneralPredicates — or
    EssentialPredicates, no resource fit, for critical pods) yields wantToRun / shouldSchedule /
    shouldContinueRunning; missing pods are created, failed pods deleted (FailedDaemonPod, and
    the sync errors so it backs off), duplicates beyond the oldest deleted, pods on nodes that
    should not run them deleted; creates go out in slow-start batches under expectations
    (burstReplicas 250) — a node wanted but unschedulable is remembered (suspended) and its
    DaemonSets requeued when a non-daemon pod on it goes away;
  * RollingUpdate: old-template pods that are not available go, then available ones while fewer
    than maxUnavailable (of the desired count, rounded up) are unavailable;
  * cleanupHistory keeps revisionHistoryLimit old revisions plus any a live pod uses;
  * status: desired / current / misscheduled / ready / updated / available / unavailable.
Pods are "updated" when their template-generation label matches spec.templateGeneration or their
hash label matches the current revision. apps/v1 DaemonSets carry no templateGeneration, so
for them only the hash counts (docs/PARITY.md).
"""
from __future__ import annotations

import asyncio
import time

from ..api import meta as m
from ..api.helpers import is_pod_ready
from ..api.labels import selector_from_label_selector
from ..scheduler.cache import NodeInfo
from ..scheduler import predicates as P
from . import history as H
from .base import Controller
from .controller_utils import (SLOW_START_INITIAL_BATCH, ControllerExpectations, ControllerRefManager, adopt_patch,
                               recheck_deletion, release_patch)
from .deployment import compute_hash, int_or_percent, safe_encode
from .replicaset import RealPodControl, is_pod_available

HASH_LABEL = "controller-revision-hash"          # DefaultDaemonSetUniqueLabelKey
TEMPLATE_GEN_LABEL = "pod-template-generation"   # DaemonSetTemplateGenerationKey
CRITICAL_ANNOTATION = "scheduler.alpha.kubernetes.io/critical-pod"
BURST_REPLICAS = 250
STATUS_UPDATE_RETRIES = 1

SELECTING_ALL = "SelectingAll"
FAILED_PLACEMENT = "FailedPlacement"
FAILED_DAEMON_POD = "FailedDaemonPod"

TAINT_NOT_READY = "node.kubernetes.io/not-ready"
TAINT_UNREACHABLE = "node.kubernetes.io/unreachable"
TAINT_OUT_OF_DISK = "node.kubernetes.io/out-of-disk"
TAINT_MEMORY_PRESSURE = "node.kubernetes.io/memory-pressure"
TAINT_DISK_PRESSURE = "node.kubernetes.io/disk-pressure"


# ============================================================================ util
def _spec(o) -> dict:
    return (o or {}).get("spec") or {}


def _status(o) -> dict:
    return (o or {}).get("status") or {}


def add_or_update_toleration(spec: dict, tol: dict) -> bool:
    """AddOrUpdateTolerationInPodSpec: appended unless an identical one is there."""
    tols = spec.get("tolerations")
    if tols is None:
        tols = spec["tolerations"] = []
    want = (tol.get("key", ""), tol.get("effect", ""), tol.get("operator", ""), tol.get("value", ""))
    for t in tols:
        if (t.get("key", ""), t.get("effect", ""), t.get("operator", ""), t.get("value", "")) == want:
            return False
    tols.append(dict(tol))
    return True


def is_critical(namespace: str, annotations: dict | None) -> bool:
    """kubelet/types IsCritical: kube-system and the critical-pod annotation with an empty value."""
    return namespace == "kube-system" and (annotations or {}).get(CRITICAL_ANNOTATION) == ""


def template_generation(ds):
    """spec.templateGeneration (extensions/v1beta1); None for apps/v1 objects."""
    return _spec(ds).get("templateGeneration")


def create_pod_template(template: dict, generation, hash_: str, critical_gate: bool = False,
                        namespace: str = "") -> dict:
    """CreatePodTemplate: the daemon tolerations, the template-generation label and the hash."""
    tpl = m.deepcopy(template or {})
    spec = tpl.setdefault("spec", {})
    add_or_update_toleration(spec, {"key": TAINT_NOT_READY, "operator": "Exists", "effect": "NoExecute"})
    add_or_update_toleration(spec, {"key": TAINT_UNREACHABLE, "operator": "Exists", "effect": "NoExecute"})
    add_or_update_toleration(spec, {"key": TAINT_DISK_PRESSURE, "operator": "Exists", "effect": "NoSchedule"})
    add_or_update_toleration(spec, {"key": TAINT_MEMORY_PRESSURE, "operator": "Exists", "effect": "NoSchedule"})
    md = tpl.setdefault("metadata", {})
    if critical_gate and is_critical(md.get("namespace") or namespace, md.get("annotations")):
        add_or_update_toleration(spec, {"key": TAINT_OUT_OF_DISK, "operator": "Exists", "effect": "NoExecute"})
    labels = dict((template or {}).get("metadata", {}).get("labels") or {})
    if generation is not None:
        labels[TEMPLATE_GEN_LABEL] = str(generation)
    if hash_:
        labels[HASH_LABEL] = hash_
    md["labels"] = labels
    return tpl


def is_pod_updated(generation, pod: dict, hash_: str) -> bool:
    labels = m.labels_of(pod)
    template_matches = generation is not None and labels.get(TEMPLATE_GEN_LABEL) == str(generation)
    hash_matches = bool(hash_) and labels.get(HASH_LABEL) == hash_
    return hash_matches or template_matches


def split_by_available_pods(min_ready: int, pods: list, now: float):
    available, unavailable = [], []
    for p in pods:
        (available if is_pod_available(p, min_ready, now) else unavailable).append(p)
    return available, unavailable


def get_patch(ds) -> dict:
    tpl = m.deepcopy(_spec(ds).get("template") or {})
    tpl["$patch"] = "replace"
    return {"spec": {"template": tpl}}


def match(ds, rev) -> bool:
    return H.raw(get_patch(ds)) == H.raw(rev.get("data"))


def new_pod(ds, node_name: str) -> dict:
    """NewPod: the template's metadata and spec, in the DaemonSet's namespace, on the node."""
    tpl = m.deepcopy(_spec(ds).get("template") or {})
    md = tpl.get("metadata") or {}
    md["namespace"] = m.namespace_of(ds)
    spec = tpl.get("spec") or {}
    spec["nodeName"] = node_name
    return {"metadata": md, "spec": spec}


def _creation_key(o):
    return (m.parse_time((o.get("metadata") or {}).get("creationTimestamp")) or 0.0, m.name_of(o))


def daemon_predicates(pi: P.PodInfo, ni, critical: bool) -> list:
    """Predicates (daemon_controller.go:1332-1361): taints, then General- (or, for critical
    pods, Essential-) predicates; every failure reason."""
    reasons = list(P.pod_tolerates_node_taints(pi, ni)[1])
    checks = (P.pod_fits_host, P.pod_fits_host_ports, P.pod_match_node_selector) if critical else \
        (P.pod_fits_resources, P.pod_fits_host, P.pod_fits_host_ports, P.pod_match_node_selector)
    for fn in checks:
        reasons += fn(pi, ni)[1]
    return reasons


_SKIP = {P.ERR_NODE_SELECTOR_NOT_MATCH, P.ERR_POD_NOT_MATCH_HOST_NAME, P.ERR_NODE_LABEL_PRESENCE_VIOLATED,
         P.ERR_POD_NOT_FITS_HOST_PORTS}
_NO_SCHEDULE = {P.ERR_DISK_CONFLICT, P.ERR_VOLUME_ZONE_CONFLICT, P.ERR_MAX_VOLUME_COUNT_EXCEEDED,
                P.ERR_NODE_UNDER_MEMORY_PRESSURE, P.ERR_NODE_UNDER_DISK_PRESSURE}
_UNEXPECTED = {P.ERR_POD_AFFINITY_NOT_MATCH, P.ERR_SERVICE_AFFINITY_VIOLATED}


class DaemonPodControl(RealPodControl):
    """PodControl with CreatePodsOnNode."""

    async def create_pods_on_node(self, node_name: str, ns: str, template: dict, owner: dict, controller_ref: dict):
        from .replicaset import pod_from_template
        pod = pod_from_template(template, owner, controller_ref)
        if node_name:
            pod["spec"]["nodeName"] = node_name
        try:
            created = await self.client.create(pod, ns)
        except Exception as e:
            self._event(owner, "Warning", "FailedCreate", f"Error creating: {e}")
            raise
        self._event(owner, "Normal", "SuccessfulCreate", f"Created pod: {m.name_of(created)}")
        return created


# ============================================================================ controller
class DaemonSetController(Controller):
    name = "daemonset"
    workers = 2
    api_version, kind = "apps/v1", "DaemonSet"

    def __init__(self, mgr, pod_control=None, clock=time.time, critical_pods: bool = False,
                 burst_replicas: int = BURST_REPLICAS):
        super().__init__(mgr)
        self.clock = clock
        self.critical_gate = critical_pods               # --feature-gates ExperimentalCriticalPodAnnotation
        self.burst_replicas = burst_replicas
        self.expectations = ControllerExpectations(clock=time.monotonic)
        self.suspended: dict[str, set] = {}               # node -> DaemonSet keys wanted there but unschedulable
        self.pod_control = pod_control

    @property
    def recorder(self):
        return getattr(self.mgr, "recorder", None)

    def _event(self, obj, etype, reason, msg):
        if self.recorder is not None:
            self.recorder.event(obj, etype, reason, msg)

    def setup(self):
        f = self.mgr.factory
        self.ds_inf = f.informer("daemonsets")
        self.rev_inf = f.informer("controllerrevisions.apps")
        self.node_inf = self.mgr.nodes
        self.pod_inf = self.mgr.pods
        if self.pod_control is None:
            self.pod_control = DaemonPodControl(self.client, self.recorder)
        self.ds_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.rev_inf.add_handler(on_add=self.add_history, on_update=self.update_history, on_delete=self.delete_history)
        self.pod_inf.add_handler(on_add=self.add_pod, on_update=self.update_pod, on_delete=self.delete_pod)
        self.node_inf.add_handler(on_add=self.add_node, on_update=self.update_node)

    # ------------------------------------------------------------------ queueing
    def enqueue_rate_limited(self, ds):
        self.queue.add_rate_limited(m.key_of(ds))

    def enqueue_after(self, ds, after: float):
        try:
            self.queue.add_after(m.key_of(ds), after)
        except RuntimeError:                              # no running loop (a synchronous caller)
            self.queue.add(m.key_of(ds))

    def resolve(self, ns, ref):
        if ref.get("kind") != "DaemonSet":
            return None
        ds = self.ds_inf.get(f"{ns}/{ref.get('name')}")
        if ds is None or m.uid_of(ds) != ref.get("uid"):
            return None
        return ds

    def _selecting(self, obj) -> list:
        """GetPodDaemonSets / GetHistoryDaemonSets: the namespace's sets whose (non-empty)
        selector matches the object's labels."""
        labels = m.labels_of(obj)
        if not labels:
            return []
        out = []
        for ds in self.ds_inf.list():
            if m.namespace_of(ds) != m.namespace_of(obj):
                continue
            try:
                sel = selector_from_label_selector(_spec(ds).get("selector"))
            except Exception:
                continue
            if sel.empty() or not sel.matches(labels):
                continue
            out.append(ds)
        return out

    # ------------------------------------------------------------------ history events
    def add_history(self, rev):
        if (rev.get("metadata") or {}).get("deletionTimestamp"):
            self.delete_history(rev)
            return
        ref = m.controller_ref(rev)
        if ref is not None:
            ds = self.resolve(m.namespace_of(rev), ref)
            if ds is not None:
                self.enqueue(ds)
            return
        for ds in self._selecting(rev):
            self.enqueue(ds)

    def update_history(self, old, cur):
        if (old.get("metadata") or {}).get("resourceVersion") == (cur.get("metadata") or {}).get("resourceVersion"):
            return
        cur_ref, old_ref = m.controller_ref(cur), m.controller_ref(old)
        changed = cur_ref != old_ref
        if changed and old_ref is not None:
            ds = self.resolve(m.namespace_of(old), old_ref)
            if ds is not None:
                self.enqueue(ds)
        if cur_ref is not None:
            ds = self.resolve(m.namespace_of(cur), cur_ref)
            if ds is not None:
                self.enqueue(ds)
            return
        if changed or m.labels_of(cur) != m.labels_of(old):
            for ds in self._selecting(cur):
                self.enqueue(ds)

    def delete_history(self, rev):
        ref = m.controller_ref(rev)
        if ref is None:
            return
        ds = self.resolve(m.namespace_of(rev), ref)
        if ds is not None:
            self.enqueue(ds)

    # ------------------------------------------------------------------ pod events
    def add_pod(self, pod):
        if (pod.get("metadata") or {}).get("deletionTimestamp"):
            self.delete_pod(pod)
            return
        ref = m.controller_ref(pod)
        if ref is not None:
            ds = self.resolve(m.namespace_of(pod), ref)
            if ds is None:
                return
            self.expectations.creation_observed(m.key_of(ds))
            self.enqueue(ds)
            return
        for ds in self._selecting(pod):
            self.enqueue(ds)

    def update_pod(self, old, cur):
        if (old.get("metadata") or {}).get("resourceVersion") == (cur.get("metadata") or {}).get("resourceVersion"):
            return
        cur_ref, old_ref = m.controller_ref(cur), m.controller_ref(old)
        changed = cur_ref != old_ref
        if changed and old_ref is not None:
            ds = self.resolve(m.namespace_of(old), old_ref)
            if ds is not None:
                self.enqueue(ds)
        if cur_ref is not None:
            ds = self.resolve(m.namespace_of(cur), cur_ref)
            if ds is None:
                return
            self.enqueue(ds)
            mrs = int(_spec(ds).get("minReadySeconds") or 0)
            if not is_pod_ready(old) and is_pod_ready(cur) and mrs > 0:
                self.enqueue_after(ds, mrs + 1.0)
            return
        dss = self._selecting(cur)
        if dss and (m.labels_of(cur) != m.labels_of(old) or changed):
            for ds in dss:
                self.enqueue(ds)

    def delete_pod(self, pod):
        ref = m.controller_ref(pod)
        node = _spec(pod).get("nodeName")
        ds = self.resolve(m.namespace_of(pod), ref) if ref is not None else None
        if ds is None:
            if node:
                self.requeue_suspended(node)              # a non-daemon pod freed room on the node
            return
        self.expectations.deletion_observed(m.key_of(ds))
        self.enqueue(ds)

    # ------------------------------------------------------------------ suspended daemon pods
    def requeue_suspended(self, node: str):
        for key in list(self.suspended.get(node, ())):
            ds = self.ds_inf.get(key)
            if ds is not None:
                self.enqueue_rate_limited(ds)

    def _suspend(self, node, key):
        self.suspended.setdefault(node, set()).add(key)

    def _unsuspend(self, node, key):
        s = self.suspended.get(node)
        if s is None:
            return
        s.discard(key)
        if not s:
            del self.suspended[node]

    # ------------------------------------------------------------------ node events
    def add_node(self, node):
        for ds in self.ds_inf.list():
            try:
                _, should_schedule, _ = self.node_should_run(node, ds)
            except Exception:
                continue
            if should_schedule:
                self.enqueue(ds)

    @staticmethod
    def node_in_same_condition(old: list, cur: list) -> bool:
        if not old and not cur:
            return True
        trues = {c.get("type") for c in old or [] if c.get("status") == "True"}
        for c in cur or []:
            if c.get("status") != "True":
                continue
            if c.get("type") not in trues:
                return False
            trues.discard(c.get("type"))
        return not trues

    def update_node(self, old, cur):
        if m.labels_of(old) == m.labels_of(cur) and _spec(old).get("taints") == _spec(cur).get("taints") and \
                self.node_in_same_condition(_status(old).get("conditions"), _status(cur).get("conditions")):
            return
        for ds in self.ds_inf.list():
            try:
                _, old_sched, old_cont = self.node_should_run(old, ds)
                _, cur_sched, cur_cont = self.node_should_run(cur, ds)
            except Exception:
                continue
            if old_sched != cur_sched or old_cont != cur_cont:
                self.enqueue(ds)

    # ------------------------------------------------------------------ pods of a DaemonSet
    async def daemon_pods(self, ds) -> list:
        """getDaemonPods: claim the namespace's pods (adopt / release through the pod control)."""
        sel = selector_from_label_selector(_spec(ds).get("selector"))
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == m.namespace_of(ds)]
        client, pc = self.client, self.pod_control

        async def fresh():
            f = await client.get("daemonsets", m.name_of(ds), m.namespace_of(ds))
            if m.uid_of(f) != m.uid_of(ds):
                raise RuntimeError(f"original DaemonSet {m.key_of(ds)} is gone: got uid {m.uid_of(f)}, "
                                   f"wanted {m.uid_of(ds)}")
            return f

        async def adopt(pod):
            await pc.patch_pod(m.namespace_of(pod), m.name_of(pod), adopt_patch(ds, self.api_version, self.kind, pod))

        async def release(pod):
            try:
                await pc.patch_pod(m.namespace_of(pod), m.name_of(pod), release_patch(ds, pod))
            except m.StatusError as e:
                if not (m.is_not_found(e) or e.code == 422):
                    raise
        return await ControllerRefManager(ds, sel, adopt, release, recheck_deletion(fresh)).claim(pods)

    async def nodes_to_daemon_pods(self, ds) -> dict:
        out: dict[str, list] = {}
        for p in await self.daemon_pods(ds):
            out.setdefault(_spec(p).get("nodeName") or "", []).append(p)
        return out

    # ------------------------------------------------------------------ nodeShouldRunDaemonPod
    def _is_controlled_by(self, pod, ds) -> bool:
        ref = m.controller_ref(pod)
        return ref is not None and ref.get("uid") == m.uid_of(ds)

    def simulate(self, pod: dict, node: dict, ds):
        spec = pod.setdefault("spec", {})
        add_or_update_toleration(spec, {"key": TAINT_NOT_READY, "operator": "Exists", "effect": "NoExecute"})
        add_or_update_toleration(spec, {"key": TAINT_UNREACHABLE, "operator": "Exists", "effect": "NoExecute"})
        add_or_update_toleration(spec, {"key": TAINT_DISK_PRESSURE, "operator": "Exists", "effect": "NoSchedule"})
        add_or_update_toleration(spec, {"key": TAINT_MEMORY_PRESSURE, "operator": "Exists", "effect": "NoSchedule"})
        critical = self.critical_gate and is_critical(m.namespace_of(pod), m.annotations_of(pod))
        if critical:
            add_or_update_toleration(spec, {"key": TAINT_OUT_OF_DISK, "operator": "Exists", "effect": "NoSchedule"})
        ni = NodeInfo(m.name_of(node))
        ni.set_node(node)
        for i, p in enumerate(self.pod_inf.list()):
            if _spec(p).get("nodeName") != m.name_of(node):
                continue
            if _status(p).get("phase") in ("Succeeded", "Failed") or self._is_controlled_by(p, ds):
                continue
            ni.add_pod(f"{m.namespace_of(p)}/{m.name_of(p)}/{i}", p)
        pi = P.PodInfo(pod)
        return daemon_predicates(pi, ni, critical), pi, ni

    def node_should_run(self, node: dict, ds) -> tuple[bool, bool, bool]:
        """(wantToRun, shouldSchedule, shouldContinueRunning); FailedPlacement events as the
        reference emits them (each call may emit)."""
        pod = new_pod(ds, m.name_of(node))
        want = schedule = cont = True
        nn = (_spec(ds).get("template") or {}).get("spec", {}).get("nodeName") or ""
        if nn and nn != m.name_of(node):
            return False, False, False
        reasons, pi, ni = self.simulate(pod, node, ds)
        insufficient = None
        for r in reasons:
            if r.startswith("Insufficient "):
                insufficient = r
                continue
            emit = False
            if r in _SKIP:
                return False, False, False
            if r == P.ERR_TAINTS_TOLERATIONS_NOT_MATCH:
                if not P.pod_tolerates_node_no_execute_taints(pi, ni)[0]:
                    return False, False, False
                want = schedule = False
            elif r in _NO_SCHEDULE:
                schedule = False
                emit = True
            elif r in _UNEXPECTED:
                raise ValueError(f"unexpected reason: DaemonSet Predicates should not return reason {r}")
            else:
                want = schedule = cont = False
                emit = True
            if emit:
                self._event(ds, "Warning", FAILED_PLACEMENT, f'failed to place pod on "{m.name_of(node)}": {r}')
        if schedule and insufficient is not None:
            self._event(ds, "Warning", FAILED_PLACEMENT, f'failed to place pod on "{m.name_of(node)}": {insufficient}')
            schedule = False
        return want, schedule, cont

    # ------------------------------------------------------------------ manage / syncNodes
    async def manage(self, ds, hash_: str):
        node_pods = await self.nodes_to_daemon_pods(ds)
        key = m.key_of(ds)
        to_create, to_delete, failed = [], [], 0
        for node in self.node_inf.list():
            try:
                want, schedule, cont = self.node_should_run(node, ds)
            except Exception:
                continue
            nn = m.name_of(node)
            pods = node_pods.get(nn)
            self._unsuspend(nn, key)
            if want and not schedule:
                self._suspend(nn, key)
            elif schedule and pods is None:
                to_create.append(nn)
            elif cont:
                running = []
                for p in pods or []:
                    if (p.get("metadata") or {}).get("deletionTimestamp"):
                        continue
                    if _status(p).get("phase") == "Failed":
                        self._event(ds, "Warning", FAILED_DAEMON_POD,
                                    f"Found failed daemon pod {m.namespace_of(p)}/{m.name_of(p)} on node {nn}, "
                                    f"will try to kill it")
                        to_delete.append(m.name_of(p))
                        failed += 1
                    else:
                        running.append(p)
                if len(running) > 1:
                    running.sort(key=_creation_key)
                    to_delete += [m.name_of(p) for p in running[1:]]
            elif pods is not None:
                to_delete += [m.name_of(p) for p in pods]
        await self.sync_nodes(ds, to_delete, to_create, hash_)
        if failed:
            raise RuntimeError(f"deleted {failed} failed pods of DaemonSet {key}")

    async def sync_nodes(self, ds, to_delete: list, to_create: list, hash_: str):
        key = m.key_of(ds)
        create_diff = min(len(to_create), self.burst_replicas)
        delete_diff = min(len(to_delete), self.burst_replicas)
        self.expectations.set_expectations(key, create_diff, delete_diff)
        errors: list[BaseException] = []
        template = create_pod_template(_spec(ds).get("template") or {}, template_generation(ds), hash_,
                                       self.critical_gate, m.namespace_of(ds))
        ref = m.new_controller_ref(ds, self.api_version, self.kind)

        async def create(node_name):
            try:
                await self.pod_control.create_pods_on_node(node_name, m.namespace_of(ds), template, ds, ref)
            except asyncio.TimeoutError:
                return                                    # the pod may still be created; its event will tell
            except Exception as e:                        # noqa: BLE001
                self.expectations.creation_observed(key)
                errors.append(e)

        pos, batch = 0, min(create_diff, SLOW_START_INITIAL_BATCH)
        while pos < create_diff:
            before = len(errors)
            await asyncio.gather(*(create(to_create[i]) for i in range(pos, pos + batch)))
            skipped = create_diff - (pos + batch)
            if len(errors) > before and skipped > 0:
                for _ in range(skipped):
                    self.expectations.creation_observed(key)
                break
            pos += batch
            batch = min(2 * batch, create_diff - pos)

        async def delete(name):
            try:
                await self.pod_control.delete_pod(m.namespace_of(ds), name, ds)
            except Exception as e:                        # noqa: BLE001
                self.expectations.deletion_observed(key)
                errors.append(e)
        await asyncio.gather(*(delete(to_delete[i]) for i in range(delete_diff)))
        if errors:
            raise errors[0] if len(errors) == 1 else RuntimeError("[" + ", ".join(str(e) for e in errors) + "]")

    # ------------------------------------------------------------------ status
    async def update_status(self, ds, hash_: str):
        node_pods = await self.nodes_to_daemon_pods(ds)
        desired = current = misscheduled = ready = updated = available = 0
        now = self.clock()
        mrs = int(_spec(ds).get("minReadySeconds") or 0)
        for node in self.node_inf.list():
            want, _, _ = self.node_should_run(node, ds)
            pods = node_pods.get(m.name_of(node)) or []
            if want:
                desired += 1
                if pods:
                    current += 1
                    pod = sorted(pods, key=_creation_key)[0]
                    if is_pod_ready(pod):
                        ready += 1
                        if is_pod_available(pod, mrs, now):
                            available += 1
                    if is_pod_updated(template_generation(ds), pod, hash_):
                        updated += 1
            elif pods:
                misscheduled += 1
        await self.store_status(ds, desired, current, misscheduled, ready, updated, available, desired - available)

    async def store_status(self, ds, desired, current, misscheduled, ready, updated, available, unavailable):
        st = {"desiredNumberScheduled": desired, "currentNumberScheduled": current,
              "numberMisscheduled": misscheduled, "numberReady": ready, "updatedNumberScheduled": updated,
              "numberAvailable": available, "numberUnavailable": unavailable}
        cur = _status(ds)
        gen = int((ds.get("metadata") or {}).get("generation") or 0)
        if all(int(cur.get(k) or 0) == v for k, v in st.items()) and int(cur.get("observedGeneration") or 0) >= gen:
            return
        to_update = m.deepcopy(ds)
        err = None
        for _ in range(STATUS_UPDATE_RETRIES):
            to_update.setdefault("status", {}).update(st, observedGeneration=gen)
            try:
                await self.client.update(dict(to_update, apiVersion=to_update.get("apiVersion") or self.api_version,
                                              kind=self.kind), "status")
                return
            except m.StatusError as e:
                err = e
            to_update = await self.client.get("daemonsets", m.name_of(ds), m.namespace_of(ds))
        if err is not None:
            raise err

    # ------------------------------------------------------------------ sync
    async def sync(self, key):
        ds = self.ds_inf.get(key)
        if ds is None:
            self.expectations.delete_expectations(key)
            return
        sel = _spec(ds).get("selector")
        if sel is not None and not sel.get("matchLabels") and not sel.get("matchExpressions"):
            self._event(ds, "Warning", SELECTING_ALL,
                        "This daemon set is selecting all pods. A non-empty selector is required.")
            return
        cur, old = await self.construct_history(ds)
        hash_ = m.labels_of(cur).get(HASH_LABEL, "")
        if (ds.get("metadata") or {}).get("deletionTimestamp") or not self.expectations.satisfied_expectations(key):
            await self.update_status(ds, hash_)
            return
        await self.manage(ds, hash_)
        if self.expectations.satisfied_expectations(key):
            if ((_spec(ds).get("updateStrategy") or {}).get("type") or "RollingUpdate") == "RollingUpdate":
                await self.rolling_update(ds, hash_)
        await self.cleanup_history(ds, old)
        await self.update_status(ds, hash_)

    # ------------------------------------------------------------------ rolling update (update.go)
    async def rolling_update(self, ds, hash_: str):
        node_pods = await self.nodes_to_daemon_pods(ds)
        old_pods = [p for pods in node_pods.values() for p in pods
                    if not is_pod_updated(template_generation(ds), p, hash_)]
        max_unavailable, num_unavailable = self.unavailable_numbers(ds, node_pods)
        avail, unavail = split_by_available_pods(int(_spec(ds).get("minReadySeconds") or 0), old_pods, self.clock())
        to_delete = [m.name_of(p) for p in unavail if not (p.get("metadata") or {}).get("deletionTimestamp")]
        for p in avail:
            if num_unavailable >= max_unavailable:
                break
            to_delete.append(m.name_of(p))
            num_unavailable += 1
        await self.sync_nodes(ds, to_delete, [], hash_)

    def unavailable_numbers(self, ds, node_pods: dict) -> tuple[int, int]:
        unavailable = desired = 0
        now = self.clock()
        mrs = int(_spec(ds).get("minReadySeconds") or 0)
        for node in self.node_inf.list():
            want, _, _ = self.node_should_run(node, ds)
            if not want:
                continue
            desired += 1
            pods = node_pods.get(m.name_of(node))
            if pods is None:
                unavailable += 1
                continue
            if not any(is_pod_available(p, mrs, now) and not (p.get("metadata") or {}).get("deletionTimestamp")
                       for p in pods):
                unavailable += 1
        ru = (_spec(ds).get("updateStrategy") or {}).get("rollingUpdate") or {}
        return int_or_percent(ru.get("maxUnavailable", 1), desired, True), unavailable

    # ------------------------------------------------------------------ history (update.go)
    async def controlled_histories(self, ds) -> list:
        sel = selector_from_label_selector(_spec(ds).get("selector"))
        revs = [r for r in self.rev_inf.list() if m.namespace_of(r) == m.namespace_of(ds)]
        client = self.client

        async def fresh():
            f = await client.get("daemonsets", m.name_of(ds), m.namespace_of(ds))
            if m.uid_of(f) != m.uid_of(ds):
                raise RuntimeError(f"original DaemonSet {m.key_of(ds)} is gone")
            return f

        async def adopt(r):
            await client.patch(H.History.resource, m.name_of(r), adopt_patch(ds, self.api_version, self.kind, r),
                               m.namespace_of(r), patch_type="application/strategic-merge-patch+json")

        async def release(r):
            try:
                await client.patch(H.History.resource, m.name_of(r), release_patch(ds, r), m.namespace_of(r),
                                   patch_type="application/strategic-merge-patch+json")
            except m.StatusError as e:
                if not (m.is_not_found(e) or e.code == 422):
                    raise
        return await ControllerRefManager(ds, sel, adopt, release, recheck_deletion(fresh)).claim(revs)

    async def construct_history(self, ds):
        """constructHistory: (current revision, old revisions)."""
        current, old = [], []
        for r in await self.controlled_histories(ds):
            if HASH_LABEL not in m.labels_of(r):
                r = m.deepcopy(r)
                r["metadata"].setdefault("labels", {})[HASH_LABEL] = m.name_of(r)
                r = await self.client.update(dict(r, apiVersion="apps/v1", kind="ControllerRevision"))
            (current if match(ds, r) else old).append(r)
        cur_revision = max([H.revision_of(r) for r in old] or [0]) + 1
        if not current:
            cur = await self.snapshot(ds, cur_revision)
        else:
            cur = await self.dedup_current(ds, current)
            if H.revision_of(cur) < cur_revision:
                cur = await self.client.update(dict(m.deepcopy(cur), revision=cur_revision, apiVersion="apps/v1",
                                                    kind="ControllerRevision"))
        return cur, old

    async def dedup_current(self, ds, current: list):
        if len(current) == 1:
            return current[0]
        keep = None
        for r in current:
            if keep is None or H.revision_of(r) >= H.revision_of(keep):
                keep = r
        keep_hash = m.labels_of(keep).get(HASH_LABEL)
        for r in current:
            if m.name_of(r) == m.name_of(keep):
                continue
            for p in await self.daemon_pods(ds):
                if m.labels_of(p).get(HASH_LABEL) != keep_hash:
                    p = m.deepcopy(p)
                    p["metadata"].setdefault("labels", {})[HASH_LABEL] = keep_hash
                    await self.client.update(dict(p, apiVersion="v1", kind="Pod"))
            await self.client.delete(H.History.resource, m.name_of(r), m.namespace_of(ds))
        return keep

    async def snapshot(self, ds, revision: int):
        tpl = _spec(ds).get("template") or {}
        hash_ = compute_hash(tpl, _status(ds).get("collisionCount"))
        name = f"{m.name_of(ds)}-{safe_encode(hash_)}"
        labels = dict((tpl.get("metadata") or {}).get("labels") or {})
        labels[HASH_LABEL] = hash_
        rev = {"apiVersion": "apps/v1", "kind": "ControllerRevision",
               "metadata": {"name": name, "namespace": m.namespace_of(ds), "labels": labels,
                            "annotations": dict(m.annotations_of(ds) or {}),
                            "ownerReferences": [m.new_controller_ref(ds, self.api_version, self.kind)]},
               "data": get_patch(ds), "revision": int(revision)}
        try:
            return await self.client.create(rev, m.namespace_of(ds))
        except m.StatusError as e:
            if not m.is_already_exists(e):
                raise
            existing = await self.client.get(H.History.resource, name, m.namespace_of(ds))
            if match(ds, existing):
                return existing
            cur_ds = await self.client.get("daemonsets", m.name_of(ds), m.namespace_of(ds))
            st = cur_ds.setdefault("status", {})
            st["collisionCount"] = int(st.get("collisionCount") or 0) + 1
            await self.client.update(dict(cur_ds, apiVersion=cur_ds.get("apiVersion") or self.api_version,
                                          kind=self.kind), "status")
            raise

    async def cleanup_history(self, ds, old: list):
        node_pods = await self.nodes_to_daemon_pods(ds)
        to_kill = len(old) - int(_spec(ds).get("revisionHistoryLimit", 10))
        if to_kill <= 0:
            return
        live = {m.labels_of(p).get(HASH_LABEL) for pods in node_pods.values() for p in pods} - {None, ""}
        for r in sorted(old, key=H.revision_of):
            if to_kill <= 0:
                break
            if m.labels_of(r).get(HASH_LABEL) in live:
                continue
            await self.client.delete(H.History.resource, m.name_of(r), m.namespace_of(ds))
            to_kill -= 1
