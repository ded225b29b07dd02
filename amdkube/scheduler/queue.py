"""Scheduling queue: PriorityQueue with an unschedulable sub-queue and nominated pods.

Reference: plugin/pkg/scheduler/core/scheduling_queue.go:163-468 — activeQ ordered by pod
priority (then arrival), unschedulableQ parked until a cluster event (node add/update,
assigned pod deleted/terminated) calls MoveAllToActiveQueue (receivedMoveRequest sends a pod
that failed during such an event straight back to activeQ); nominatedPods, node name -> pods
nominated to run there after a preemption (addNominatedPodIfNeeded / deleteNominatedPodIfExists
/ updateNominatedPod, WaitingPodsForNode), kept for pods in either sub-queue and dropped when a
pod is popped for scheduling; Update moves an unschedulable pod back to activeQ only when its
spec or metadata changed (isPodUpdated); AssignedPodAdded/Updated move the unschedulable pods
whose pod-affinity terms the bound pod matches. FIFO order without the PodPriority gate.
Unschedulable pods are also retried on a timer so nothing is stranded.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools

from ..api import meta as m

NOMINATED_NODE_ANNOTATION = "NominatedNodeName"


def nominated_node_name(pod: dict) -> str:
    return ((pod.get("metadata") or {}).get("annotations") or {}).get(NOMINATED_NODE_ANNOTATION) or ""


def is_pod_unschedulable(pod: dict) -> bool:
    return any(c.get("type") == "PodScheduled" and c.get("status") == "False" and c.get("reason") == "Unschedulable"
               for c in (pod.get("status") or {}).get("conditions") or [])


def _strip(pod: dict) -> dict:
    md = {k: v for k, v in (pod.get("metadata") or {}).items() if k not in ("resourceVersion", "generation")}
    return {k: v for k, v in pod.items() if k != "status"} | {"metadata": md}


def is_pod_updated(old: dict | None, new: dict) -> bool:
    """isPodUpdated (:321-333): a change other than status / resourceVersion / generation."""
    return old is None or _strip(old) != _strip(new)


class SchedulingQueue:
    def __init__(self, use_priority: bool = True, unschedulable_retry: float = 30.0):
        self.use_priority = use_priority
        self.heap: list = []
        self.items: dict[str, dict] = {}
        self.unschedulable: dict[str, dict] = {}
        self.nominated: dict[str, dict[str, dict]] = {}    # node -> pod key -> pod
        self._nominated_of: dict[str, str] = {}             # pod key -> node
        self.seq = itertools.count()
        self._waiters: list[asyncio.Future] = []
        self.retry = unschedulable_retry
        self.received_move = False

    def __len__(self):
        return len(self.items)

    def _prio(self, pod):
        return -int((pod.get("spec") or {}).get("priority") or 0) if self.use_priority else 0

    # ---------------------------------------------------------------- nominated pods
    def _add_nominated(self, pod: dict):
        node = nominated_node_name(pod)
        key = m.key_of(pod)
        if not node:
            return
        self._nominated_of[key] = node
        self.nominated.setdefault(node, {})[key] = pod

    def _delete_nominated(self, key: str):
        node = self._nominated_of.pop(key, None)
        if node is None:
            return
        pods = self.nominated.get(node)
        if pods is not None:
            pods.pop(key, None)
            if not pods:
                del self.nominated[node]

    def _update_nominated(self, pod: dict):
        self._delete_nominated(m.key_of(pod))
        self._add_nominated(pod)

    def waiting_pods_for_node(self, node: str) -> list:
        """WaitingPodsForNode: pods nominated to run on `node` once its victims are gone."""
        pods = self.nominated.get(node)
        return list(pods.values()) if pods else []

    # ---------------------------------------------------------------- queue
    def add(self, pod: dict):
        key = m.key_of(pod)
        self.unschedulable.pop(key, None)
        self._update_nominated(pod)
        if key in self.items:
            self.items[key] = pod
            return
        self.items[key] = pod
        heapq.heappush(self.heap, (self._prio(pod), next(self.seq), key))
        self._wake()

    def update(self, pod: dict, old: dict | None = None):
        key = m.key_of(pod)
        if key in self.items:
            self.items[key] = pod
            self._update_nominated(pod)
        elif key in self.unschedulable:
            prev = self.unschedulable[key]
            if is_pod_updated(old if old is not None else prev, pod):
                self.unschedulable.pop(key)
                self.add(pod)
            else:
                self.unschedulable[key] = pod
                self._update_nominated(pod)
        else:
            self.add(pod)

    def delete(self, pod: dict):
        key = m.key_of(pod)
        self._delete_nominated(key)
        self.items.pop(key, None)
        self.unschedulable.pop(key, None)

    def add_unschedulable(self, pod: dict, marked: bool | None = None):
        """AddUnschedulableIfNotPresent: nothing if the pod is queued already; the unschedulable
        sub-queue if it is marked unschedulable (the PodScheduled=False/Unschedulable condition,
        or `marked` when the caller is setting that condition itself) and no move request came
        in while it was being scheduled; the active queue otherwise."""
        key = m.key_of(pod)
        if key in self.items or key in self.unschedulable:
            return
        if marked is None:
            marked = is_pod_unschedulable(pod)
        if self.received_move or not marked:
            self.received_move = False
            self.add(pod)
            return
        self.unschedulable[key] = pod
        self._update_nominated(pod)
        try:
            asyncio.get_running_loop().call_later(self.retry, self._retry_one, key)
        except RuntimeError:
            pass        # no loop (table tests): the timer retry is the asyncio scheduler's

    def _retry_one(self, key):
        pod = self.unschedulable.pop(key, None)
        if pod is not None:
            self.add(pod)

    def move_all_to_active(self):
        if not self.unschedulable:
            self.received_move = True
            return
        pods = list(self.unschedulable.values())
        self.unschedulable.clear()
        for p in pods:
            self.add(p)
        self.received_move = True

    def _move(self, pods):
        for p in pods:
            self.unschedulable.pop(m.key_of(p), None)
            self.add(p)
        self.received_move = True

    def assigned_pod_added(self, pod: dict):
        """AssignedPodAdded / AssignedPodUpdated: a bound pod may satisfy the pod affinity of
        unschedulable pods."""
        moves = self._matching_affinity(pod)
        if moves:
            self._move(moves)

    assigned_pod_updated = assigned_pod_added

    def _matching_affinity(self, pod: dict) -> list:
        from ..api.labels import SelectorError, selector_from_label_selector
        labels = m.labels_of(pod)
        out = []
        for up in self.unschedulable.values():
            pa = ((up.get("spec") or {}).get("affinity") or {}).get("podAffinity") or {}
            for term in pa.get("requiredDuringSchedulingIgnoredDuringExecution") or []:
                nss = term.get("namespaces") or [m.namespace_of(up)]
                if m.namespace_of(pod) not in nss:
                    continue
                try:
                    sel = selector_from_label_selector(term.get("labelSelector"))
                except SelectorError:
                    continue
                if sel.matches(labels):
                    out.append(up)
                    break
        return out

    def _wake(self):
        if not self._waiters:
            return
        while self._waiters:
            f = self._waiters.pop()
            if not f.done():
                f.set_result(None)
                return

    def pop_nowait(self):
        while self.heap:
            _, _, key = heapq.heappop(self.heap)
            pod = self.items.pop(key, None)
            if pod is not None:
                self._delete_nominated(key)
                return pod
        return None

    async def pop(self) -> dict:
        while True:
            pod = self.pop_nowait()
            if pod is not None:
                self.received_move = False
                return pod
            f = asyncio.get_running_loop().create_future()
            self._waiters.append(f)
            await f
