"""kubectl cordon / uncordon / drain.

Reference: pkg/kubectl/cmd/drain.go —
  * SetupDrain (:206-268): one NODE or `-l selector` over nodes, never both;
  * RunCordonOrUncordon (:681-740): `node "x" already cordoned` when nothing changes, else a
    strategic-merge patch of spec.unschedulable and `node "x" cordoned`; --dry-run touches
    nothing;
  * RunDrain (:271-309): cordon, then per node getPodsForDeletion → deleteOrEvictPods; the first
    node that fails aborts the command, listing the nodes still pending;
  * getPodsForDeletion (:457-492) runs every pod on the node through mirrorPodFilter (mirror
    pods are skipped silently), localStorageFilter (emptyDir: fatal without
    --delete-local-data), unreplicatedFilter (finished pods always go; a pod without a
    controller is fatal without --force; a controller that no longer exists is a warning with
    --force, else fatal) and daemonsetFilter (DaemonSet pods are never deleted; fatal without
    --ignore-daemonsets); fatal messages abort before anything is evicted, warnings print as
    `WARNING: ...`;
  * deleteOrEvictPods (:525-616): the eviction subresource when discovery offers it
    (SupportEviction :649-677), retried every 5 s while a PodDisruptionBudget answers 429, a
    pod already gone counts as done; plain DELETE otherwise; each with --grace-period;
  * waitForDelete (:618-645): polled every second until the pod is gone or replaced (new UID),
    printing `pod "x" evicted|deleted`; --timeout (0 = forever) bounds the whole node.
"""
from __future__ import annotations

import asyncio
import sys
import time

from ..api import meta as m

K_DAEMONSET_FATAL = "DaemonSet-managed pods (use --ignore-daemonsets to ignore)"
K_DAEMONSET_WARNING = "Ignoring DaemonSet-managed pods"
K_LOCAL_STORAGE_FATAL = "pods with local storage (use --delete-local-data to override)"
K_LOCAL_STORAGE_WARNING = "Deleting pods with local storage"
K_UNMANAGED_FATAL = ("pods not managed by ReplicationController, ReplicaSet, Job, DaemonSet or StatefulSet "
                     "(use --force to override)")
K_UNMANAGED_WARNING = "Deleting pods not managed by ReplicationController, ReplicaSet, Job, DaemonSet or StatefulSet"
MIRROR_ANNOTATION = "kubernetes.io/config.mirror"
CONTROLLER_RESOURCES = {"ReplicationController": "replicationcontrollers", "DaemonSet": "daemonsets", "Job": "jobs",
                        "ReplicaSet": "replicasets", "StatefulSet": "statefulsets"}
INTERVAL = 1.0            # kubectl.Interval
EVICTION_RETRY = 5.0      # the 429 back-off of evictPods


class DrainError(Exception):
    pass


def print_success(resource: str, name: str, operation: str, dry_run: bool = False, short: bool = False, out=None):
    """PrintSuccess (factory_builder.go:85-106)."""
    out = out or sys.stdout
    if short:
        print(f"{resource}/{name}" if resource else name, file=out)
    else:
        print((f'{resource} "{name}" ' if resource else f'"{name}" ') + operation + (" (dry run)" if dry_run else ""), file=out)


class Drainer:
    def __init__(self, client, *, force=False, ignore_daemonsets=False, delete_local_data=False, grace_period=-1,
                 timeout=0.0, dry_run=False, out=None, err=None, interval=INTERVAL, eviction_retry=EVICTION_RETRY):
        self.c = client
        self.force, self.ignore_daemonsets, self.delete_local_data = force, ignore_daemonsets, delete_local_data
        self.grace_period, self.timeout, self.dry_run = grace_period, timeout, dry_run
        self.out, self.err = out or sys.stdout, err or sys.stderr
        self.interval, self.eviction_retry = interval, eviction_retry

    # ----------------------------------------------------------------- filters
    async def _controller_of(self, pod):
        """getPodController: the controller reference, after checking the controller exists
        (its NotFound error is passed up)."""
        ref = m.controller_ref(pod)
        if ref is None:
            return None
        res = CONTROLLER_RESOURCES.get(ref.get("kind", ""))
        if res is None:
            raise DrainError(f'Unknown controller kind "{ref.get("kind", "")}"')
        await self.c.get(res, ref.get("name", ""), m.namespace_of(pod))
        return ref

    @staticmethod
    def mirror_pod_filter(pod):
        return MIRROR_ANNOTATION not in m.annotations_of(pod), None, None

    def local_storage_filter(self, pod):
        if not any("emptyDir" in v for v in (pod.get("spec") or {}).get("volumes") or []):
            return True, None, None
        if not self.delete_local_data:
            return False, None, K_LOCAL_STORAGE_FATAL
        return True, K_LOCAL_STORAGE_WARNING, None

    async def unreplicated_filter(self, pod):
        if (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
            return True, None, None
        try:
            ref = await self._controller_of(pod)
        except m.StatusError as e:
            if m.is_not_found(e) and self.force:
                return True, e.message, None
            return False, None, e.message
        except DrainError as e:
            return False, None, str(e)
        if ref is not None:
            return True, None, None
        if not self.force:
            return False, None, K_UNMANAGED_FATAL
        return True, K_UNMANAGED_WARNING, None

    async def daemonset_filter(self, pod):
        try:
            ref = await self._controller_of(pod)
        except m.StatusError as e:
            if m.is_not_found(e) and self.force:
                return True, e.message, None
            return False, None, e.message
        except DrainError as e:
            return False, None, str(e)
        if ref is None or ref.get("kind") != "DaemonSet":
            return True, None, None
        if not self.ignore_daemonsets:
            return False, None, K_DAEMONSET_FATAL
        return False, K_DAEMONSET_WARNING, None

    async def pods_for_deletion(self, node: str) -> list[dict]:
        """getPodsForDeletion: DrainError carries the fatal messages."""
        items, _ = await self.c.list("pods", "", field_selector=f"spec.nodeName={node}")
        warnings: dict[str, list[str]] = {}
        fatals: dict[str, list[str]] = {}
        keep = []
        for pod in items:
            ok = True
            results = [self.mirror_pod_filter(pod), self.local_storage_filter(pod), await self.unreplicated_filter(pod),
                       await self.daemonset_filter(pod)]
            for include, w, f in results:
                ok = ok and include
                if w:
                    warnings.setdefault(w, []).append(m.name_of(pod))
                if f:
                    fatals.setdefault(f, []).append(m.name_of(pod))
            if ok:
                keep.append(pod)
        if fatals:
            raise DrainError("; ".join(f"{k}: {', '.join(v)}" for k, v in fatals.items()))
        if warnings:
            print("WARNING: " + "; ".join(f"{k}: {', '.join(v)}" for k, v in warnings.items()), file=self.err)
        return keep

    # ------------------------------------------------------------ evict/delete
    async def supports_eviction(self) -> bool:
        """SupportEviction: the policy group is served and v1 lists pods/eviction."""
        try:
            groups = await self.c.request("GET", "/apis")
            if not any(g.get("name") == "policy" for g in (groups or {}).get("groups") or []):
                return False
            core = await self.c.request("GET", "/api/v1")
        except m.StatusError:
            return False
        return any(r.get("name") == "pods/eviction" and r.get("kind") == "Eviction" for r in (core or {}).get("resources") or [])

    async def _evict(self, pod):
        body = {"apiVersion": "policy/v1beta1", "kind": "Eviction",
                "metadata": {"name": m.name_of(pod), "namespace": m.namespace_of(pod)}}
        if self.grace_period >= 0:
            body["deleteOptions"] = {"gracePeriodSeconds": self.grace_period}
        ri = self.c.resource_info("pods")
        return await self.c.request("POST", self.c.path(ri, m.namespace_of(pod), m.name_of(pod), "eviction"), body=body)

    async def wait_for_delete(self, pods: list[dict], verb: str, timeout: float | None) -> list[dict]:
        """waitForDelete: the pods still present when `timeout` ran out (TimeoutError), else []."""
        end = None if not timeout else time.monotonic() + timeout
        while True:
            pending = []
            for pod in pods:
                cur = await self.c.get_or_none("pods", m.name_of(pod), m.namespace_of(pod))
                if cur is None or m.uid_of(cur) != m.uid_of(pod):
                    print_success("pod", m.name_of(pod), verb, out=self.out)
                else:
                    pending.append(pod)
            pods = pending
            if not pods:
                return []
            if end is not None and time.monotonic() >= end:
                raise TimeoutError("timed out waiting for the condition")
            await asyncio.sleep(self.interval)

    async def evict_pods(self, pods: list[dict]):
        async def one(pod):
            while True:
                try:
                    await self._evict(pod)
                    break
                except m.StatusError as e:
                    if m.is_not_found(e):
                        return
                    if e.code == 429:
                        await asyncio.sleep(self.eviction_retry)
                        continue
                    raise DrainError(f'error when evicting pod "{m.name_of(pod)}": {e.message}') from None
            try:
                await self.wait_for_delete([pod], "evicted", None)
            except Exception as e:
                raise DrainError(f'error when waiting for pod "{m.name_of(pod)}" terminating: {e}') from None
        tasks = [asyncio.ensure_future(one(p)) for p in pods]
        try:
            done, pending = await asyncio.wait(tasks, timeout=self.timeout or None, return_when=asyncio.FIRST_EXCEPTION)
            for t in done:
                if t.exception() is not None:
                    raise t.exception()
            if pending:
                raise DrainError(f"Drain did not complete within {_go_duration(self.timeout)}")
        finally:
            for t in tasks:
                t.cancel()

    async def delete_pods(self, pods: list[dict]):
        for pod in pods:
            try:
                await self.c.delete("pods", m.name_of(pod), m.namespace_of(pod),
                                    grace=self.grace_period if self.grace_period >= 0 else None)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise DrainError(e.message) from None
        try:
            await self.wait_for_delete(pods, "deleted", self.timeout or None)
        except TimeoutError as e:
            raise DrainError(str(e)) from None

    async def delete_or_evict(self, pods: list[dict]):
        if not pods:
            return
        if await self.supports_eviction():
            await self.evict_pods(pods)
        else:
            await self.delete_pods(pods)

    async def drain_node(self, node: str):
        """deleteOrEvictPodsSimple."""
        pods = await self.pods_for_deletion(node)
        try:
            await self.delete_or_evict(pods)
        except DrainError as e:
            pending = await self.pods_for_deletion(node)
            print(f'There are pending pods in node "{node}" when an error occurred: {e}', file=self.err)
            for p in pending:
                print(f"pod/{m.name_of(p)}", file=self.err)
            raise

    # ------------------------------------------------------------ cordon/drain
    async def cordon(self, nodes: list[dict], desired: bool):
        """RunCordonOrUncordon."""
        for node in nodes:
            name = m.name_of(node)
            if bool((node.get("spec") or {}).get("unschedulable")) == desired:
                print_success("node", name, "already cordoned" if desired else "already uncordoned", self.dry_run, out=self.out)
                continue
            if not self.dry_run:
                await self.c.patch("nodes", name, {"spec": {"unschedulable": True if desired else None}},
                                   patch_type="application/strategic-merge-patch+json")
            print_success("node", name, "cordoned" if desired else "uncordoned", self.dry_run, out=self.out)

    async def drain(self, nodes: list[dict]):
        """RunDrain."""
        await self.cordon(nodes, True)
        drained = set()
        for node in nodes:
            name = m.name_of(node)
            try:
                if not self.dry_run:
                    await self.drain_node(name)
            except DrainError:
                print(f'error: unable to drain node "{name}", aborting command...\n', file=self.err)
                remaining = [m.name_of(n) for n in nodes if m.name_of(n) not in drained]
                if remaining:
                    print("There are pending nodes to be drained:", file=self.err)
                    for r in remaining:
                        print(f" {r}", file=self.err)
                raise
            drained.add(name)
            print_success("node", name, "drained", self.dry_run, out=self.out)


def _go_duration(s: float) -> str:
    if s >= 60 and s % 60 == 0:
        return f"{int(s // 60)}m0s"
    return f"{s:g}s"


async def _nodes(c, a, use: str) -> list[dict]:
    """SetupDrain: the NODE argument (`node/NAME` works too) or the --selector's nodes."""
    args = list(a.args)
    if not args and not a.selector:
        raise DrainError(f"USAGE: {use} [flags]")
    if args and a.selector:
        raise DrainError("error: cannot specify both a node name and a --selector option")
    if len(args) > 1:
        raise DrainError(f"USAGE: {use} [flags]")
    if args:
        ref = args[0]
        if "/" in ref:
            kind, ref = ref.split("/", 1)
            if kind not in ("node", "nodes", "no"):
                raise DrainError(f'error: expected resource of type node, got "{kind}"')
        return [await c.get("nodes", ref)]
    items, _ = await c.list("nodes", "", a.selector)
    return items


def _drainer(c, a) -> Drainer:
    from .main import timeout_of
    return Drainer(c, force=bool(getattr(a, "force", False)), ignore_daemonsets=bool(a.ignore_daemonsets),
                   delete_local_data=bool(getattr(a, "delete_local_data", False)), grace_period=a.grace_period,
                   timeout=timeout_of(a, 0.0), dry_run=bool(getattr(a, "dry_run", False)))


async def cmd_cordon(c, a):
    try:
        await _drainer(c, a).cordon(await _nodes(c, a, "cordon NODE"), True)
    except DrainError as e:
        print(str(e) if str(e).startswith(("error:", "USAGE")) else f"error: {e}", file=sys.stderr)
        return 1
    return 0


async def cmd_uncordon(c, a):
    try:
        await _drainer(c, a).cordon(await _nodes(c, a, "uncordon NODE"), False)
    except DrainError as e:
        print(str(e) if str(e).startswith(("error:", "USAGE")) else f"error: {e}", file=sys.stderr)
        return 1
    return 0


async def cmd_drain(c, a):
    d = _drainer(c, a)
    try:
        nodes = await _nodes(c, a, "drain NODE")
        await d.drain(nodes)
    except DrainError as e:
        msg = str(e)
        print(msg if msg.startswith(("error:", "USAGE")) else f"error: {msg}", file=sys.stderr)
        return 1
    return 0


def add_arguments(sp):
    sp.add_argument("--delete-local-data", action="store_true")
