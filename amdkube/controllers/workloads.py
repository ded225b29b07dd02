"""Workload controllers: ReplicaSet, Deployment, DaemonSet, Job.

Reference: pkg/controller/replicaset (manage replicas via controllerRef + expectations),
pkg/controller/deployment (ReplicaSets per pod-template-hash; Recreate / RollingUpdate),
pkg/controller/daemon (one pod per eligible node — how the AMD device plugin is rolled
out, deploy/amd-gpu-device-plugin.yaml), pkg/controller/job (parallelism / completions /
backoffLimit). Slimmed to the behaviour the GPU-pod path needs (P1).
"""
from __future__ import annotations

import hashlib
import json

from ..api import meta as m
from ..api.helpers import find_untolerated_taint, is_pod_ready, is_pod_terminal
from ..api.labels import node_requirements_as_selector, selector_from_label_selector
from .base import Controller, split_key


def _owned(pods, owner):
    uid = m.uid_of(owner)
    return [p for p in pods if (m.controller_ref(p) or {}).get("uid") == uid]


def _pod_from_template(owner, api_version, kind, extra_labels=None, node=None):
    tpl = json.loads(json.dumps((owner.get("spec") or {}).get("template") or {}))
    md = tpl.get("metadata") or {}
    labels = dict(md.get("labels") or {})
    labels.update(extra_labels or {})
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"generateName": m.name_of(owner) + "-", "namespace": m.namespace_of(owner), "labels": labels,
                        "annotations": dict(md.get("annotations") or {}),
                        "ownerReferences": [m.new_controller_ref(owner, api_version, kind)]},
           "spec": tpl.get("spec") or {}}
    if node:
        pod["spec"]["nodeName"] = node
    return pod


class ReplicaSetController(Controller):
    name = "replicaset"
    burst = 500
    owner_api, owner_kind, plural = "apps/v1", "ReplicaSet", "replicasets"

    def setup(self):
        f = self.mgr.factory
        self.rs_inf = f.informer("replicasets")
        self.pod_inf = self.mgr.pods
        self.rs_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _pod(self, pod):
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "ReplicaSet":
            self.enqueue(f"{m.namespace_of(pod)}/{ref['name']}")

    async def sync(self, key):
        rs = self.rs_inf.get(key)
        if rs is None or (rs.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        pods = [p for p in _owned(self.pod_inf.list(), rs) if not is_pod_terminal(p)
                and not (p.get("metadata") or {}).get("deletionTimestamp")]
        want = int((rs.get("spec") or {}).get("replicas", 1))
        diff = want - len(pods)
        if diff > 0:
            for _ in range(min(diff, self.burst)):
                await self.client.create(_pod_from_template(rs, self.owner_api, self.owner_kind), ns)
        elif diff < 0:
            # delete not-ready / unscheduled pods first (controller_utils ActivePods ordering)
            pods.sort(key=lambda p: (bool((p.get("spec") or {}).get("nodeName")), is_pod_ready(p),
                                     (p.get("metadata") or {}).get("creationTimestamp", "")))
            for p in pods[:-diff]:
                try:
                    await self.client.delete("pods", m.name_of(p), ns)
                except m.StatusError:
                    pass
        ready = sum(1 for p in pods if is_pod_ready(p))
        st = {"replicas": len(pods), "readyReplicas": ready, "availableReplicas": ready,
              "fullyLabeledReplicas": len(pods), "observedGeneration": (rs.get("metadata") or {}).get("generation", 1)}
        if {k: (rs.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch(self.plural, name, {"status": st}, ns, sub="status")


def template_hash(tpl) -> str:
    return hashlib.sha1(json.dumps(tpl, sort_keys=True).encode()).hexdigest()[:10]


class DeploymentController(Controller):
    name = "deployment"

    def setup(self):
        f = self.mgr.factory
        self.d_inf = f.informer("deployments")
        self.rs_inf = f.informer("replicasets")
        self.d_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.rs_inf.add_handler(on_add=self._rs, on_update=lambda o, n: self._rs(n), on_delete=self._rs)

    def _rs(self, rs):
        ref = m.controller_ref(rs)
        if ref and ref.get("kind") == "Deployment":
            self.enqueue(f"{m.namespace_of(rs)}/{ref['name']}")

    async def sync(self, key):
        d = self.d_inf.get(key)
        if d is None or (d.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec = d.get("spec") or {}
        h = template_hash(spec.get("template") or {})
        rss = _owned(self.rs_inf.list(), d)
        cur = next((r for r in rss if m.labels_of(r).get("pod-template-hash") == h), None)
        want = int(spec.get("replicas", 1))
        if cur is None:
            tpl = json.loads(json.dumps(spec.get("template") or {}))
            tpl.setdefault("metadata", {}).setdefault("labels", {})["pod-template-hash"] = h
            sel = json.loads(json.dumps(spec.get("selector") or {}))
            sel.setdefault("matchLabels", {})["pod-template-hash"] = h
            rs = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
                  "metadata": {"name": f"{name}-{h}", "namespace": ns, "labels": {**(tpl["metadata"]["labels"])},
                               "ownerReferences": [m.new_controller_ref(d, "apps/v1", "Deployment")]},
                  "spec": {"replicas": want, "selector": sel, "template": tpl}}
            cur = await self.client.create(rs, ns)
        elif int((cur.get("spec") or {}).get("replicas", 0)) != want:
            await self.client.patch("replicasets", m.name_of(cur), {"spec": {"replicas": want}}, ns)
        old_ready = 0
        for r in rss:
            if r is cur or m.name_of(r) == m.name_of(cur):
                continue
            if int((r.get("spec") or {}).get("replicas", 0)) != 0:
                # Recreate: drop old immediately; RollingUpdate: drop once the new RS is fully ready
                new_ready = int((cur.get("status") or {}).get("readyReplicas", 0))
                if (spec.get("strategy") or {}).get("type") == "Recreate" or new_ready >= want:
                    await self.client.patch("replicasets", m.name_of(r), {"spec": {"replicas": 0}}, ns)
            old_ready += int((r.get("status") or {}).get("readyReplicas", 0))
        cst = cur.get("status") or {}
        st = {"replicas": int(cst.get("replicas", 0)) + old_ready, "updatedReplicas": int(cst.get("replicas", 0)),
              "readyReplicas": int(cst.get("readyReplicas", 0)) + old_ready, "availableReplicas": int(cst.get("availableReplicas", 0)),
              "observedGeneration": (d.get("metadata") or {}).get("generation", 1)}
        if {k: (d.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch("deployments", name, {"status": st}, ns, sub="status")


class DaemonSetController(Controller):
    name = "daemonset"

    def setup(self):
        f = self.mgr.factory
        self.ds_inf = f.informer("daemonsets")
        self.node_inf = self.mgr.nodes
        self.pod_inf = self.mgr.pods
        self.ds_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.node_inf.add_handler(on_add=lambda n: self._all(), on_update=lambda o, n: self._all(), on_delete=lambda n: self._all())
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _all(self):
        for ds in self.ds_inf.list():
            self.enqueue(ds)

    def _pod(self, pod):
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "DaemonSet":
            self.enqueue(f"{m.namespace_of(pod)}/{ref['name']}")

    @staticmethod
    def should_run(ds, node) -> bool:
        spec = ((ds.get("spec") or {}).get("template") or {}).get("spec") or {}
        labels = m.labels_of(node)
        for k, v in (spec.get("nodeSelector") or {}).items():
            if labels.get(k) != v:
                return False
        terms = ((((spec.get("affinity") or {}).get("nodeAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or {})
                 .get("nodeSelectorTerms") or [])
        if terms and not any(node_requirements_as_selector(t.get("matchExpressions")).matches(labels) for t in terms):
            return False
        return find_untolerated_taint((node.get("spec") or {}).get("taints"), spec.get("tolerations"),
                                      ("NoSchedule", "NoExecute")) is None

    async def sync(self, key):
        ds = self.ds_inf.get(key)
        if ds is None or (ds.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        pods = [p for p in _owned(self.pod_inf.list(), ds) if not (p.get("metadata") or {}).get("deletionTimestamp")]
        by_node: dict[str, list] = {}
        for p in pods:
            by_node.setdefault((p.get("spec") or {}).get("nodeName", ""), []).append(p)
        desired = current = ready = 0
        for node in self.node_inf.list():
            nn = m.name_of(node)
            run = self.should_run(ds, node)
            have = [p for p in by_node.get(nn, []) if not is_pod_terminal(p)]
            if run:
                desired += 1
                if not have:
                    await self.client.create(_pod_from_template(ds, "apps/v1", "DaemonSet", node=nn), ns)
                else:
                    current += 1
                    ready += sum(1 for p in have[:1] if is_pod_ready(p))
                    for extra in have[1:]:
                        await self.client.delete("pods", m.name_of(extra), ns)
            else:
                for p in have:
                    await self.client.delete("pods", m.name_of(p), ns)
            for p in by_node.get(nn, []):
                if is_pod_terminal(p) and run:
                    await self.client.delete("pods", m.name_of(p), ns, grace=0)
        st = {"desiredNumberScheduled": desired, "currentNumberScheduled": current, "numberReady": ready,
              "numberMisscheduled": 0, "observedGeneration": (ds.get("metadata") or {}).get("generation", 1)}
        if {k: (ds.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch("daemonsets", name, {"status": st}, ns, sub="status")


class JobController(Controller):
    name = "job"

    def setup(self):
        f = self.mgr.factory
        self.job_inf = f.informer("jobs")
        self.pod_inf = self.mgr.pods
        self.job_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _pod(self, pod):
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "Job":
            self.enqueue(f"{m.namespace_of(pod)}/{ref['name']}")

    async def sync(self, key):
        job = self.job_inf.get(key)
        if job is None or (job.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        st = job.get("status") or {}
        if any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True" for c in st.get("conditions") or []):
            return
        spec = job.get("spec") or {}
        pods = _owned(self.pod_inf.list(), job)
        succeeded = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Succeeded")
        failed = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Failed")
        active = [p for p in pods if not is_pod_terminal(p) and not (p.get("metadata") or {}).get("deletionTimestamp")]
        completions, parallelism = int(spec.get("completions", 1)), int(spec.get("parallelism", 1))
        new = {"succeeded": succeeded, "failed": failed, "active": len(active), "startTime": st.get("startTime") or m.now_rfc3339()}
        conds = []
        if succeeded >= completions:
            conds = [{"type": "Complete", "status": "True", "lastTransitionTime": m.now_rfc3339()}]
            new["completionTime"] = m.now_rfc3339()
            for p in active:
                await self.client.delete("pods", m.name_of(p), ns)
            new["active"] = 0
        elif failed > int(spec.get("backoffLimit", 6)):
            conds = [{"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                      "message": "Job has reached the specified backoff limit", "lastTransitionTime": m.now_rfc3339()}]
            for p in active:
                await self.client.delete("pods", m.name_of(p), ns)
            new["active"] = 0
        else:
            want = min(parallelism, completions - succeeded) - len(active)
            for _ in range(max(0, want)):
                await self.client.create(_pod_from_template(job, "batch/v1", "Job", {"job-name": name}), ns)
            new["active"] = len(active) + max(0, want)
        if conds:
            new["conditions"] = conds
        if {k: st.get(k) for k in new if k not in ("startTime",)} != {k: v for k, v in new.items() if k != "startTime"}:
            await self.client.patch("jobs", name, {"status": new}, ns, sub="status")
