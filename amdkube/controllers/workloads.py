"""Workload controllers: ReplicaSet, Deployment, DaemonSet, Job.

Reference: pkg/controller/replicaset (manage replicas via controllerRef + expectations),
pkg/controller/deployment (ReplicaSets per pod-template-hash; Recreate / RollingUpdate),
pkg/controller/daemon (controllers/daemonset.py: one pod per eligible node — how the AMD
device plugin is rolled out, deploy/amd-gpu-device-plugin.yaml). The Job controller is in
controllers/job.py.
"""
from __future__ import annotations

import json

from ..api import meta as m


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


from .replicaset import ReplicaSetController  # noqa: E402,F401  (controllers/replicaset.py)


from .deployment import DeploymentController  # noqa: E402,F401  (controllers/deployment.py)


from .daemonset import DaemonSetController  # noqa: E402,F401  (controllers/daemonset.py)


from .job import JobController  # noqa: E402,F401  (moved to controllers/job.py)
