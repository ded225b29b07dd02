"""Cluster addon manager: keeps the manifests under an addon directory applied to the cluster.

Reference: cluster/addons/addon-manager/kube-addons.sh. Its loop (:120-146 and the main loop)
every ADDON_CHECK_INTERVAL_SEC:

  * `ensure_addons`: `kubectl create -f $ADDON_PATH -l addonmanager.kubernetes.io/mode=EnsureExists
    --recursive` — created when absent, never updated or deleted afterwards (AlreadyExists is
    quiet), so users may edit them;
  * `reconcile_addons`: two `kubectl apply --prune --recursive` passes in kube-system, one over
    `kubernetes.io/cluster-service=true,addonmanager.kubernetes.io/mode!=EnsureExists` (the
    deprecated label) and one over `kubernetes.io/cluster-service!=true,
    addonmanager.kubernetes.io/mode=Reconcile`: live objects follow the files, and objects of
    that label set that left the directory are pruned;
  * only the leader acts: the holder of kube-controller-manager's endpoints leader annotation
    (`control-plane.alpha.kubernetes.io/leader`), or everyone when that cannot be read;
  * at start it creates the kube-system namespace and waits for its default ServiceAccount,
    then creates every manifest under the admission-controls directory once.

Differences, on purpose: the loop is in-process over the client (kubectl's three-way apply and
pruner in kubectl/more.py, not a subprocess per pass); a pass whose selector matches no file
still prunes (kubectl's "no objects passed to apply" makes removing an addon's LAST manifest a
no-op in the reference); the prune list also covers the ServiceAccounts and RBAC objects that
addons ship (the later addon manager passes the same list as --prune-whitelist). deploy/addons/
holds this repo's addons: the AMD device plugin, the amdgpu exporter and the
node-problem-detector with its amdgpu rules.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import socket
import time

from .api import meta as m
from .api.scheme import SCHEME

log = logging.getLogger("amdkube.addons")

ADDON_MANAGER_LABEL = "addonmanager.kubernetes.io/mode"
CLUSTER_SERVICE_LABEL = "kubernetes.io/cluster-service"
LEADER_ANNOTATION = "control-plane.alpha.kubernetes.io/leader"
SYSTEM_NAMESPACE = "kube-system"

RECONCILE_DEPRECATED = f"{CLUSTER_SERVICE_LABEL}=true,{ADDON_MANAGER_LABEL}!=EnsureExists"
RECONCILE = f"{CLUSTER_SERVICE_LABEL}!=true,{ADDON_MANAGER_LABEL}=Reconcile"
ENSURE = f"{ADDON_MANAGER_LABEL}=EnsureExists"

PRUNE_WHITELIST = [
    "core/v1/ConfigMap", "core/v1/Endpoints", "core/v1/Namespace", "core/v1/PersistentVolumeClaim",
    "core/v1/PersistentVolume", "core/v1/Pod", "core/v1/ReplicationController", "core/v1/Secret",
    "core/v1/Service", "core/v1/ServiceAccount", "batch/v1/Job", "extensions/v1beta1/DaemonSet",
    "apps/v1beta2/Deployment", "extensions/v1beta1/Ingress", "extensions/v1beta1/ReplicaSet",
    "apps/v1beta1/StatefulSet", "rbac.authorization.k8s.io/v1/Role", "rbac.authorization.k8s.io/v1/RoleBinding",
    "rbac.authorization.k8s.io/v1/ClusterRole", "rbac.authorization.k8s.io/v1/ClusterRoleBinding",
]


class AddonManager:
    def __init__(self, client, addon_path: str, admission_controls: str | None = None, interval: float = 60.0,
                 leader_election: bool = True, identity: str | None = None, namespace_manifest: str | None = None):
        self.client, self.addon_path, self.admission_controls = client, addon_path, admission_controls
        self.interval, self.leader_election = interval, leader_election
        self.identity = identity or os.environ.get("HOSTNAME") or socket.gethostname()
        self.namespace_manifest = namespace_manifest
        self.passes = 0
        self.log_lines: list[str] = []
        self._task: asyncio.Task | None = None

    def _out(self, line: str):
        self.log_lines.append(line)
        if len(self.log_lines) > 1000:
            del self.log_lines[:500]
        if not line.endswith((" unchanged", " configured")):   # kube-addons.sh: `| grep -v configured`
            log.info("%s", line)

    def _docs(self, path: str) -> list[dict]:
        from .kubectl.main import _read_files
        if not os.path.exists(path):
            return []
        try:
            return _read_files([path], recursive=True)
        except Exception as e:   # a broken file must not stop the other addons
            log.error("reading addons under %s: %r", path, e)
            return []

    # ------------------------------------------------------------------ leader
    async def is_leader(self) -> bool:
        if not self.leader_election:
            return True
        try:
            ep = await self.client.get_or_none("endpoints", "kube-controller-manager", SYSTEM_NAMESPACE)
        except Exception:    # better several addon managers than none
            return True
        raw = m.annotations_of(ep).get(LEADER_ANNOTATION) if ep else None
        if not raw:
            return True
        try:
            holder = (json.loads(raw) or {}).get("holderIdentity") or ""
        except ValueError:
            return True
        return holder in ("", self.identity) or holder.split("_", 1)[0] == self.identity

    # ------------------------------------------------------------------ passes
    async def create_docs(self, docs: list[dict], namespace: str) -> int:
        """`kubectl create --namespace=<ns> -f …`: AlreadyExists is not an error."""
        created = 0
        for doc in docs:
            ri = SCHEME.for_object(doc)
            if ri is None:
                log.error("addon %s/%s: unknown kind", doc.get("apiVersion"), doc.get("kind"))
                continue
            ns = (m.namespace_of(doc) or namespace) if ri.namespaced else ""
            try:
                await self.client.create(doc, ns if ri.namespaced else None)
                created += 1
                self._out(f"{ri.kind.lower()}/{m.name_of(doc)} created")
            except m.StatusError as e:
                if e.code != 409:
                    log.warning("creating addon %s/%s: %s", ri.kind, m.name_of(doc), e)
        return created

    async def ensure_addons(self) -> int:
        from .api.labels import parse_selector
        sel = parse_selector(ENSURE)
        docs = [d for d in self._docs(self.addon_path) if sel.matches(m.labels_of(d))]
        return await self.create_docs(docs, SYSTEM_NAMESPACE)

    async def _apply_pass(self, docs: list[dict], selector: str):
        from .kubectl.more import apply_docs
        a = argparse.Namespace(selector=selector, namespace=SYSTEM_NAMESPACE, prune=True, all=False, force=False,
                               prune_whitelist=PRUNE_WHITELIST)
        try:
            await apply_docs(self.client, a, [json.loads(json.dumps(d)) for d in docs], out=self._out,
                             allow_empty=True)
        except (SystemExit, m.StatusError) as e:
            log.error("reconciling %s: %s", selector, e)

    async def reconcile_addons(self):
        docs = self._docs(self.addon_path)
        await self._apply_pass(docs, RECONCILE_DEPRECATED)
        await self._apply_pass(docs, RECONCILE)

    async def sync_once(self) -> bool:
        if not await self.is_leader():
            log.info("not elected leader, going back to sleep")
            return False
        await self.ensure_addons()
        await self.reconcile_addons()
        self.passes += 1
        return True

    # ------------------------------------------------------------------ startup
    async def bootstrap(self, timeout: float = 60.0):
        ns_doc = {"apiVersion": "v1", "kind": "Namespace",
                  "metadata": {"name": SYSTEM_NAMESPACE, "labels": {ADDON_MANAGER_LABEL: "EnsureExists"}}}
        if self.namespace_manifest:
            ns_docs = self._docs(self.namespace_manifest)
        else:
            ns_docs = [ns_doc]
        await self.create_docs(ns_docs, "")
        end = time.monotonic() + timeout
        while time.monotonic() < end:       # the token controller has run for kube-system
            sa = await self.client.get_or_none("serviceaccounts", "default", SYSTEM_NAMESPACE)
            if sa is not None:
                break
            await asyncio.sleep(0.5)
        else:
            log.warning("no default ServiceAccount in %s after %.0fs; continuing", SYSTEM_NAMESPACE, timeout)
        if self.admission_controls:
            await self.create_docs(self._docs(self.admission_controls), "default")

    async def start(self, bootstrap_timeout: float = 60.0):
        await self.bootstrap(bootstrap_timeout)
        self._task = asyncio.create_task(self._loop(), name="addon-manager")
        return self

    async def stop(self):
        from .utils import cancel_and_wait
        await cancel_and_wait([self._task])

    async def _loop(self):
        log.info("entering periodical apply loop (interval %.0fs, addons under %s)", self.interval, self.addon_path)
        while True:
            t0 = time.monotonic()
            try:
                await self.sync_once()
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.error("addon pass failed: %r", e)
            await asyncio.sleep(max(0.0, self.interval - (time.monotonic() - t0)))
