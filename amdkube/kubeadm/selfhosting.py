"""kubeadm self-hosting: turn the static-Pod control plane into DaemonSets that the cluster runs
itself (reference: cmd/kubeadm/app/phases/selfhosting/selfhosting.go CreateSelfHostedControlPlane,
podspec_mutation.go; `kubeadm init --feature-gates SelfHosting=true` and
`kubeadm alpha phase selfhosting convert-from-staticpods`).

For each of kube-apiserver, kube-controller-manager and kube-scheduler, in that order:
  1. read its static Pod manifest (skipped when the file is gone: the conversion is idempotent);
  2. mutate the PodSpec for self-hosting: the master nodeSelector, the master toleration,
     dnsPolicy ClusterFirstWithHostNet;
  3. create or update DaemonSet kube-system/self-hosted-<component> (labels
     k8s-app=self-hosted-<component>, RollingUpdate) — retried, the API may blink;
  4. wait until its Pods run;
  5. remove the static manifest, wait for the mirror Pod <component>-<node> to go (the kubelet
     stopped the static copy) and for the API to answer healthy again.

amdkube specifics:
  * The apiserver over the embedded store (no --etcd-servers) owns its data directory
    exclusively (store/mvcc.py lock_data_dir). Its self-hosted copy therefore starts blocked on
    that lock (--data-dir-lock-wait 600) and takes over the moment the static copy exits, with
    the same WAL. An apiserver on etcd has no such hand-off.
  * Both copies of the apiserver want the same host port. The self-hosted one is "running"
    while it waits for the lock, which is the state step 4 waits for. It binds after the hand-off.
  * StoreCertsInSecrets (certificates as Secrets, projected volumes) is not implemented: the
    self-hosted Pods read the same host paths as the static ones.
"""
from __future__ import annotations

import asyncio
import os
import time

import yaml

from ..api import meta as m

PREFIX = "self-hosted-"
COMPONENTS = ("kube-apiserver", "kube-controller-manager", "kube-scheduler")
MASTER_LABEL = "node-role.kubernetes.io/master"
LOCK_WAIT = "600"


def labels(component: str) -> dict:
    return {"k8s-app": PREFIX + component}


def mutate_pod_spec(component: str, spec: dict) -> dict:
    """podspec_mutation.go's default mutators, plus the store hand-off for the apiserver."""
    spec.setdefault("nodeSelector", {})[MASTER_LABEL] = ""
    tol = {"key": MASTER_LABEL, "effect": "NoSchedule"}
    if tol not in (spec.get("tolerations") or []):
        spec["tolerations"] = [*(spec.get("tolerations") or []), tol]
    spec["dnsPolicy"] = "ClusterFirstWithHostNet"
    if component == "kube-apiserver":
        for ct in spec.get("containers") or []:
            args = ct.get("args") or []
            if "--data-dir" in args and "--data-dir-lock-wait" not in args:
                ct["args"] = [*args, "--data-dir-lock-wait", LOCK_WAIT]
    return spec


def build_daemonset(component: str, pod_spec: dict) -> dict:
    spec = mutate_pod_spec(component, dict(pod_spec))
    return {"apiVersion": "apps/v1", "kind": "DaemonSet",
            "metadata": {"name": PREFIX + component, "namespace": "kube-system", "labels": labels(component)},
            "spec": {"selector": {"matchLabels": labels(component)},
                     "template": {"metadata": {"labels": labels(component)}, "spec": spec},
                     "updateStrategy": {"type": "RollingUpdate"}}}


async def _retry(fn, attempts: int = 5, delay: float = 1.0):
    for i in range(attempts):
        try:
            return await fn()
        except (m.StatusError, OSError, asyncio.TimeoutError) as e:
            if i == attempts - 1 or (isinstance(e, m.StatusError) and e.code < 500 and e.code != 409):
                raise
            await asyncio.sleep(delay)


async def create_or_update_daemonset(c, ds: dict):
    async def once():
        cur = await c.get_or_none("daemonsets.apps", ds["metadata"]["name"], "kube-system")
        if cur is None:
            return await c.create(ds, "kube-system")
        ds["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return await c.update(ds)
    return await _retry(once)


async def _poll(cond, timeout: float, interval: float = 0.3) -> bool:
    """cond() until true; API errors while the apiserver itself is changing hands count as 'not yet'."""
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            if await cond():
                return True
        except Exception:         # noqa: BLE001 — connection refused/reset during the hand-off
            pass
        await asyncio.sleep(interval)
    return False


async def pods_running(c, component: str) -> bool:
    pods, _ = await c.list("pods", "kube-system", label_selector=f"k8s-app={PREFIX}{component}")
    return bool(pods) and all((p.get("status") or {}).get("phase") == "Running" for p in pods)


async def api_healthy(c) -> bool:
    import aiohttp
    async with c.session.get(f"{c.server}/healthz", timeout=aiohttp.ClientTimeout(total=5)) as r:
        return r.status == 200


async def create_self_hosted_control_plane(c, manifests_dir: str, node_name: str, timeout: float = 120.0,
                                           dry_run: bool = False, out=print) -> list[str]:
    """Convert every static control-plane Pod still on disk; returns the components converted."""
    done = []
    for comp in COMPONENTS:
        t0 = time.monotonic()
        path = os.path.join(manifests_dir, f"{comp}.yaml")
        if not os.path.exists(path):
            out(f"[self-hosted] The Static Pod for the component {comp!r} doesn't seem to be on the disk; trying the next one")
            continue
        with open(path) as f:
            pod = yaml.safe_load(f) or {}
        ds = build_daemonset(comp, pod.get("spec") or {})
        if dry_run:
            out(yaml.safe_dump(ds, sort_keys=False))
            continue
        await create_or_update_daemonset(c, ds)
        if not await _poll(lambda: pods_running(c, comp), timeout):
            raise TimeoutError(f"the self-hosted {comp} Pods did not start within {timeout:.0f}s")
        os.remove(path)
        if not await _poll(lambda: _gone(c, f"{comp}-{node_name}"), timeout):
            raise TimeoutError(f"the static Pod {comp}-{node_name} did not go away within {timeout:.0f}s")
        if not await _poll(lambda: api_healthy(c), timeout):
            raise TimeoutError(f"the API server did not become healthy within {timeout:.0f}s after converting {comp}")
        out(f"[self-hosted] self-hosted {comp} ready after {time.monotonic() - t0:.1f} seconds")
        done.append(comp)
    return done


async def _gone(c, name: str) -> bool:
    return await c.get_or_none("pods", name, "kube-system") is None
