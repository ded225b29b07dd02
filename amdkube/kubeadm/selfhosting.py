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
  * StoreCertsInSecrets=true (selfhosting_volumes.go): the certificates and the scheduler's and
    controller-manager's kubeconfigs go to kube-system Secrets (ca, apiserver,
    apiserver-kubelet-client, sa, front-proxy-ca, front-proxy-client as kubernetes.io/tls with
    tls.crt/tls.key; controller-manager.conf and scheduler.conf as Opaque), and the DaemonSets
    read them from a projected volume `k8s-certs` over the certificates directory and a secret
    volume `kubeconfig` at <kubeconfig dir>/kubeconfig (--kubeconfig rewritten there, as the
    reference does). `sa` is Opaque with sa.key: amdkube's PKI writes no sa.pub. A process
    container without a mount namespace sees those volumes under $AMDKUBE_ROOTFS; the command
    line's absolute paths are resolved there first (amdkube/__main__.py).
  * Without StoreCertsInSecrets the self-hosted Pods read the same host paths as the static ones.
"""
from __future__ import annotations

import asyncio
import base64
import os
import time

import yaml

from ..api import meta as m

PREFIX = "self-hosted-"
COMPONENTS = ("kube-apiserver", "kube-controller-manager", "kube-scheduler")
MASTER_LABEL = "node-role.kubernetes.io/master"
LOCK_WAIT = "600"
CERTS_VOLUME, KUBECONFIG_VOLUME = "k8s-certs", "kubeconfig"
# getTLSKeyPairs: (secret, certificate file, key file)
TLS_PAIRS = (("ca", "ca.crt", "ca.key"), ("apiserver", "apiserver.crt", "apiserver.key"),
             ("apiserver-kubelet-client", "apiserver-kubelet-client.crt", "apiserver-kubelet-client.key"),
             ("front-proxy-ca", "front-proxy-ca.crt", "front-proxy-ca.key"),
             ("front-proxy-client", "front-proxy-client.crt", "front-proxy-client.key"))
SA_SECRET, SA_KEY = "sa", "sa.key"
CERT_SECRETS = {"kube-apiserver": ("ca", "apiserver", "apiserver-kubelet-client", "front-proxy-ca", "front-proxy-client", SA_SECRET),
                "kube-controller-manager": ("ca", SA_SECRET)}
KUBECONFIG_SECRETS = {"kube-controller-manager": "controller-manager.conf", "kube-scheduler": "scheduler.conf"}


def labels(component: str) -> dict:
    return {"k8s-app": PREFIX + component}


def secrets_of(mc: dict, p: dict) -> tuple[str, str] | None:
    """(certificates dir, kubeconfig dir) when the StoreCertsInSecrets gate is on."""
    return (p["pki"], p["kubeconfig_dir"]) if (mc.get("featureGates") or {}).get("StoreCertsInSecrets") else None


def _pairs(pki_dir: str):
    return [t for t in TLS_PAIRS if all(os.path.exists(os.path.join(pki_dir, f)) for f in t[1:])]


def _put(items: list, item: dict, key: str = "name") -> None:
    items[:] = [x for x in items if x.get(key) != item[key]] + [item]


def set_secret_volumes(component: str, spec: dict, pki_dir: str, kubeconfig_dir: str) -> dict:
    """setSelfHostedVolumesFor{APIServer,ControllerManager,Scheduler}: the certificates and the
    kubeconfig from the Secrets upload_secrets wrote."""
    vols, ct = spec.setdefault("volumes", []), (spec.get("containers") or [{}])[0]
    mounts = ct.setdefault("volumeMounts", [])
    if component in CERT_SECRETS:
        want = CERT_SECRETS[component]
        sources = [{"secret": {"name": n, "items": [{"key": "tls.crt", "path": crt}, {"key": "tls.key", "path": key}]}}
                   for n, crt, key in _pairs(pki_dir) if n in want]
        if SA_SECRET in want:
            sources.append({"secret": {"name": SA_SECRET, "items": [{"key": SA_KEY, "path": SA_KEY}]}})
        _put(vols, {"name": CERTS_VOLUME, "projected": {"sources": sources}})
        _put(mounts, {"name": CERTS_VOLUME, "mountPath": pki_dir, "readOnly": True})
    if component in KUBECONFIG_SECRETS:
        f, d = KUBECONFIG_SECRETS[component], os.path.join(kubeconfig_dir, "kubeconfig")
        _put(vols, {"name": KUBECONFIG_VOLUME, "secret": {"secretName": f}})
        _put(mounts, {"name": KUBECONFIG_VOLUME, "mountPath": d, "readOnly": True})
        args = list(ct.get("args") or [])
        if "--kubeconfig" in args:
            args[args.index("--kubeconfig") + 1] = os.path.join(d, f)
            ct["args"] = args
    return spec


def _secret(name: str, typ: str, files: dict) -> dict:
    data = {}
    for key, path in files.items():
        with open(path, "rb") as fh:
            data[key] = base64.b64encode(fh.read()).decode()
    return {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name, "namespace": "kube-system"},
            "type": typ, "data": data}


async def upload_secrets(c, pki_dir: str, kubeconfig_dir: str) -> list[str]:
    """uploadTLSSecrets + uploadKubeConfigSecrets; returns the Secrets written."""
    out = []
    secrets = [_secret(n, "kubernetes.io/tls", {"tls.crt": os.path.join(pki_dir, crt), "tls.key": os.path.join(pki_dir, key)})
               for n, crt, key in _pairs(pki_dir)]
    secrets.append(_secret(SA_SECRET, "Opaque", {SA_KEY: os.path.join(pki_dir, SA_KEY)}))
    secrets += [_secret(f, "Opaque", {f: os.path.join(kubeconfig_dir, f)}) for f in KUBECONFIG_SECRETS.values()]
    for sec in secrets:
        await create_or_update(c, "secrets", sec)
        out.append(sec["metadata"]["name"])
    return out


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


def build_daemonset(component: str, pod_spec: dict, secrets: tuple[str, str] | None = None) -> dict:
    """`secrets` = (certificates dir, kubeconfig dir) when StoreCertsInSecrets is on."""
    spec = mutate_pod_spec(component, dict(pod_spec))
    if secrets:
        spec = set_secret_volumes(component, spec, *secrets)
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


async def create_or_update(c, resource: str, obj: dict):
    """apiclient.CreateOrUpdate{DaemonSet,Secret}, retried while the API blinks."""
    async def once():
        cur = await c.get_or_none(resource, obj["metadata"]["name"], "kube-system")
        if cur is None:
            return await c.create(obj, "kube-system")
        obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return await c.update(obj)
    return await _retry(once)


async def create_or_update_daemonset(c, ds: dict):
    return await create_or_update(c, "daemonsets.apps", ds)


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
                                           dry_run: bool = False, out=print,
                                           secrets: tuple[str, str] | None = None) -> list[str]:
    """Convert every static control-plane Pod still on disk; returns the components converted.
    `secrets` = (certificates dir, kubeconfig dir) for StoreCertsInSecrets."""
    done = []
    if secrets and not dry_run:
        names = await upload_secrets(c, *secrets)
        out(f"[self-hosted] Uploaded the certificates and kubeconfigs as Secrets in kube-system: {', '.join(names)}")
    for comp in COMPONENTS:
        t0 = time.monotonic()
        path = os.path.join(manifests_dir, f"{comp}.yaml")
        if not os.path.exists(path):
            out(f"[self-hosted] The Static Pod for the component {comp!r} doesn't seem to be on the disk; trying the next one")
            continue
        with open(path) as f:
            pod = yaml.safe_load(f) or {}
        ds = build_daemonset(comp, pod.get("spec") or {}, secrets)
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
