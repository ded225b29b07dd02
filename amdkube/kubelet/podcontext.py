"""Per-pod content and environment resolution (kubelet_pods.go makeEnvironmentVariables and
the content half of the kubelet-rendered volume plugins).

Volume content (used by amdkube/volume/local.py; the volume manager owns the lifecycle):
configMap and secret (items key→path with mode, defaultMode, optional), downwardAPI (fieldRef
and resourceFieldRef with divisor), projected (secret / configMap / downwardAPI sources into
one directory), gitRepo (clone + checkout of a revision into `directory`); files are written
atomically (atomic_writer.go).

Environment (kubelet_pods.go:504-640): service variables of every service of the pod's
namespace plus the master `kubernetes` service (envvars.FromServices: <NAME>_SERVICE_HOST,
_SERVICE_PORT, _SERVICE_PORT_<PORT NAME>, docker-link <NAME>_PORT*), envFrom (configMapRef /
secretRef with prefix; keys that are not valid variable names are skipped), then env entries
with value (with $(VAR) expansion, third_party/forked/golang/expansion) or valueFrom (fieldRef,
resourceFieldRef, configMapKeyRef, secretKeyRef with `optional`). status.podIP is resolved
when the container starts, once the sandbox has its address.
"""
from __future__ import annotations

import base64
import math
import os
import re
import subprocess

from ..api import meta as m
from ..api.quantity import Quantity

POD_IP = "\x00podIP\x00"                    # replaced with the sandbox IP at container start
_ENV_NAME = re.compile(r"^[-._a-zA-Z][-._a-zA-Z0-9]*$")
_EXPAND = re.compile(r"\$\(([^)]*)\)|\$\$")


def atomic_write(path: str, data: bytes, mode: int | None = None):
    """atomic_writer.go: readers never see a half-written file; unchanged files stay."""
    try:
        with open(path, "rb") as f:
            same = f.read() == data
    except OSError:
        same = False
    if not same:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    if mode is not None:
        try:
            os.chmod(path, mode)
        except OSError:
            pass


def volume_file(d: str, rel: str) -> str:
    """The host path of a file a secret/configMap/projected/downwardAPI volume writes: `rel` must
    be relative with no '..' element (validateLocalDescendingPath), and the resolved target —
    after any symlink already inside the volume — must stay under the volume directory. The API
    server validates the same rule; this is the kubelet's own check on what it writes as root."""
    if not rel or rel.startswith("/") or ".." in rel.split("/"):
        raise ValueError(f"volume item path {rel!r} must be relative and must not contain '..'")
    base = os.path.realpath(d)
    target = os.path.realpath(os.path.join(base, rel))
    if os.path.commonpath([base, target]) != base or target == base:
        raise ValueError(f"volume item path {rel!r} escapes the volume directory")
    return target


def expand(s: str, env: dict[str, str]) -> str:
    """$(VAR) → env[VAR] when defined, else left as written; $$ → $."""
    def rep(mt):
        if mt.group(0) == "$$":
            return "$"
        name = mt.group(1)
        return env[name] if name in env else mt.group(0)
    return _EXPAND.sub(rep, s)


def service_env(services: list[dict]) -> dict[str, str]:
    """envvars.FromServices for services with a cluster IP."""
    out = {}
    for svc in services:
        spec = svc.get("spec") or {}
        ip = spec.get("clusterIP")
        if not ip or ip == "None":
            continue
        name = m.name_of(svc).upper().replace("-", "_")
        ports = spec.get("ports") or []
        if not ports:
            continue
        out[f"{name}_SERVICE_HOST"] = ip
        out[f"{name}_SERVICE_PORT"] = str(ports[0]["port"])
        for p in ports:
            if p.get("name"):
                out[f"{name}_SERVICE_PORT_{p['name'].upper().replace('-', '_')}"] = str(p["port"])
        proto = (ports[0].get("protocol") or "TCP").lower()
        out[f"{name}_PORT"] = f"{proto}://{ip}:{ports[0]['port']}"
        for p in ports:
            pr = (p.get("protocol") or "TCP")
            pre = f"{name}_PORT_{p['port']}_{pr.upper()}"
            out[pre] = f"{pr.lower()}://{ip}:{p['port']}"
            out[f"{pre}_PROTO"] = pr.lower()
            out[f"{pre}_PORT"] = str(p["port"])
            out[f"{pre}_ADDR"] = ip
    return out


def resource_value(pod: dict, container_name: str, ref: dict, node_alloc: dict) -> str:
    """resourceFieldRef: limits.cpu|memory|ephemeral-storage, requests.*; an unset limit is
    the node's allocatable (downward API defaulting); divisor rounds up (ExtractResourceValue)."""
    res = ref.get("resource", "")
    spec = pod.get("spec") or {}
    c = next((x for x in (spec.get("containers") or []) + (spec.get("initContainers") or [])
              if x["name"] == (ref.get("containerName") or container_name)), {})
    kind, _, rname = res.partition(".")
    rr = (c.get("resources") or {}).get(kind) or {}
    if rname in rr:
        q = Quantity(rr[rname])
    elif kind == "limits" and rname in node_alloc:
        q = Quantity(str(node_alloc[rname]))
    elif kind == "requests":
        q = Quantity(rr.get(rname) or "0")
    else:
        raise ValueError(f"unsupported container resource: {res}")
    div = Quantity(ref.get("divisor") or "1")
    if rname == "cpu":
        return str(math.ceil(q.milli_value() / max(1, div.milli_value())))
    return str(math.ceil(q.value() / max(1, div.value())))


class PodContext:
    def __init__(self, kubelet):
        self.k = kubelet

    # ------------------------------------------------------------------- fields
    def field(self, pod: dict, path: str) -> str:
        md = pod.get("metadata") or {}
        vals = {"metadata.name": md.get("name", ""), "metadata.namespace": md.get("namespace", ""),
                "metadata.uid": md.get("uid", ""), "spec.nodeName": self.k.node_name,
                "spec.serviceAccountName": (pod.get("spec") or {}).get("serviceAccountName", ""),
                "status.podIP": POD_IP, "status.hostIP": self.k.cfg.node_ip}
        if path.startswith("metadata.labels['"):
            return (md.get("labels") or {}).get(path[len("metadata.labels['"):-2], "")
        if path.startswith("metadata.annotations['"):
            return (md.get("annotations") or {}).get(path[len("metadata.annotations['"):-2], "")
        if path == "metadata.labels":
            return "\n".join(f'{k}="{v}"' for k, v in sorted((md.get("labels") or {}).items()))
        if path == "metadata.annotations":
            return "\n".join(f'{k}="{v}"' for k, v in sorted((md.get("annotations") or {}).items()))
        return vals.get(path, "")

    def _alloc(self) -> dict:
        from ..api.helpers import node_allocatable
        a = node_allocatable(self.k.node or {})
        return {k: (f"{v}m" if k == "cpu" else v) for k, v in a.items()}

    async def _obj(self, kind, name, ns, optional, what):
        obj = await self.k.client.get_or_none(kind, name, ns)
        if obj is None and not optional:
            raise RuntimeError(f"{what}: {kind[:-1]} {name!r} not found")
        return obj or {}

    # ------------------------------------------------------------------ volumes
    async def _projection(self, pod, d, kind, ref, default_mode, what):
        ns = m.namespace_of(pod)
        name = ref.get("name") or ref.get("secretName")
        obj = await self._obj(kind, name, ns, ref.get("optional"), what)
        data = obj.get("data") or {}
        items = ref.get("items")
        if items is None:
            items = [{"key": k, "path": k} for k in data]
        for it in items:
            if it["key"] not in data:
                if ref.get("optional"):
                    continue
                raise RuntimeError(f"{what}: key {it['key']!r} not found in {kind[:-1]} {name!r}")
            val = data[it["key"]]
            atomic_write(volume_file(d, it.get("path") or ""), base64.b64decode(val) if kind == "secrets" else val.encode(),
                         it.get("mode", ref.get("defaultMode", default_mode)))

    async def _downward(self, pod, d, items, default_mode):
        alloc = self._alloc()
        for it in items or []:
            if it.get("fieldRef"):
                val = self.field(pod, it["fieldRef"].get("fieldPath", ""))
                if val == POD_IP:
                    val = ""
            elif it.get("resourceFieldRef"):
                val = resource_value(pod, it["resourceFieldRef"].get("containerName", ""), it["resourceFieldRef"], alloc)
            else:
                val = ""
            atomic_write(volume_file(d, it.get("path") or ""), val.encode(), it.get("mode", default_mode))

    async def _git_repo(self, d: str, spec: dict, what: str) -> str:
        """git_repo.go SetUpAt: clone once into `directory` (or a subdirectory named after the
        repository), then check out `revision` and hard-reset."""
        if os.path.isdir(d) and os.path.exists(os.path.join(d, ".ready")):
            return d
        os.makedirs(d, exist_ok=True)
        repo, rev, sub = spec.get("repository", ""), spec.get("revision", ""), spec.get("directory", "")
        target = os.path.join(d, sub) if sub and sub != "." else (d if sub == "." else os.path.join(d, os.path.basename(repo.rstrip("/")).removesuffix(".git")))

        def run():
            r = subprocess.run(["git", "clone", "--", repo, target], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError(f"{what}: git clone failed: {r.stderr.strip()[-300:]}")
            if rev:
                for cmd in (["git", "checkout", rev], ["git", "reset", "--hard"]):
                    r = subprocess.run(cmd, cwd=target, capture_output=True, text=True, timeout=120)
                    if r.returncode != 0:
                        raise RuntimeError(f"{what}: {' '.join(cmd)} failed: {r.stderr.strip()[-300:]}")
            open(os.path.join(d, ".ready"), "w").close()
        import asyncio
        await asyncio.to_thread(run)
        return d

    # --------------------------------------------------------------------- env
    async def env(self, pod: dict, c: dict, services: list[dict]) -> dict[str, str]:
        ns = m.namespace_of(pod)
        e: dict[str, str] = dict(service_env(services))
        for ef in c.get("envFrom") or []:
            ref = ef.get("configMapRef") or ef.get("secretRef")
            if not ref:
                continue
            kind = "configmaps" if "configMapRef" in ef else "secrets"
            obj = await self._obj(kind, ref["name"], ns, ref.get("optional"), f"envFrom of {c['name']}")
            for k, val in (obj.get("data") or {}).items():
                key = (ef.get("prefix") or "") + k
                if _ENV_NAME.match(key):
                    e[key] = base64.b64decode(val).decode() if kind == "secrets" else val
        alloc = None
        for ev in c.get("env") or []:
            if "valueFrom" not in ev:
                e[ev["name"]] = expand(str(ev.get("value", "")), e)
                continue
            vf = ev["valueFrom"]
            if "fieldRef" in vf:
                e[ev["name"]] = self.field(pod, vf["fieldRef"].get("fieldPath", ""))
            elif "resourceFieldRef" in vf:
                alloc = alloc if alloc is not None else self._alloc()
                e[ev["name"]] = resource_value(pod, c["name"], vf["resourceFieldRef"], alloc)
            else:
                for kind, key in (("configmaps", "configMapKeyRef"), ("secrets", "secretKeyRef")):
                    if key in vf:
                        ref = vf[key]
                        obj = await self._obj(kind, ref["name"], ns, ref.get("optional"), f"env {ev['name']}")
                        data = obj.get("data") or {}
                        if ref["key"] not in data:
                            if ref.get("optional"):
                                break
                            raise RuntimeError(f"env {ev['name']}: key {ref['key']!r} not found in {kind[:-1]} {ref['name']!r}")
                        val = data[ref["key"]]
                        e[ev["name"]] = base64.b64decode(val).decode() if kind == "secrets" else val
        e.setdefault("HOSTNAME", (pod.get("spec") or {}).get("hostname") or m.name_of(pod))
        e.setdefault("KUBERNETES_POD_NAME", m.name_of(pod))
        e.setdefault("KUBERNETES_NAMESPACE", ns)
        return e


def hosts_file(pod: dict, ip: str, cluster_domain: str = "") -> str:
    """kubelet_pods.go managedHostsFileContent + hostAliases."""
    spec = pod.get("spec") or {}
    hostname = spec.get("hostname") or m.name_of(pod)
    lines = ["# Kubernetes-managed hosts file.", "127.0.0.1\tlocalhost", "::1\tlocalhost ip6-localhost ip6-loopback",
             "fe00::0\tip6-localnet", "fe00::0\tip6-mcastprefix", "fe00::1\tip6-allnodes", "fe00::2\tip6-allrouters"]
    sub = spec.get("subdomain")
    if sub and cluster_domain:
        lines.append(f"{ip}\t{hostname}.{sub}.{m.namespace_of(pod)}.svc.{cluster_domain}\t{hostname}")
    else:
        lines.append(f"{ip}\t{hostname}")
    if spec.get("hostAliases"):
        lines.append("")
        lines.append("# Entries added by HostAliases.")
        for ha in spec["hostAliases"]:
            lines.append(f"{ha.get('ip', '')}\t" + "\t".join(ha.get("hostnames") or []))
    return "\n".join(lines) + "\n"
