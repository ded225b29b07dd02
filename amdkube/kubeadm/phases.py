"""kubeadm phases and cluster configuration (cmd/kubeadm/app/cmd/phases/*.go, app/apis/kubeadm/
v1alpha1 MasterConfiguration, app/phases/uploadconfig, app/phases/addons, app/cmd/config.go).

`kubeadm init` is the phases below run in order; `kubeadm alpha phase <name> [<sub>]` runs one
of them on its own, against the same --base-dir and --config:

  preflight        checks before touching the host
  certs            ca, apiserver, apiserver-kubelet-client, sa, front-proxy-ca, front-proxy-client
  kubeconfig       admin, kubelet, controller-manager, scheduler, kube-proxy, user (--client-name)
  controlplane     static Pod manifests: apiserver, controller-manager, scheduler
  etcd local       where the apiserver keeps its objects (etcd_mode): by default the
                   apiserver's embedded MVCC store (--data-dir), this phase preparing that
                   directory; with `etcd.dataDir` set, an `amdkube etcd` static Pod on that
                   directory that the apiserver reaches through --etcd-servers (the
                   reference's local etcd, app/phases/etcd/local.go); with `etcd.endpoints`,
                   an external etcd (caFile/certFile/keyFile) and no local store at all
  mark-master      master label + NoSchedule taint
  bootstrap-token  create, cluster-info, node allow-post-csrs, node allow-auto-approve
  upload-config    the MasterConfiguration in kube-system/kubeadm-config (read back by
                   `kubeadm config view` and `kubeadm upgrade`)
  addon            kube-proxy, kube-dns, amd-gpu-device-plugin
  selfhosting      convert-from-staticpods: the control plane as DaemonSets (selfhosting.py);
                   `init --feature-gates SelfHosting=true` runs it last

The MasterConfiguration (kubeadm.k8s.io/v1alpha1) is built from flags or read from --config;
its api/networking/nodeName/kubernetesVersion/certificatesDir/apiServerCertSANs/
*ExtraArgs/featureGates/token/tokenTTL fields drive every phase.
"""
from __future__ import annotations

import asyncio
import ipaddress
import os
import re
import secrets
import socket
import sys
import time

import yaml

from .. import GIT_VERSION
from . import (ADMISSION, GPU_LABEL, MASTER_LABEL, ROOT, _bootstrap_rbac, _client, _component_pod,
               kubeconfig, new_ca, new_cert, new_token, token_secret, write_yaml)

CONFIG_MAP = "kubeadm-config"
CONFIG_KEY = "MasterConfiguration"
VERSION_ANNOTATION = "amdkube.io/kubernetes-version"


def _duration(s) -> float:
    """Go duration ("24h0m0s", "90m", "0s") or seconds → seconds."""
    if isinstance(s, (int, float)):
        return float(s)
    tot = 0.0
    for n, u in re.findall(r"([\d.]+)(h|m|s)", s or ""):
        tot += float(n) * {"h": 3600, "m": 60, "s": 1}[u]
    return tot


def _fmt_duration(sec: float) -> str:
    sec = int(sec)
    return f"{sec // 3600}h{sec % 3600 // 60}m{sec % 60}s"


def master_config(a) -> dict:
    """Defaults ← flags ← --config file (the file wins, as in the reference where --config
    excludes most flags)."""
    mc = {"apiVersion": "kubeadm.k8s.io/v1alpha1", "kind": "MasterConfiguration",
          "api": {"advertiseAddress": getattr(a, "apiserver_advertise_address", None) or "127.0.0.1",
                  "bindPort": getattr(a, "apiserver_bind_port", None) or 6443},
          "networking": {"serviceSubnet": getattr(a, "service_cidr", None) or "10.96.0.0/12",
                         "podSubnet": getattr(a, "pod_network_cidr", None) or "",
                         "dnsDomain": getattr(a, "service_dns_domain", None) or "cluster.local"},
          "kubernetesVersion": getattr(a, "kubernetes_version", None) or GIT_VERSION,
          "nodeName": getattr(a, "node_name", None) or socket.gethostname(),
          "certificatesDir": os.path.join(a.base_dir, "pki"),
          "apiServerCertSANs": [x for x in (getattr(a, "apiserver_cert_extra_sans", "") or "").split(",") if x],
          "apiServerExtraArgs": {}, "controllerManagerExtraArgs": {}, "schedulerExtraArgs": {},
          "featureGates": {}, "token": getattr(a, "token", None) or "",
          "tokenTTL": _fmt_duration(getattr(a, "token_ttl", None) or 24 * 3600)}
    for kv in (getattr(a, "feature_gates", "") or "").split(","):
        if "=" in kv:
            k, v = kv.split("=", 1)
            mc["featureGates"][k.strip()] = v.strip().lower() == "true"
    path = getattr(a, "config", None)
    mc = merge_config(mc, load_config_file(path)) if path else mc
    resolve_gate_dependencies(mc.setdefault("featureGates", {}))
    return mc


def resolve_gate_dependencies(gates: dict) -> dict:
    """features.ResolveFeatureGateDependencies: StoreCertsInSecrets needs SelfHosting;
    HighAvailability needs both."""
    if gates.get("StoreCertsInSecrets"):
        gates["SelfHosting"] = True
    if gates.get("HighAvailability"):
        gates["SelfHosting"] = gates["StoreCertsInSecrets"] = True
    return gates


def load_config_file(path: str) -> dict:
    with open(path) as f:
        user = yaml.safe_load(f) or {}
    if user.get("kind") not in (None, "MasterConfiguration"):
        raise SystemExit(f"error: {path}: expected kind MasterConfiguration, got {user.get('kind')}")
    return user


def merge_config(base: dict, user: dict) -> dict:
    out = dict(base)
    for k, v in user.items():
        out[k] = {**out[k], **v} if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def paths(base: str, mc: dict | None = None) -> dict:
    return {"base": base, "pki": (mc or {}).get("certificatesDir") or os.path.join(base, "pki"), "kubeconfig_dir": base,
            "manifests": os.path.join(base, "manifests"), "data_dir": os.path.join(base, "data"),
            "node_dir": os.path.join(base, "node")}


def server_url(mc: dict) -> str:
    return f"https://{mc['api']['advertiseAddress']}:{mc['api']['bindPort']}"


# ------------------------------------------------------------------------------ preflight
def phase_preflight(mc: dict, p: dict, ignore=()) -> tuple[list, list]:
    import shutil
    errs, warns = [], []
    if shutil.which("openssl") is None:
        errs.append("FileExisting-openssl: openssl is required for the PKI phase")
    with socket.socket() as s:
        try:
            s.bind((mc["api"]["advertiseAddress"], mc["api"]["bindPort"]))
        except OSError:
            errs.append(f"Port-{mc['api']['bindPort']}: port {mc['api']['bindPort']} is in use")
    if os.path.isdir(p["manifests"]) and os.listdir(p["manifests"]):
        errs.append(f"DirAvailable--{p['manifests']}: {p['manifests']} is not empty")
    try:
        ipaddress.ip_network(mc["networking"]["serviceSubnet"], strict=False)
    except ValueError as e:
        errs.append(f"ServiceSubnet: {e}")
    if not os.path.exists("/dev/kfd"):
        warns.append("no /dev/kfd: this node has no MI355X (ROCm KFD) device; GPU pods will not schedule here")
    errs = [e for e in errs if not any(x and (e.startswith(x) or x == "all") for x in ignore)]
    return errs, warns


# ---------------------------------------------------------------------------------- certs
CERTS = ("ca", "apiserver", "apiserver-kubelet-client", "sa", "front-proxy-ca", "front-proxy-client")


def apiserver_sans(mc: dict) -> list[str]:
    first_svc = str(next(ipaddress.ip_network(mc["networking"]["serviceSubnet"], strict=False).hosts()))
    adv, node, dom = mc["api"]["advertiseAddress"], mc["nodeName"], mc["networking"]["dnsDomain"]
    sans = [f"IP:{adv}", "IP:127.0.0.1", f"IP:{first_svc}", f"DNS:{node}", "DNS:kubernetes", "DNS:kubernetes.default",
            "DNS:kubernetes.default.svc", f"DNS:kubernetes.default.svc.{dom}", "DNS:localhost"]
    for extra in mc.get("apiServerCertSANs") or []:
        try:
            ipaddress.ip_address(extra)
            sans.append(f"IP:{extra}")
        except ValueError:
            sans.append(f"DNS:{extra}")
    return list(dict.fromkeys(sans))


def phase_certs(mc: dict, p: dict, which: str = "all") -> list[str]:
    """Existing CAs and keys are reused (kubeadm's "Using the existing ..."), leaf certificates
    are re-issued only when missing."""
    d = p["pki"]
    os.makedirs(d, exist_ok=True)
    done = []
    want = CERTS if which == "all" else (which,)
    for name in want:
        if name not in CERTS:
            raise SystemExit(f"error: unknown certificate {name!r} (one of {', '.join(CERTS)})")
        if name == "ca" and not os.path.exists(f"{d}/ca.crt"):
            new_ca(d)
        elif name == "front-proxy-ca" and not os.path.exists(f"{d}/front-proxy-ca.crt"):
            new_ca(d, "front-proxy-ca", "front-proxy-ca")
        elif name == "apiserver" and not os.path.exists(f"{d}/apiserver.crt"):
            new_cert(d, "apiserver", "kube-apiserver", sans=apiserver_sans(mc), server=True)
        elif name == "apiserver-kubelet-client" and not os.path.exists(f"{d}/apiserver-kubelet-client.crt"):
            new_cert(d, "apiserver-kubelet-client", "kube-apiserver-kubelet-client", orgs=("system:masters",))
        elif name == "front-proxy-client" and not os.path.exists(f"{d}/front-proxy-client.crt"):
            new_cert(d, "front-proxy-client", "front-proxy-client", ca="front-proxy-ca")
        elif name == "sa" and not os.path.exists(f"{d}/sa.key"):
            with open(f"{d}/sa.key", "wb") as f:
                f.write(secrets.token_hex(32).encode())
            os.chmod(f"{d}/sa.key", 0o600)
        else:
            continue
        done.append(name)
    return done


# ----------------------------------------------------------------------------- kubeconfig
KUBECONFIGS = {"admin": ("kubernetes-admin", ("system:masters",)), "kubelet": (None, ("system:nodes",)),
               "controller-manager": ("system:kube-controller-manager", ()), "scheduler": ("system:kube-scheduler", ()),
               "kube-proxy": ("system:kube-proxy", ())}


def phase_kubeconfig(mc: dict, p: dict, which: str = "all", client_name: str | None = None, orgs=()) -> list[str]:
    d = p["pki"]
    ca = open(f"{d}/ca.crt", "rb").read()
    server = server_url(mc)
    out = []
    if which == "user":
        if not client_name:
            raise SystemExit("error: --client-name is required for the user kubeconfig")
        nm = f"user-{client_name}"
        new_cert(d, nm, client_name, orgs=tuple(orgs))
        return [yaml.safe_dump(kubeconfig(server, ca, client_name, open(f"{d}/{nm}.crt", "rb").read(),
                                          open(f"{d}/{nm}.key", "rb").read()), sort_keys=False)]
    for name in (KUBECONFIGS if which == "all" else (which,)):
        if name not in KUBECONFIGS:
            raise SystemExit(f"error: unknown kubeconfig {name!r} (one of {', '.join(KUBECONFIGS)}, user)")
        cn, org = KUBECONFIGS[name]
        cn = cn or f"system:node:{mc['nodeName']}"
        target = os.path.join(p["kubeconfig_dir"], f"{name}.conf")
        if os.path.exists(target):
            continue
        new_cert(d, name, cn, orgs=org)
        write_yaml(target, kubeconfig(server, ca, cn, open(f"{d}/{name}.crt", "rb").read(), open(f"{d}/{name}.key", "rb").read()))
        out.append(f"{name}.conf")
    return out


# --------------------------------------------------------------------------- controlplane
def _with_extra(args: list[str], extra: dict) -> list[str]:
    """ExtraArgs override the generated flag of the same name or are appended."""
    out, i, seen = [], 0, set()
    while i < len(args):
        flag = args[i]
        key = flag[2:]
        if key in extra:
            out += [flag, str(extra[key])]
            seen.add(key)
        else:
            out += [flag, args[i + 1]]
        i += 2
    for k, v in extra.items():
        if k not in seen:
            out += [f"--{k}", str(v)]
    return out


def etcd_mode(mc: dict) -> str:
    """"external" (etcd.endpoints), "local" (etcd.dataDir: an `amdkube etcd` static Pod) or
    "embedded" (neither: the apiserver's own store, amdkube's default and fastest path)."""
    e = mc.get("etcd") or {}
    return "external" if e.get("endpoints") else "local" if e.get("dataDir") else "embedded"


def local_etcd_url(mc: dict) -> str:
    extra = (mc.get("etcd") or {}).get("extraArgs") or {}
    return str(extra.get("listen-client-urls") or "http://127.0.0.1:2379").split(",")[0]


def etcd_manifest(mc: dict) -> dict:
    """The local etcd static Pod (GetEtcdPodSpec): `amdkube etcd` on etcd.dataDir."""
    e = mc.get("etcd") or {}
    args = _with_extra(["--listen-client-urls", local_etcd_url(mc), "--advertise-client-urls", local_etcd_url(mc),
                        "--data-dir", e["dataDir"]], e.get("extraArgs") or {})
    pod = _component_pod("etcd", ["etcd", *args])
    pod["metadata"]["annotations"][VERSION_ANNOTATION] = mc["kubernetesVersion"]
    return pod


def _store_args(mc: dict, p: dict) -> list[str]:
    mode, e = etcd_mode(mc), mc.get("etcd") or {}
    if mode == "embedded":
        return ["--data-dir", p["data_dir"]]
    if mode == "local":
        return ["--etcd-servers", local_etcd_url(mc)]
    out = ["--etcd-servers", ",".join(e["endpoints"])]
    for key, flag in (("caFile", "--etcd-cafile"), ("certFile", "--etcd-certfile"), ("keyFile", "--etcd-keyfile")):
        if e.get(key):
            out += [flag, e[key]]
    return out


def control_plane_manifests(mc: dict, p: dict) -> dict[str, dict]:
    d, k = p["pki"], p["kubeconfig_dir"]
    api = ["--bind-address", mc["api"]["advertiseAddress"], "--port", str(mc["api"]["bindPort"]),
           "--tls-cert-file", f"{d}/apiserver.crt", "--tls-private-key-file", f"{d}/apiserver.key",
           "--client-ca-file", f"{d}/ca.crt", "--authorization-mode", "Node,RBAC", "--anonymous-auth", "true",
           "--admission-control", ADMISSION, "--service-account-key-file", f"{d}/sa.key",
           "--service-cluster-ip-range", mc["networking"]["serviceSubnet"], *_store_args(mc, p),
           "--kubelet-client-certificate", f"{d}/apiserver-kubelet-client.crt",
           "--kubelet-client-key", f"{d}/apiserver-kubelet-client.key"]
    if (mc.get("featureGates") or {}).get("HighAvailability"):      # several apiservers share the endpoints
        api += ["--endpoint-reconciler-type", "lease"]
    if os.path.exists(f"{d}/front-proxy-ca.crt"):
        api += ["--requestheader-client-ca-file", f"{d}/front-proxy-ca.crt", "--requestheader-allowed-names", "front-proxy-client",
                "--proxy-client-cert-file", f"{d}/front-proxy-client.crt", "--proxy-client-key-file", f"{d}/front-proxy-client.key"]
    cm = ["--kubeconfig", f"{k}/controller-manager.conf", "--leader-elect", "true",
          "--service-account-private-key-file", f"{d}/sa.key", "--root-ca-file", f"{d}/ca.crt",
          "--cluster-signing-cert-file", f"{d}/ca.crt", "--cluster-signing-key-file", f"{d}/ca.key",
          "--controllers", "*,bootstrapsigner,tokencleaner", "--hostpath-pv-root", os.path.join(p["data_dir"], "pv")]
    if mc["networking"].get("podSubnet"):
        cm += ["--allocate-node-cidrs", "true", "--cluster-cidr", mc["networking"]["podSubnet"]]
    sched = ["--kubeconfig", f"{k}/scheduler.conf", "--leader-elect", "true", "--port", "0"]
    from ..utils.features import KNOWN
    # kubeadm's own gates (SelfHosting, StoreCertsInSecrets, HighAvailability, CoreDNS) stay
    # with kubeadm (cmd/kubeadm/app/features); only component gates reach the scheduler
    gates = ",".join(f"{g}={str(v).lower()}" for g, v in sorted((mc.get("featureGates") or {}).items()) if g in KNOWN)
    out = {}
    for name, comp, args, extra in (("kube-apiserver", "apiserver", api, mc.get("apiServerExtraArgs") or {}),
                                    ("kube-controller-manager", "controller-manager", cm, mc.get("controllerManagerExtraArgs") or {}),
                                    ("kube-scheduler", "scheduler", sched, mc.get("schedulerExtraArgs") or {})):
        argv = _with_extra(args, extra)
        if gates and comp == "scheduler" and "feature-gates" not in extra:   # the kubelet takes its own
            argv += ["--feature-gates", gates]
        pod = _component_pod(name, [comp, *argv])
        pod["metadata"]["annotations"][VERSION_ANNOTATION] = mc["kubernetesVersion"]
        out[name] = pod
    return out


def phase_controlplane(mc: dict, p: dict, which: str = "all") -> list[str]:
    os.makedirs(p["manifests"], exist_ok=True)
    names = {"apiserver": "kube-apiserver", "controller-manager": "kube-controller-manager", "scheduler": "kube-scheduler"}
    if which != "all" and which not in names:
        raise SystemExit(f"error: unknown control plane component {which!r} (one of {', '.join(names)})")
    man = control_plane_manifests(mc, p)
    out = []
    for short, name in names.items():
        if which in ("all", short):
            write_yaml(os.path.join(p["manifests"], f"{name}.yaml"), man[name], 0o644)
            out.append(name)
    return out


def phase_etcd_local(mc: dict, p: dict) -> str:
    """What this node keeps the cluster's objects in; returns a line for the init log."""
    mode = etcd_mode(mc)
    if mode == "external":
        return f"Using the external etcd at {', '.join(mc['etcd']['endpoints'])}"
    if mode == "local":
        os.makedirs(p["manifests"], exist_ok=True)
        path = os.path.join(p["manifests"], "etcd.yaml")
        write_yaml(path, etcd_manifest(mc), 0o644)
        return f"Wrote Static Pod manifest for a local etcd instance to {path} (data directory {mc['etcd']['dataDir']})"
    os.makedirs(p["data_dir"], exist_ok=True)
    return f"The store is embedded in kube-apiserver (data directory {p['data_dir']})"


# -------------------------------------------------------------------- cluster-side phases
async def _create_or_replace(c, obj):
    from ..api import meta as m
    from ..api.scheme import SCHEME
    try:
        await c.create(obj, obj["metadata"].get("namespace"))
    except m.StatusError as e:
        if not m.is_already_exists(e):
            raise
        ri = SCHEME.for_object(obj)
        res = ri.plural if not ri.group else f"{ri.plural}.{ri.group}"
        cur = await c.get(res, obj["metadata"]["name"], obj["metadata"].get("namespace") or "")
        obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        if obj["kind"] == "ConfigMap":      # keep the bootstrap signer's jws-kubeconfig-<id> signatures
            obj["data"] = {**{k: v for k, v in (cur.get("data") or {}).items() if k.startswith("jws-kubeconfig-")},
                           **obj.get("data", {})}
        await c.update(obj)


async def phase_mark_master(c, node: str, timeout: float = 60.0) -> bool:
    end = time.time() + timeout
    while time.time() < end and await c.get_or_none("nodes", node) is None:
        await asyncio.sleep(0.2)
    n = await c.get_or_none("nodes", node)
    if n is None:
        return False
    taints = [t for t in (n.get("spec") or {}).get("taints") or [] if t.get("key") != MASTER_LABEL]
    await c.patch("nodes", node, {"metadata": {"labels": {MASTER_LABEL: ""}},
                                  "spec": {"taints": taints + [{"key": MASTER_LABEL, "effect": "NoSchedule"}]}})
    return True


def cluster_info(mc: dict, p: dict) -> dict:
    ca = open(os.path.join(p["pki"], "ca.crt"), "rb").read()
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cluster-info", "namespace": "kube-public"},
            "data": {"kubeconfig": yaml.safe_dump(kubeconfig(server_url(mc), ca, "", None, None))}}


async def phase_bootstrap_token(c, mc: dict, p: dict, which: str = "all", token: str | None = None) -> list[str]:
    rb = _bootstrap_rbac()
    done = []
    if which in ("all", "create"):
        t = token or mc.get("token") or new_token()
        mc["token"] = t
        await _create_or_replace(c, token_secret(t, _duration(mc.get("tokenTTL") or "24h") or None,
                                                 description="default kubeadm bootstrap token"))
        done.append("create")
    if which in ("all", "allow-post-csrs"):
        await _create_or_replace(c, rb[0])
        done.append("allow-post-csrs")
    if which in ("all", "allow-auto-approve"):
        await _create_or_replace(c, rb[1])
        done.append("allow-auto-approve")
    if which in ("all", "cluster-info"):
        await _create_or_replace(c, cluster_info(mc, p))
        for o in rb[2:]:
            await _create_or_replace(c, o)
        done.append("cluster-info")
    if not done:
        raise SystemExit(f"error: unknown bootstrap-token phase {which!r}")
    return done


async def phase_upload_config(c, mc: dict):
    stored = {k: v for k, v in mc.items() if k != "token"}     # the token is a secret of its own
    await _create_or_replace(c, {"apiVersion": "v1", "kind": "ConfigMap",
                                 "metadata": {"name": CONFIG_MAP, "namespace": "kube-system"},
                                 "data": {CONFIG_KEY: yaml.safe_dump(stored, sort_keys=False)}})


async def read_cluster_config(c) -> dict | None:
    cm = await c.get_or_none("configmaps", CONFIG_MAP, "kube-system")
    if cm is None:
        return None
    return yaml.safe_load((cm.get("data") or {}).get(CONFIG_KEY) or "{}")


ADDONS = ("kube-proxy", "kube-dns", "amd-gpu-device-plugin")


def dns_ip(mc: dict) -> str:
    net = ipaddress.ip_network(mc["networking"]["serviceSubnet"], strict=False)
    return str(net.network_address + 10)


def addon_objects(mc: dict, p: dict, which: str = "all") -> list[dict]:
    from ..api.scheme import load_manifests
    env = [{"name": "PYTHONPATH", "value": ROOT}]
    tol = [{"key": MASTER_LABEL, "effect": "NoSchedule"}]
    out = []
    if which in ("all", "kube-proxy"):
        out.append({"apiVersion": "apps/v1", "kind": "DaemonSet",
                    "metadata": {"name": "kube-proxy", "namespace": "kube-system", "labels": {"k8s-app": "kube-proxy"},
                                 "annotations": {VERSION_ANNOTATION: mc["kubernetesVersion"]}},
                    "spec": {"selector": {"matchLabels": {"k8s-app": "kube-proxy"}},
                             "template": {"metadata": {"labels": {"k8s-app": "kube-proxy"}},
                                          "spec": {"hostNetwork": True, "tolerations": tol,
                                                   "containers": [{"name": "kube-proxy", "image": "python:3",
                                                                   "args": ["-m", "amdkube", "proxy", "--kubeconfig",
                                                                            os.path.join(p["base"], "kube-proxy.conf"),
                                                                            "--healthz-port", "0", "--bind-address", "127.0.0.1"],
                                                                   "env": env}]}}}})
    if which in ("all", "kube-dns") and (mc.get("featureGates") or {}).get("CoreDNS"):
        out += coredns_objects(mc, p, env, tol)
    elif which in ("all", "kube-dns"):
        labels = {"k8s-app": "kube-dns"}
        out.append({"apiVersion": "apps/v1", "kind": "Deployment",
                    "metadata": {"name": "kube-dns", "namespace": "kube-system", "labels": labels,
                                 "annotations": {VERSION_ANNOTATION: mc["kubernetesVersion"]}},
                    "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                             "template": {"metadata": {"labels": labels},
                                          "spec": {"tolerations": tol + [{"key": "CriticalAddonsOnly", "operator": "Exists"}],
                                                   "priorityClassName": "system-cluster-critical",
                                                   "containers": [{"name": "kubedns", "image": "python:3",
                                                                   "args": ["-m", "amdkube", "dns", "--kubeconfig",
                                                                            os.path.join(p["base"], "kube-proxy.conf"),
                                                                            "--domain", mc["networking"]["dnsDomain"],
                                                                            "--dns-bind-address", "0.0.0.0", "--dns-port", "10053"],
                                                                   "ports": [{"name": "dns", "containerPort": 10053, "protocol": "UDP"},
                                                                             {"name": "dns-tcp", "containerPort": 10053, "protocol": "TCP"}],
                                                                   "env": env}]}}}})
        out.append({"apiVersion": "v1", "kind": "Service",
                    "metadata": {"name": "kube-dns", "namespace": "kube-system",
                                 "labels": dict(labels, **{"kubernetes.io/name": "KubeDNS"})},
                    "spec": {"selector": labels, "clusterIP": dns_ip(mc),
                             "ports": [{"name": "dns", "port": 53, "protocol": "UDP", "targetPort": 10053},
                                       {"name": "dns-tcp", "port": 53, "protocol": "TCP", "targetPort": 10053}]}})
    if which in ("all", "amd-gpu-device-plugin"):
        for d in load_manifests(open(os.path.join(ROOT, "deploy", "amd-gpu-device-plugin.yaml")).read()):
            if d and d.get("kind") == "DaemonSet":
                tpl = d["spec"]["template"]["spec"]
                tpl.setdefault("nodeSelector", {})[GPU_LABEL] = "true"
                for ct in tpl.get("containers") or []:
                    ct.setdefault("env", []).append({"name": "PYTHONPATH", "value": ROOT})
                d["metadata"].setdefault("namespace", "kube-system")
                out.append(d)
    if which not in ("all", *ADDONS):
        raise SystemExit(f"error: unknown addon {which!r} (one of {', '.join(ADDONS)})")
    return out


COREFILE = """.:53 {{
    errors
    log
    health
    kubernetes {domain} {cidr} {{
       pods insecure
    }}
    prometheus
    proxy . /etc/resolv.conf
    cache 30
}}
"""


def coredns_objects(mc: dict, p: dict, env: list, tol: list) -> list[dict]:
    """The CoreDNS feature gate (addons/dns/dns.go coreDNSAddon, manifests.go): ConfigMap
    coredns with the Corefile, ServiceAccount coredns, ClusterRole/Binding system:coredns, a
    Deployment coredns whose pods carry k8s-app=kube-dns and read the Corefile from the
    ConfigMap volume at /etc/coredns (`amdkube dns -conf`, dns/corefile.py), and the Service
    kube-dns. The pods listen on 10053 (unprivileged); the Service maps 53 to it."""
    labels, rb = {"k8s-app": "kube-dns"}, "rbac.authorization.k8s.io/v1"
    corefile = COREFILE.format(domain=mc["networking"]["dnsDomain"], cidr=mc["networking"]["serviceSubnet"])
    ann = {VERSION_ANNOTATION: mc["kubernetesVersion"]}
    return [
        {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "coredns", "namespace": "kube-system"},
         "data": {"Corefile": corefile}},
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "coredns", "namespace": "kube-system"}},
        {"apiVersion": rb, "kind": "ClusterRole",
         "metadata": {"name": "system:coredns", "labels": {"kubernetes.io/bootstrapping": "rbac-defaults"}},
         "rules": [{"apiGroups": [""], "resources": ["endpoints", "services", "pods", "namespaces"], "verbs": ["list", "watch"]}]},
        {"apiVersion": rb, "kind": "ClusterRoleBinding",
         "metadata": {"name": "system:coredns", "labels": {"kubernetes.io/bootstrapping": "rbac-defaults"},
                      "annotations": {"rbac.authorization.kubernetes.io/autoupdate": "true"}},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "system:coredns"},
         "subjects": [{"kind": "ServiceAccount", "name": "coredns", "namespace": "kube-system"}]},
        {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"name": "coredns", "namespace": "kube-system", "labels": labels, "annotations": ann},
         "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                  "template": {"metadata": {"labels": labels},
                               "spec": {"serviceAccountName": "coredns",
                                        "tolerations": tol + [{"key": "CriticalAddonsOnly", "operator": "Exists"}],
                                        "priorityClassName": "system-cluster-critical",
                                        "volumes": [{"name": "config-volume", "configMap": {
                                            "name": "coredns", "items": [{"key": "Corefile", "path": "Corefile"}]}}],
                                        "containers": [{"name": "coredns", "image": "python:3",
                                                        "args": ["-m", "amdkube", "dns", "-conf", "/etc/coredns/Corefile",
                                                                 "--kubeconfig", os.path.join(p["base"], "kube-proxy.conf"),
                                                                 "--dns-bind-address", "0.0.0.0", "--dns-port", "10053"],
                                                        "volumeMounts": [{"name": "config-volume", "mountPath": "/etc/coredns"}],
                                                        "ports": [{"name": "dns", "containerPort": 10053, "protocol": "UDP"},
                                                                  {"name": "dns-tcp", "containerPort": 10053, "protocol": "TCP"}],
                                                        "env": env}]}}}},
        {"apiVersion": "v1", "kind": "Service",
         "metadata": {"name": "kube-dns", "namespace": "kube-system",
                      "labels": dict(labels, **{"kubernetes.io/name": "CoreDNS"})},
         "spec": {"selector": labels, "clusterIP": dns_ip(mc),
                  "ports": [{"name": "dns", "port": 53, "protocol": "UDP", "targetPort": 10053},
                            {"name": "dns-tcp", "port": 53, "protocol": "TCP", "targetPort": 10053}]}},
    ]


async def phase_addons(c, mc: dict, p: dict, which: str = "all") -> list[str]:
    objs = addon_objects(mc, p, which)
    for o in objs:
        await _create_or_replace(c, o)
    return [f"{o['kind'].lower()}/{o['metadata']['name']}" for o in objs]


# ------------------------------------------------------------------------ `alpha phase` CLI
def add_phase_parser(sub):
    ph = sub.add_parser("phase", help="run one phase of kubeadm init")
    ph.add_argument("phase", choices=("preflight", "certs", "kubeconfig", "controlplane", "etcd", "mark-master",
                                      "bootstrap-token", "upload-config", "addon", "selfhosting"))
    ph.add_argument("--dry-run", action="store_true", help="selfhosting: print the DaemonSets instead")
    ph.add_argument("--timeout", type=float, default=120.0)
    ph.add_argument("sub", nargs="*", default=[])
    ph.add_argument("--base-dir", default="/etc/kubernetes")
    ph.add_argument("--config", default=None)
    ph.add_argument("--kubeconfig", default=None, help="admin kubeconfig for the cluster-side phases")
    ph.add_argument("--node-name", default=None)
    ph.add_argument("--apiserver-advertise-address", default=None)
    ph.add_argument("--apiserver-bind-port", type=int, default=None)
    ph.add_argument("--service-cidr", default=None)
    ph.add_argument("--pod-network-cidr", default=None)
    ph.add_argument("--service-dns-domain", default=None)
    ph.add_argument("--apiserver-cert-extra-sans", default="")
    ph.add_argument("--kubernetes-version", default=None)
    ph.add_argument("--feature-gates", default="")
    ph.add_argument("--token", default=None)
    ph.add_argument("--token-ttl", type=float, default=None)
    ph.add_argument("--client-name", default=None)
    ph.add_argument("--client-org", action="append", default=[])
    ph.add_argument("--ignore-preflight-errors", default="")
    return ph


def run_phase(a) -> int:
    mc = master_config(a)
    p = paths(a.base_dir, mc)
    sub = a.sub[0] if a.sub else "all"
    if a.phase == "preflight":
        errs, warns = phase_preflight(mc, p, tuple(x for x in a.ignore_preflight_errors.split(",") if x))
        for w in warns:
            print(f"[preflight] WARNING: {w}")
        if errs:
            print("[preflight] Some fatal errors occurred:\n" + "\n".join(f"\t[ERROR {e}]" for e in errs), file=sys.stderr)
            return 1
        print("[preflight] All checks passed")
        return 0
    if a.phase == "certs":
        done = phase_certs(mc, p, sub)
        print(f"[certificates] Generated {', '.join(done) or 'nothing (all present)'} in {p['pki']}")
        return 0
    if a.phase == "kubeconfig":
        if sub == "user":
            print(phase_kubeconfig(mc, p, "user", a.client_name, a.client_org)[0], end="")
        else:
            done = phase_kubeconfig(mc, p, sub)
            print(f"[kubeconfig] Wrote {', '.join(done) or 'nothing (all present)'} to {p['kubeconfig_dir']}")
        return 0
    if a.phase == "controlplane":
        print(f"[controlplane] Wrote static Pod manifests for {', '.join(phase_controlplane(mc, p, sub))} to {p['manifests']}")
        return 0
    if a.phase == "etcd":
        if sub not in ("all", "local"):
            raise SystemExit("error: only `etcd local` is supported")
        print(f"[etcd] {phase_etcd_local(mc, p)}")
        return 0
    kc = a.kubeconfig or os.path.join(a.base_dir, "admin.conf")

    async def cluster():
        c = _client(kc)
        try:
            if a.phase == "mark-master":
                ok = await phase_mark_master(c, mc["nodeName"])
                print(f"[markmaster] Node {mc['nodeName']} " + ("labelled and tainted as master" if ok else "not found"))
                return 0 if ok else 1
            if a.phase == "bootstrap-token":
                which = a.sub[1] if sub == "node" and len(a.sub) > 1 else sub
                done = await phase_bootstrap_token(c, mc, p, which, a.token)
                print(f"[bootstraptoken] Done: {', '.join(done)}" + (f"; token {mc['token']}" if "create" in done else ""))
                return 0
            if a.phase == "upload-config":
                await phase_upload_config(c, mc)
                print(f"[uploadconfig] Stored the configuration in ConfigMap kube-system/{CONFIG_MAP}")
                return 0
            if a.phase == "addon":
                print(f"[addons] Applied: {', '.join(await phase_addons(c, mc, p, sub))}")
                return 0
            if a.phase == "selfhosting":
                if sub not in ("all", "convert-from-staticpods"):
                    raise SystemExit("error: the selfhosting phase is `selfhosting convert-from-staticpods`")
                from .selfhosting import create_self_hosted_control_plane, secrets_of
                done = await create_self_hosted_control_plane(c, p["manifests"], mc["nodeName"], a.timeout, a.dry_run,
                                                              secrets=secrets_of(mc, p))
                if not a.dry_run:
                    print(f"[self-hosted] Converted {', '.join(done) or 'nothing (no static control-plane Pods left)'}")
                return 0
        finally:
            await c.close()
        return 1
    return asyncio.run(cluster())
