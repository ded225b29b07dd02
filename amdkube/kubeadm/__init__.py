"""kubeadm equivalent: bootstrap an MI355X cluster.

Reference cmd/kubeadm/app (1.9): `kubeadm init` runs the phases
  preflight → certs (phases/certs: CA, apiserver serving cert with the kubernetes.default SANs,
  apiserver-kubelet-client, sa key) → kubeconfig (phases/kubeconfig: admin.conf with
  O=system:masters, kubelet.conf CN=system:node:<name>, controller-manager.conf, scheduler.conf)
  → controlplane (phases/controlplane/manifests.go: static pods for apiserver,
  controller-manager and scheduler; the fork's admission list includes ResourceV2,
  manifests.go:45-47) → wait for the apiserver → markmaster (label
  node-role.kubernetes.io/master, NoSchedule taint) → bootstraptoken (token secret with
  auth + signing usages, RBAC for bootstrappers to post CSRs and be auto-approved,
  cluster-info ConfigMap in kube-public readable anonymously) → addons (kube-proxy).
  `kubeadm join` does token discovery (fetch cluster-info anonymously; check the JWS
  signature made with the token; pin the CA by the sha256 of its public key,
  --discovery-token-ca-cert-hash), then TLS bootstrap (CSR as system:bootstrap:<id>,
  auto-approved, signed by the cluster CA) and writes kubelet.conf. `kubeadm reset` undoes a
  node; `kubeadm token create|list|delete` manages bootstrap tokens.

MI355X specifics: a node that exposes /dev/kfd is labelled amd.com/gpu.present=true, and the
AMD device-plugin DaemonSet (deploy/amd-gpu-device-plugin.yaml) is an addon selecting those
nodes. Components run as `python -m amdkube <component>` static pods (image python:3).
`--start-kubelet` starts rocshim and the kubelet itself, in place of systemd.
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import hashlib
import ipaddress
import json
import os
import secrets
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GPU_LABEL = "amd.com/gpu.present"
MASTER_LABEL = "node-role.kubernetes.io/master"
BOOTSTRAP_GROUP = "system:bootstrappers:kubeadm:default-node-token"
ADMISSION = ("NamespaceLifecycle,LimitRanger,ServiceAccount,DefaultStorageClass,StorageObjectInUseProtection,"
             "DefaultTolerationSeconds,Priority,ResourceV2,ExtendedResourceToleration,NodeRestriction,ResourceQuota")


# ------------------------------------------------------------------------------ PKI
def _ssl(*args, input=None):
    r = subprocess.run(["openssl", *args], capture_output=True, input=input, timeout=60)
    if r.returncode != 0:
        raise RuntimeError(f"openssl {args[0]} failed: {r.stderr.decode()[-400:]}")
    return r.stdout


def new_ca(d, name="ca", cn="kubernetes"):
    _ssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/{name}.key", "-out", f"{d}/{name}.crt",
         "-days", "3650", "-subj", f"/CN={cn}")
    os.chmod(f"{d}/{name}.key", 0o600)


def new_cert(d, name, cn, orgs=(), sans=(), server=False, ca="ca", days=365):
    subj = "".join(f"/O={o}" for o in orgs) + f"/CN={cn}"
    _ssl("req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/{name}.key", "-out", f"{d}/{name}.csr", "-subj", subj)
    os.chmod(f"{d}/{name}.key", 0o600)
    ext = f"{d}/{name}.ext"
    with open(ext, "w") as f:
        f.write("basicConstraints=CA:FALSE\nkeyUsage=digitalSignature,keyEncipherment\n")
        f.write(f"extendedKeyUsage={'serverAuth' if server else 'clientAuth'}\n")
        if sans:
            f.write("subjectAltName=" + ",".join(sans) + "\n")
    _ssl("x509", "-req", "-in", f"{d}/{name}.csr", "-CA", f"{d}/{ca}.crt", "-CAkey", f"{d}/{ca}.key", "-CAcreateserial",
         "-CAserial", f"{d}/{ca}.srl", "-out", f"{d}/{name}.crt", "-days", str(days), "-sha256", "-extfile", ext)
    os.unlink(f"{d}/{name}.csr")
    os.unlink(ext)


def ca_cert_hash(ca_pem: bytes) -> str:
    """pubkeypin.Hash: sha256 over the DER SubjectPublicKeyInfo of the CA certificate."""
    pub = _ssl("x509", "-pubkey", "-noout", input=ca_pem)
    der = _ssl("pkey", "-pubin", "-outform", "DER", input=pub)
    return "sha256:" + hashlib.sha256(der).hexdigest()


def kubeconfig(server: str, ca_pem: bytes, user: str, cert: bytes | None = None, key: bytes | None = None,
               token: str | None = None, cluster="kubernetes") -> dict:
    u = {}
    if cert:
        u = {"client-certificate-data": base64.b64encode(cert).decode(), "client-key-data": base64.b64encode(key).decode()}
    if token:
        u["token"] = token
    ctx = f"{user}@{cluster}"
    return {"apiVersion": "v1", "kind": "Config", "current-context": ctx,
            "clusters": [{"name": cluster, "cluster": {"server": server,
                                                       "certificate-authority-data": base64.b64encode(ca_pem).decode()}}],
            "users": [{"name": user, "user": u}],
            "contexts": [{"name": ctx, "context": {"cluster": cluster, "user": user}}]}


def write_yaml(path, obj, mode=0o600):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        yaml.safe_dump(obj, f, sort_keys=False)
    os.chmod(tmp, mode)
    os.replace(tmp, path)


# --------------------------------------------------------------------------- tokens
def new_token() -> str:
    alphabet = "abcdefghijklmnopqrstuvwxyz0123456789"
    pick = lambda n: "".join(secrets.choice(alphabet) for _ in range(n))  # noqa: E731
    return f"{pick(6)}.{pick(16)}"


def token_secret(token: str, ttl: float | None = 24 * 3600, usages=("authentication", "signing"),
                 groups=(BOOTSTRAP_GROUP,), description="") -> dict:
    tid, tsec = token.split(".")
    data = {"token-id": tid, "token-secret": tsec, "auth-extra-groups": ",".join(groups), "description": description}
    for u in usages:
        data[f"usage-bootstrap-{u}"] = "true"
    if ttl:
        data["expiration"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(time.time() + ttl))
    return {"apiVersion": "v1", "kind": "Secret", "type": "bootstrap.kubernetes.io/token",
            "metadata": {"name": f"bootstrap-token-{tid}", "namespace": "kube-system"},
            "data": {k: base64.b64encode(v.encode()).decode() for k, v in data.items()}}


# ------------------------------------------------------------------- static manifests
def _component_pod(name, args, env_root=ROOT, extra_mounts=()):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "kube-system", "labels": {"component": name, "tier": "control-plane"},
                         "annotations": {"scheduler.alpha.kubernetes.io/critical-pod": ""}},
            "spec": {"hostNetwork": True, "priorityClassName": "system-cluster-critical",
                     "containers": [{"name": name, "image": "python:3", "args": ["-m", "amdkube", *args],
                                     "env": [{"name": "PYTHONPATH", "value": env_root}]}]}}


def control_plane_manifests(cfg: dict) -> dict[str, dict]:
    p, k = cfg["pki"], cfg["kubeconfig_dir"]
    api = ["apiserver", "--bind-address", cfg["advertise"], "--port", str(cfg["port"]),
           "--tls-cert-file", f"{p}/apiserver.crt", "--tls-private-key-file", f"{p}/apiserver.key",
           "--client-ca-file", f"{p}/ca.crt", "--authorization-mode", "Node,RBAC", "--anonymous-auth", "true",
           "--admission-control", ADMISSION, "--service-account-key-file", f"{p}/sa.key",
           "--service-cluster-ip-range", cfg["service_cidr"], "--data-dir", cfg["data_dir"]]
    cm = ["controller-manager", "--kubeconfig", f"{k}/controller-manager.conf", "--leader-elect", "true",
          "--service-account-private-key-file", f"{p}/sa.key", "--root-ca-file", f"{p}/ca.crt",
          "--cluster-signing-cert-file", f"{p}/ca.crt", "--cluster-signing-key-file", f"{p}/ca.key",
          "--controllers", "*,bootstrapsigner,tokencleaner", "--hostpath-pv-root", os.path.join(cfg["data_dir"], "pv")]
    if cfg.get("pod_cidr"):
        cm += ["--allocate-node-cidrs", "true", "--cluster-cidr", cfg["pod_cidr"]]
    sched = ["scheduler", "--kubeconfig", f"{k}/scheduler.conf", "--leader-elect", "true", "--port", "0"]
    out = {}
    for name, args in (("kube-apiserver", api), ("kube-controller-manager", cm), ("kube-scheduler", sched)):
        out[name] = _component_pod(name, args)
    return out


# ------------------------------------------------------------------------- helpers
def _preflight(cfg, errors_ok=()):
    errs, warns = [], []
    if shutil.which("openssl") is None:
        errs.append("openssl is required for the PKI phase")
    with socket.socket() as s:
        try:
            s.bind((cfg["advertise"], cfg["port"]))
        except OSError:
            errs.append(f"Port-{cfg['port']}: port {cfg['port']} is in use")
    if os.path.isdir(cfg["manifests"]) and os.listdir(cfg["manifests"]):
        errs.append(f"DirAvailable--{cfg['manifests']}: {cfg['manifests']} is not empty")
    if not os.path.exists("/dev/kfd"):
        warns.append("no /dev/kfd: this node has no MI355X (ROCm KFD) device; GPU pods will not schedule here")
    errs = [e for e in errs if not any(e.startswith(x) for x in errors_ok)]
    return errs, warns


def _spawn(argv, log_path, env=None):
    logf = open(log_path, "ab")
    p = subprocess.Popen([sys.executable, "-m", "amdkube", *argv], stdout=logf, stderr=subprocess.STDOUT,
                         env=dict(os.environ, PYTHONPATH=ROOT, **(env or {})), start_new_session=True)
    return p.pid


def start_node_agents(cfg, kubeconfig_path, node_name, labels=""):
    """What systemd does for the reference: rocshim + kubelet with the manifests dir."""
    d = cfg["node_dir"]
    os.makedirs(os.path.join(d, "logs"), exist_ok=True)
    sock = os.path.join(d, "rocshim.sock")
    pids = {"rocshim": _spawn(["rocshim", "--listen", sock, "--state-dir", os.path.join(d, "rocshim"),
                               "--hooks-dir", os.path.join(d, "hooks.d")], os.path.join(d, "logs", "rocshim.log"))}
    for _ in range(200):
        if os.path.exists(sock):
            break
        time.sleep(0.05)
    args = ["kubelet", "--kubeconfig", kubeconfig_path, "--node-name", node_name, "--root-dir", os.path.join(d, "kubelet"),
            "--container-runtime-endpoint", sock, "--port", str(cfg.get("kubelet_port", 0)),
            "--node-status-update-frequency", "2", "--pleg-relist-period", "0.5", "--gpu-stats-backend", "none"]
    if cfg.get("manifests"):
        args += ["--pod-manifest-path", cfg["manifests"], "--file-check-frequency", "1"]
    if labels:
        args += ["--node-labels", labels]
    pids["kubelet"] = _spawn(args, os.path.join(d, "logs", "kubelet.log"))
    with open(os.path.join(d, "pids.json"), "w") as f:
        json.dump(pids, f)
    return pids


def _client(kc_path):
    from ..client import Client
    return Client.from_kubeconfig(kc_path)


async def _wait_healthy(client, timeout):
    import aiohttp
    end = time.time() + timeout
    while time.time() < end:
        try:
            async with client.session.get(f"{client.server}/healthz", timeout=aiohttp.ClientTimeout(total=5)) as r:
                if r.status == 200 and (await r.text()).strip() == "ok":
                    return True
        except (aiohttp.ClientError, OSError, asyncio.TimeoutError):
            pass
        await asyncio.sleep(0.2)
    return False


# ---------------------------------------------------------------------------- init
def _paths(base):
    return {"base": base, "pki": os.path.join(base, "pki"), "kubeconfig_dir": base, "manifests": os.path.join(base, "manifests"),
            "data_dir": os.path.join(base, "data"), "node_dir": os.path.join(base, "node")}


def init(a) -> int:
    cfg = _paths(a.base_dir)
    cfg.update(advertise=a.apiserver_advertise_address, port=a.apiserver_bind_port, service_cidr=a.service_cidr,
               pod_cidr=a.pod_network_cidr, kubelet_port=a.kubelet_port)
    node = a.node_name or socket.gethostname()
    errs, warns = _preflight(cfg, tuple(a.ignore_preflight_errors.split(",")) if a.ignore_preflight_errors else ())
    for w in warns:
        print(f"[preflight] WARNING: {w}")
    if errs:
        print("[preflight] Some fatal errors occurred:\n" + "\n".join(f"\t[ERROR {e}]" for e in errs), file=sys.stderr)
        return 1
    for d in (cfg["pki"], cfg["manifests"], cfg["data_dir"]):
        os.makedirs(d, exist_ok=True)
    p = cfg["pki"]
    # certs
    if not os.path.exists(f"{p}/ca.crt"):
        new_ca(p)
    first_svc = str(next(ipaddress.ip_network(a.service_cidr, strict=False).hosts()))
    sans = [f"IP:{cfg['advertise']}", "IP:127.0.0.1", f"IP:{first_svc}", f"DNS:{node}", "DNS:kubernetes", "DNS:kubernetes.default",
            "DNS:kubernetes.default.svc", f"DNS:kubernetes.default.svc.{a.service_dns_domain}", "DNS:localhost"]
    new_cert(p, "apiserver", "kube-apiserver", sans=sans, server=True)
    new_cert(p, "apiserver-kubelet-client", "kube-apiserver-kubelet-client", orgs=("system:masters",))
    with open(f"{p}/sa.key", "wb") as f:
        f.write(secrets.token_hex(32).encode())
    os.chmod(f"{p}/sa.key", 0o600)
    print(f"[certificates] Generated ca, apiserver (SANs {', '.join(sans)}), apiserver-kubelet-client and sa keys in {p}")
    # kubeconfigs
    ca = open(f"{p}/ca.crt", "rb").read()
    server = f"https://{cfg['advertise']}:{cfg['port']}"
    for fname, cn, orgs in (("admin.conf", "kubernetes-admin", ("system:masters",)),
                            ("kubelet.conf", f"system:node:{node}", ("system:nodes",)),
                            ("controller-manager.conf", "system:kube-controller-manager", ()),
                            ("scheduler.conf", "system:kube-scheduler", ()),
                            ("kube-proxy.conf", "system:kube-proxy", ())):
        nm = fname[:-5]
        new_cert(p, nm, cn, orgs=orgs)
        write_yaml(os.path.join(cfg["kubeconfig_dir"], fname),
                   kubeconfig(server, ca, cn, open(f"{p}/{nm}.crt", "rb").read(), open(f"{p}/{nm}.key", "rb").read()))
    print(f"[kubeconfig] Wrote admin.conf, kubelet.conf, controller-manager.conf, scheduler.conf, kube-proxy.conf to {cfg['base']}")
    # control plane
    for name, pod in control_plane_manifests(cfg).items():
        write_yaml(os.path.join(cfg["manifests"], f"{name}.yaml"), pod, 0o644)
    print(f"[controlplane] Wrote static Pod manifests for kube-apiserver, kube-controller-manager, kube-scheduler to {cfg['manifests']}")
    if a.start_kubelet:
        labels = f"{GPU_LABEL}=true" if os.path.exists("/dev/kfd") else ""
        start_node_agents(cfg, os.path.join(cfg["base"], "kubelet.conf"), node, labels)
        print(f"[init] Started rocshim and the kubelet (logs: {cfg['node_dir']}/logs)")
    token = a.token or new_token()
    rc = asyncio.run(_post_init(cfg, node, token, a.token_ttl, a.timeout, ca, server, a.skip_addons))
    if rc != 0:
        return rc
    h = ca_cert_hash(ca)
    print("\nYour Kubernetes master has initialized successfully!\n\n"
          f"To use the cluster:  export KUBECONFIG={os.path.join(cfg['base'], 'admin.conf')}\n\n"
          "You can now join any number of machines by running the following on each node:\n\n"
          f"  python -m amdkube kubeadm join {cfg['advertise']}:{cfg['port']} --token {token} "
          f"--discovery-token-ca-cert-hash {h}\n")
    return 0


async def _post_init(cfg, node, token, ttl, timeout, ca, server, skip_addons):
    from ..api import meta as m
    c = _client(os.path.join(cfg["base"], "admin.conf"))
    try:
        print(f"[init] Waiting for the kubelet to boot up the control plane as Static Pods from {cfg['manifests']} "
              f"(timeout {timeout:.0f}s)")
        t0 = time.time()
        if not await _wait_healthy(c, timeout):
            print("[init] the control plane did not become healthy in time", file=sys.stderr)
            return 1
        print(f"[apiclient] All control plane components are healthy after {time.time() - t0:.1f} seconds")
        # markmaster
        end = time.time() + timeout
        while time.time() < end and await c.get_or_none("nodes", node) is None:
            await asyncio.sleep(0.2)
        if await c.get_or_none("nodes", node) is not None:
            await c.patch("nodes", node, {"metadata": {"labels": {MASTER_LABEL: ""}},
                                          "spec": {"taints": [{"key": MASTER_LABEL, "effect": "NoSchedule"}]}})
            print(f"[markmaster] Node {node} labelled {MASTER_LABEL}=\"\" and tainted {MASTER_LABEL}:NoSchedule")
        # bootstrap token + RBAC + cluster-info
        await _create_or_replace(c, token_secret(token, ttl, description="default kubeadm bootstrap token"))
        for o in _bootstrap_rbac():
            await _create_or_replace(c, o)
        ci = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cluster-info", "namespace": "kube-public"},
              "data": {"kubeconfig": yaml.safe_dump(kubeconfig(server, ca, "", None, None))}}
        await _create_or_replace(c, ci)
        print(f"[bootstraptoken] Using token: {token}; RBAC rules let bootstrap tokens post CSRs that are auto-approved; "
              "cluster-info published in kube-public")
        if not skip_addons:
            for o in _addons(cfg):
                await _create_or_replace(c, o)
            print("[addons] Applied essential addon: kube-proxy; AMD GPU device plugin (nodes labelled amd.com/gpu.present)")
        return 0
    finally:
        await c.close()


async def _create_or_replace(c, obj):
    from ..api import meta as m
    try:
        await c.create(obj, obj["metadata"].get("namespace"))
    except m.StatusError as e:
        if not m.is_already_exists(e):
            raise


def _bootstrap_rbac():
    rb = "rbac.authorization.k8s.io"
    return [
        {"apiVersion": f"{rb}/v1", "kind": "ClusterRoleBinding", "metadata": {"name": "kubeadm:kubelet-bootstrap"},
         "roleRef": {"apiGroup": rb, "kind": "ClusterRole", "name": "system:node-bootstrapper"},
         "subjects": [{"kind": "Group", "apiGroup": rb, "name": BOOTSTRAP_GROUP}]},
        {"apiVersion": f"{rb}/v1", "kind": "ClusterRoleBinding", "metadata": {"name": "kubeadm:node-autoapprove-bootstrap"},
         "roleRef": {"apiGroup": rb, "kind": "ClusterRole", "name": "system:certificates.k8s.io:certificatesigningrequests:nodeclient"},
         "subjects": [{"kind": "Group", "apiGroup": rb, "name": BOOTSTRAP_GROUP}]},
        {"apiVersion": f"{rb}/v1", "kind": "Role", "metadata": {"name": "kubeadm:bootstrap-signer-clusterinfo", "namespace": "kube-public"},
         "rules": [{"apiGroups": [""], "resources": ["configmaps"], "resourceNames": ["cluster-info"], "verbs": ["get"]}]},
        {"apiVersion": f"{rb}/v1", "kind": "RoleBinding", "metadata": {"name": "kubeadm:bootstrap-signer-clusterinfo",
                                                                        "namespace": "kube-public"},
         "roleRef": {"apiGroup": rb, "kind": "Role", "name": "kubeadm:bootstrap-signer-clusterinfo"},
         "subjects": [{"kind": "User", "apiGroup": rb, "name": "system:anonymous"}]},
    ]


def _addons(cfg):
    proxy = {"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "kube-proxy", "namespace": "kube-system",
                                                                         "labels": {"k8s-app": "kube-proxy"}},
             "spec": {"selector": {"matchLabels": {"k8s-app": "kube-proxy"}},
                      "template": {"metadata": {"labels": {"k8s-app": "kube-proxy"}},
                                   "spec": {"hostNetwork": True, "tolerations": [{"key": MASTER_LABEL, "effect": "NoSchedule"}],
                                            "containers": [{"name": "kube-proxy", "image": "python:3",
                                                            "args": ["-m", "amdkube", "proxy", "--kubeconfig",
                                                                     os.path.join(cfg["base"], "kube-proxy.conf"),
                                                                     "--healthz-port", "0", "--bind-address", "127.0.0.1"],
                                                            "env": [{"name": "PYTHONPATH", "value": ROOT}]}]}}}}
    from ..api.scheme import load_manifests
    out = [proxy]
    for d in load_manifests(open(os.path.join(ROOT, "deploy", "amd-gpu-device-plugin.yaml")).read()):
        if d and d.get("kind") == "DaemonSet":
            tpl = d["spec"]["template"]["spec"]
            tpl.setdefault("nodeSelector", {})[GPU_LABEL] = "true"
            for ct in tpl.get("containers") or []:
                ct.setdefault("env", []).append({"name": "PYTHONPATH", "value": ROOT})
            d["metadata"].setdefault("namespace", "kube-system")
            out.append(d)
    return out


# ---------------------------------------------------------------------------- join
async def discover(server: str, token: str, ca_hash: str | None, unsafe_skip: bool) -> bytes:
    """discovery/token: fetch cluster-info anonymously, verify the JWS, pin the CA."""
    from ..client import Client
    from ..controllers.accounts import verify_detached_jws
    tid, tsec = token.split(".")
    c = Client(server, insecure=True)
    try:
        end = time.time() + 60
        while True:
            try:
                cm = await c.get("configmaps", "cluster-info", "kube-public")
            except Exception:
                if time.time() > end:
                    raise
                await asyncio.sleep(0.5)
                continue
            jws = (cm.get("data") or {}).get(f"jws-kubeconfig-{tid}")
            if jws:
                break
            if time.time() > end:
                raise RuntimeError(f"there is no JWS signed token in the cluster-info ConfigMap for token ID {tid!r}")
            await asyncio.sleep(0.5)   # the bootstrap signer has not signed yet
    finally:
        await c.close()
    payload = cm["data"]["kubeconfig"]
    if not verify_detached_jws(jws, payload, tid, tsec):
        raise RuntimeError("failed to verify JWS signature of received cluster info object, can't trust this API Server")
    kc = yaml.safe_load(payload)
    ca = base64.b64decode(kc["clusters"][0]["cluster"]["certificate-authority-data"])
    if ca_hash:
        got = ca_cert_hash(ca)
        if got != ca_hash:
            raise RuntimeError(f"cluster CA found in cluster-info configmap does not match the pin: {got}")
    elif not unsafe_skip:
        raise RuntimeError("using token-based discovery without --discovery-token-ca-cert-hash can be unsafe; "
                           "pass --discovery-token-unsafe-skip-ca-verification to proceed")
    return ca


async def tls_bootstrap(server: str, ca: bytes, token: str, node: str, d: str, timeout: float = 60.0):
    """kubelet/certificate/bootstrap: key + CSR as the bootstrap identity, wait for the signed cert."""
    from ..client import Client
    new_key_csr = ["req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/kubelet-client.key", "-out",
                   f"{d}/kubelet-client.csr", "-subj", f"/O=system:nodes/CN=system:node:{node}"]
    _ssl(*new_key_csr)
    os.chmod(f"{d}/kubelet-client.key", 0o600)
    csr_pem = open(f"{d}/kubelet-client.csr", "rb").read()
    c = Client(server, token=token, ca_data=ca.decode())
    name = f"node-csr-{hashlib.sha256(csr_pem).hexdigest()[:20]}"
    try:
        await c.create({"apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest", "metadata": {"name": name},
                        "spec": {"request": base64.b64encode(csr_pem).decode(),
                                 "usages": ["digital signature", "key encipherment", "client auth"]}})
        end = time.time() + timeout
        while time.time() < end:
            o = await c.get("certificatesigningrequests", name)
            cert = (o.get("status") or {}).get("certificate")
            if cert:
                return base64.b64decode(cert), open(f"{d}/kubelet-client.key", "rb").read()
            if any(x.get("type") == "Denied" for x in (o.get("status") or {}).get("conditions") or []):
                raise RuntimeError(f"certificate signing request {name} was denied")
            await asyncio.sleep(0.3)
        raise RuntimeError(f"timed out waiting for the certificate of {name}")
    finally:
        await c.close()


def join(a) -> int:
    node = a.node_name or socket.gethostname()
    server = a.server if a.server.startswith("https://") else f"https://{a.server}"
    cfg = _paths(a.base_dir)
    os.makedirs(cfg["pki"], exist_ok=True)
    print(f"[discovery] Trying to connect to API Server {server!r}")
    ca = asyncio.run(discover(server, a.token, a.discovery_token_ca_cert_hash, a.discovery_token_unsafe_skip_ca_verification))
    with open(f"{cfg['pki']}/ca.crt", "wb") as f:
        f.write(ca)
    print("[discovery] Cluster info signature and contents are valid" +
          (" and the CA matches the pinned hash" if a.discovery_token_ca_cert_hash else ""))
    cert, key = asyncio.run(tls_bootstrap(server, ca, a.token, node, cfg["pki"], a.timeout))
    kc_path = os.path.join(cfg["base"], "kubelet.conf")
    write_yaml(kc_path, kubeconfig(server, ca, f"system:node:{node}", cert, key))
    print(f"[bootstrap] Received signed certificate for system:node:{node}; wrote {kc_path}")
    if a.start_kubelet:
        cfg["manifests"] = None
        labels = f"{GPU_LABEL}=true" if os.path.exists("/dev/kfd") else ""
        start_node_agents(dict(cfg, kubelet_port=a.kubelet_port), kc_path, node, labels)
        print(f"[join] Started rocshim and the kubelet (logs: {cfg['node_dir']}/logs)")
    print("\nThis node has joined the cluster:\n* Certificate signing request was sent to master and a response was received.\n"
          "* The Kubelet was informed of the new secure connection details.\n\n"
          "Run 'kubectl get nodes' on the master to see this node join the cluster.")
    return 0


# --------------------------------------------------------------------------- reset
def reset(a) -> int:
    cfg = _paths(a.base_dir)
    pids = os.path.join(cfg["node_dir"], "pids.json")
    man = cfg["manifests"]
    if os.path.isdir(man):   # the kubelet tears static pods down once their manifests go
        for f in os.listdir(man):
            os.unlink(os.path.join(man, f))
        time.sleep(a.drain_seconds)
    if os.path.exists(pids):
        for name, pid in reversed(list(json.load(open(pids)).items())):
            try:
                os.killpg(pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    # what `docker rm -f` does in the reference's reset: every container and sandbox the
    # runtime still tracks (each runs in its own session)
    for kind in ("containers", "sandboxes"):
        sd = os.path.join(cfg["node_dir"], "rocshim", kind)
        for f in [x for x in os.listdir(sd) if x.endswith(".json")] if os.path.isdir(sd) else ():
            try:
                pid = json.load(open(os.path.join(sd, f))).get("pid") or 0
                if pid > 1:
                    os.killpg(pid, signal.SIGKILL)
            except (OSError, ValueError, ProcessLookupError):
                pass
    shutil.rmtree(cfg["base"], ignore_errors=True)
    print(f"[reset] Stopped the node agents and removed {cfg['base']}")
    return 0


# --------------------------------------------------------------------------- token
def token_cmd(a) -> int:
    c = _client(a.kubeconfig)

    async def run():
        from ..api import meta as m
        try:
            if a.token_op == "create":
                t = a.token or new_token()
                await c.create(token_secret(t, a.ttl or None, description=a.description or ""), "kube-system")
                print(t)
            elif a.token_op == "list":
                items, _ = await c.list("secrets", "kube-system")
                print(f"{'TOKEN':<24}{'TTL':<10}{'EXPIRES':<22}{'USAGES':<28}DESCRIPTION")
                for s in items:
                    if s.get("type") != "bootstrap.kubernetes.io/token":
                        continue
                    d = {k: base64.b64decode(v).decode() for k, v in (s.get("data") or {}).items()}
                    exp = m.parse_time(d.get("expiration"))
                    ttl = f"{max(0, int((exp - time.time()) / 3600))}h" if exp else "<forever>"
                    usages = ",".join(k[len("usage-bootstrap-"):] for k, v in d.items() if k.startswith("usage-bootstrap-") and v == "true")
                    print(f"{d.get('token-id', '')}.{d.get('token-secret', '')}".ljust(24) + ttl.ljust(10) +
                          (d.get("expiration") or "<never>").ljust(22) + usages.ljust(28) + d.get("description", ""))
            elif a.token_op == "delete":
                tid = a.token.split(".")[0]
                await c.delete("secrets", f"bootstrap-token-{tid}", "kube-system")
                print(f"bootstrap token {tid!r} deleted")
        finally:
            await c.close()
    asyncio.run(run())
    return 0


def main(argv) -> int:
    ap = argparse.ArgumentParser("amdkube kubeadm")
    sub = ap.add_subparsers(dest="cmd", required=True)
    i = sub.add_parser("init")
    i.add_argument("--base-dir", default="/etc/kubernetes")
    i.add_argument("--apiserver-advertise-address", default="127.0.0.1")
    i.add_argument("--apiserver-bind-port", type=int, default=6443)
    i.add_argument("--service-cidr", default="10.96.0.0/12")
    i.add_argument("--service-dns-domain", default="cluster.local")
    i.add_argument("--pod-network-cidr", default=None)
    i.add_argument("--node-name", default=None)
    i.add_argument("--token", default=None)
    i.add_argument("--token-ttl", type=float, default=24 * 3600.0)
    i.add_argument("--ignore-preflight-errors", default="")
    i.add_argument("--skip-addons", action="store_true")
    i.add_argument("--start-kubelet", action="store_true", help="start rocshim + kubelet (what systemd does for kubeadm)")
    i.add_argument("--kubelet-port", type=int, default=10250)
    i.add_argument("--timeout", type=float, default=120.0)
    j = sub.add_parser("join")
    j.add_argument("server")
    j.add_argument("--token", required=True)
    j.add_argument("--discovery-token-ca-cert-hash", default=None)
    j.add_argument("--discovery-token-unsafe-skip-ca-verification", action="store_true")
    j.add_argument("--node-name", default=None)
    j.add_argument("--base-dir", default="/etc/kubernetes")
    j.add_argument("--start-kubelet", action="store_true")
    j.add_argument("--kubelet-port", type=int, default=10250)
    j.add_argument("--timeout", type=float, default=60.0)
    r = sub.add_parser("reset")
    r.add_argument("--base-dir", default="/etc/kubernetes")
    r.add_argument("--drain-seconds", type=float, default=2.0)
    t = sub.add_parser("token")
    t.add_argument("token_op", choices=("create", "list", "delete"))
    t.add_argument("token", nargs="?", default=None)
    t.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
    t.add_argument("--ttl", type=float, default=24 * 3600.0)
    t.add_argument("--description", default="")
    a = ap.parse_args(argv)
    return {"init": init, "join": join, "reset": reset, "token": token_cmd}[a.cmd](a)
