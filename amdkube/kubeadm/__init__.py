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
  node; `kubeadm token create|list|delete|generate` manages bootstrap tokens.
  The phases themselves live in phases.py (`kubeadm alpha phase ...`), the stored
  MasterConfiguration behind `kubeadm config view|upload|print-default`, and `kubeadm upgrade
  plan|apply` in upgrade.py.

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
import json
import os
import secrets
import shutil
import signal
import socket
import subprocess
import sys
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
    """`server`: False = client cert, True = server cert, "peer" = both (etcd peer certs)."""
    subj = "".join(f"/O={o}" for o in orgs) + f"/CN={cn}"
    _ssl("req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/{name}.key", "-out", f"{d}/{name}.csr", "-subj", subj)
    os.chmod(f"{d}/{name}.key", 0o600)
    ext = f"{d}/{name}.ext"
    eku = "serverAuth,clientAuth" if server == "peer" else "serverAuth" if server else "clientAuth"
    with open(ext, "w") as f:
        f.write("basicConstraints=CA:FALSE\nkeyUsage=digitalSignature,keyEncipherment\n")
        f.write(f"extendedKeyUsage={eku}\n")
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


# ------------------------------------------------------------------------- helpers
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
    if not cfg.get("kubelet_port"):     # an ephemeral API port: several kubelets share this host (tests)
        args += ["--read-only-port", "0", "--healthz-port", "0"]
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
    """`kubeadm init`: every phase of phases.py in order (cmd/init.go Run)."""
    from . import phases as ph
    mc = ph.master_config(a)
    cfg = ph.paths(a.base_dir, mc)
    cfg.update(advertise=mc["api"]["advertiseAddress"], port=mc["api"]["bindPort"], kubelet_port=a.kubelet_port)
    node = mc["nodeName"]
    errs, warns = ph.phase_preflight(mc, cfg, tuple(x for x in a.ignore_preflight_errors.split(",") if x))
    for w in warns:
        print(f"[preflight] WARNING: {w}")
    if errs:
        print("[preflight] Some fatal errors occurred:\n" + "\n".join(f"\t[ERROR {e}]" for e in errs), file=sys.stderr)
        return 1
    os.makedirs(cfg["base"], exist_ok=True)
    done = ph.phase_certs(mc, cfg)
    print(f"[certificates] Generated {', '.join(done)} in {cfg['pki']} (apiserver SANs {', '.join(ph.apiserver_sans(mc))})")
    done = ph.phase_kubeconfig(mc, cfg)
    print(f"[kubeconfig] Wrote {', '.join(done)} to {cfg['base']}")
    print(f"[controlplane] Wrote static Pod manifests for {', '.join(ph.phase_controlplane(mc, cfg))} to {cfg['manifests']}")
    print(f"[etcd] {ph.phase_etcd_local(mc, cfg)}")
    if a.start_kubelet:
        labels = f"{GPU_LABEL}=true" if os.path.exists("/dev/kfd") else ""
        start_node_agents(cfg, os.path.join(cfg["base"], "kubelet.conf"), node, labels)
        print(f"[init] Started rocshim and the kubelet (logs: {cfg['node_dir']}/logs)")
    rc = asyncio.run(_post_init(mc, cfg, a.timeout, a.skip_addons))
    if rc != 0:
        return rc
    ca = open(os.path.join(cfg["pki"], "ca.crt"), "rb").read()
    h = ca_cert_hash(ca)
    print("\nYour Kubernetes master has initialized successfully!\n\n"
          f"To use the cluster:  export KUBECONFIG={os.path.join(cfg['base'], 'admin.conf')}\n\n"
          "You can now join any number of machines by running the following on each node:\n\n"
          f"  python -m amdkube kubeadm join {cfg['advertise']}:{cfg['port']} --token {mc['token']} "
          f"--discovery-token-ca-cert-hash {h}\n")
    return 0


async def _post_init(mc, cfg, timeout, skip_addons):
    from . import phases as ph
    c = _client(os.path.join(cfg["base"], "admin.conf"))
    try:
        print(f"[init] Waiting for the kubelet to boot up the control plane as Static Pods from {cfg['manifests']} "
              f"(timeout {timeout:.0f}s)")
        t0 = time.time()
        if not await _wait_healthy(c, timeout):
            print("[init] the control plane did not become healthy in time", file=sys.stderr)
            return 1
        print(f"[apiclient] All control plane components are healthy after {time.time() - t0:.1f} seconds")
        if await ph.phase_mark_master(c, mc["nodeName"], timeout):
            print(f"[markmaster] Node {mc['nodeName']} labelled {MASTER_LABEL}=\"\" and tainted {MASTER_LABEL}:NoSchedule")
        await ph.phase_bootstrap_token(c, mc, cfg)
        print(f"[bootstraptoken] Using token: {mc['token']}; RBAC rules let bootstrap tokens post CSRs that are auto-approved; "
              "cluster-info published in kube-public")
        await ph.phase_upload_config(c, mc)
        print(f"[uploadconfig] Storing the configuration used in ConfigMap kube-system/{ph.CONFIG_MAP}")
        if not skip_addons:
            done = await ph.phase_addons(c, mc, cfg)
            print(f"[addons] Applied essential addons: {', '.join(done)} (the AMD GPU device plugin runs on nodes "
                  f"labelled {GPU_LABEL})")
        if (mc.get("featureGates") or {}).get("SelfHosting"):
            from .selfhosting import create_self_hosted_control_plane, secrets_of
            print("[self-hosted] Creating self-hosted control plane.")
            await create_self_hosted_control_plane(c, cfg["manifests"], mc["nodeName"], timeout,
                                                   secrets=secrets_of(mc, cfg))
        return 0
    finally:
        await c.close()


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
    etcd_dir = _local_etcd_data_dir(man)
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
    # unmountKubeletDirectory: volumes (secret/configMap tmpfs, bind mounts) still mounted under
    # the kubelet's root would survive the rmtree below
    from ..volume.mount import unmount_under
    unmount_under(cfg["base"])
    shutil.rmtree(cfg["base"], ignore_errors=True)
    if etcd_dir:                    # resetEtcd: the local etcd's data directory goes too
        shutil.rmtree(etcd_dir, ignore_errors=True)
    print(f"[reset] Stopped the node agents and removed {cfg['base']}" + (f" and {etcd_dir}" if etcd_dir else ""))
    return 0


def _local_etcd_data_dir(manifests: str) -> str | None:
    """--data-dir of the local etcd static Pod, read before its manifest goes (reset.go getEtcdDataDir)."""
    path = os.path.join(manifests, "etcd.yaml")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pod = yaml.safe_load(f) or {}
    args = ((pod.get("spec") or {}).get("containers") or [{}])[0].get("args") or []
    return args[args.index("--data-dir") + 1] if "--data-dir" in args[:-1] else None


# --------------------------------------------------------------------------- token
def _kubeconfig_ca(path: str) -> bytes:
    kc = yaml.safe_load(open(path))
    cl = kc["clusters"][0]["cluster"]
    if cl.get("certificate-authority-data"):
        return base64.b64decode(cl["certificate-authority-data"])
    return open(cl["certificate-authority"], "rb").read()


def token_cmd(a) -> int:
    if a.token_op == "generate":        # offline: just a well-formed random token
        print(new_token())
        return 0
    c = _client(a.kubeconfig)

    async def run():
        from ..api import meta as m
        try:
            if a.token_op == "create":
                t = a.token or new_token()
                await c.create(token_secret(t, a.ttl or None, usages=tuple(a.usages.split(",")),
                                            groups=tuple(a.groups.split(",")), description=a.description or ""), "kube-system")
                if a.print_join_command:
                    ca = _kubeconfig_ca(a.kubeconfig)
                    print(f"python -m amdkube kubeadm join {c.server.split('://', 1)[1]} --token {t} "
                          f"--discovery-token-ca-cert-hash {ca_cert_hash(ca)}")
                else:
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


def config_cmd(a) -> int:
    """kubeadm config view | upload from-file | upload from-flags | print-default (cmd/config.go)."""
    from . import phases as ph
    if a.config_op == "print-default":
        mc = ph.master_config(a)
        mc["nodeName"] = "<node name>"
        print(yaml.safe_dump(mc, sort_keys=False), end="")
        return 0

    async def run():
        c = _client(a.kubeconfig)
        try:
            if a.config_op == "view":
                cm = await c.get_or_none("configmaps", ph.CONFIG_MAP, "kube-system")
                if cm is None:
                    print(f"error: ConfigMap kube-system/{ph.CONFIG_MAP} not found (run `kubeadm config upload`)", file=sys.stderr)
                    return 1
                print(f"[config] Configuration of the cluster, from ConfigMap kube-system/{ph.CONFIG_MAP}:\n")
                print((cm.get("data") or {}).get(ph.CONFIG_KEY, ""), end="")
                return 0
            if a.config_op == "upload":
                if a.source == "from-file" and not a.config:
                    print("error: from-file needs --config", file=sys.stderr)
                    return 1
                mc = ph.master_config(a)
                await ph.phase_upload_config(c, mc)
                print(f"[uploadconfig] Stored the configuration in ConfigMap kube-system/{ph.CONFIG_MAP}")
                return 0
            return 1
        finally:
            await c.close()
    return asyncio.run(run())


def version_cmd(a) -> int:
    from .. import GIT_VERSION
    info = {"major": "1", "minor": "9", "gitVersion": GIT_VERSION, "platform": "linux/amd64", "compiler": "cpython"}
    if a.output == "short":
        print(GIT_VERSION)
    elif a.output == "json":
        print(json.dumps({"clientVersion": info}, indent=2))
    elif a.output == "yaml":
        print(yaml.safe_dump({"clientVersion": info}, sort_keys=False), end="")
    else:
        print(f"kubeadm version: &version.Info{{Major:\"1\", Minor:\"9\", GitVersion:\"{GIT_VERSION}\", "
              f"Platform:\"linux/amd64\", Compiler:\"cpython\"}}")
    return 0


def _cluster_flags(p, defaults=True):
    p.add_argument("--base-dir", default="/etc/kubernetes")
    p.add_argument("--config", default=None, help="a kubeadm.k8s.io/v1alpha1 MasterConfiguration file")
    p.add_argument("--apiserver-advertise-address", default="127.0.0.1" if defaults else None)
    p.add_argument("--apiserver-bind-port", type=int, default=6443 if defaults else None)
    p.add_argument("--apiserver-cert-extra-sans", default="")
    p.add_argument("--service-cidr", default="10.96.0.0/12" if defaults else None)
    p.add_argument("--service-dns-domain", default="cluster.local" if defaults else None)
    p.add_argument("--pod-network-cidr", default=None)
    p.add_argument("--node-name", default=None)
    p.add_argument("--kubernetes-version", default=None)
    p.add_argument("--feature-gates", default="")
    p.add_argument("--token", default=None)
    p.add_argument("--token-ttl", type=float, default=24 * 3600.0)


def main(argv) -> int:
    ap = argparse.ArgumentParser("amdkube kubeadm")
    sub = ap.add_subparsers(dest="cmd", required=True)
    i = sub.add_parser("init")
    _cluster_flags(i)
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
    t.add_argument("token_op", choices=("create", "list", "delete", "generate"))
    t.add_argument("token", nargs="?", default=None)
    t.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
    t.add_argument("--ttl", type=float, default=24 * 3600.0)
    t.add_argument("--description", default="")
    t.add_argument("--usages", default="signing,authentication")
    t.add_argument("--groups", default=BOOTSTRAP_GROUP)
    t.add_argument("--print-join-command", action="store_true")
    cf = sub.add_parser("config")
    cf.add_argument("config_op", choices=("view", "upload", "print-default"))
    cf.add_argument("source", nargs="?", choices=("from-file", "from-flags"), default="from-flags")
    cf.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
    _cluster_flags(cf)
    al = sub.add_parser("alpha")
    alsub = al.add_subparsers(dest="alpha_cmd", required=True)
    from .phases import add_phase_parser, run_phase
    add_phase_parser(alsub)
    from . import upgrade
    upgrade.add_parser(sub)
    v = sub.add_parser("version")
    v.add_argument("-o", "--output", default="", choices=("", "short", "json", "yaml"))
    a = ap.parse_args(argv)
    return {"init": init, "join": join, "reset": reset, "token": token_cmd, "config": config_cmd,
            "alpha": run_phase, "upgrade": upgrade.run, "version": version_cmd}[a.cmd](a)
