"""Process and host setup the kubelet does before it starts (cmd/kubelet/app/server.go run():
lock file, swap check, oom_score_adj, RLIMIT_NOFILE; cm/container_manager_linux.go
setupKernelTunables; pkg/kubelet/certificate/bootstrap/bootstrap.go LoadClientCert).

* `acquire_lock(path, exit_on_contention)` — --lock-file: flock the file; with
  --exit-on-lock-contention the kubelet exits as soon as another process asks for the lock
  (that process opens the file and the kubelet watches it with inotify).
* `check_swap()` — --fail-swap-on: refuse to run with swap enabled.
* `apply_oom_score_adj(v)`, `raise_nofile(n)` — --oom-score-adj, --max-open-files.
* `kernel_tunables(protect)` — --protect-kernel-defaults: the kernel settings the kubelet needs
  (vm.overcommit_memory=1, vm.panic_on_oom=0, kernel.panic=10, kernel.panic_on_oops=1); with
  protection on a mismatch is an error, otherwise the kubelet sets them (when it may).
* `bootstrap_client_cert(...)` — --bootstrap-kubeconfig: when --kubeconfig does not exist yet,
  use the bootstrap token to post a node CSR, wait for the signed certificate, store it in
  --cert-dir and write a --kubeconfig that uses it.
"""
from __future__ import annotations

import base64
import fcntl
import logging
import os
import resource

import yaml

log = logging.getLogger("amdkube.kubelet.setup")

TUNABLES = {"vm/overcommit_memory": 1, "vm/panic_on_oom": 0, "kernel/panic": 10, "kernel/panic_on_oops": 1}


def acquire_lock(path: str, exit_on_contention: bool = False, on_contention=None):
    """Returns the open lock file (keep it referenced for the process lifetime)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    f = open(path, "a+")
    try:
        fcntl.flock(f.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
    except BlockingIOError:
        if exit_on_contention:
            raise SystemExit(f"kubelet: lock {path} is held by another process")
        log.info("waiting for the lock %s", path)
        fcntl.flock(f.fileno(), fcntl.LOCK_EX)
    if exit_on_contention and on_contention is not None:
        _watch_open(path, on_contention)
    return f


def _watch_open(path: str, callback):
    """inotify IN_OPEN on the lock file: the next contender opening it triggers `callback`."""
    import ctypes
    import threading
    libc = ctypes.CDLL(None, use_errno=True)
    fd = libc.inotify_init1(os.O_CLOEXEC)
    if fd < 0 or libc.inotify_add_watch(fd, os.fsencode(path), 0x00000020) < 0:    # IN_OPEN
        log.warning("cannot watch %s for lock contention", path)
        return

    def run():
        os.read(fd, 4096)
        callback()
    threading.Thread(target=run, name="lock-contention", daemon=True).start()


def check_swap(swaps: str = "/proc/swaps"):
    try:
        lines = open(swaps).read().splitlines()[1:]
    except OSError:
        return
    if any(ln.strip() for ln in lines):
        raise SystemExit("kubelet: running with swap on is not supported, please disable swap or set --fail-swap-on "
                         f"flag to false. /proc/swaps contained: {lines}")


def apply_oom_score_adj(value: int, pid: str = "self") -> bool:
    try:
        with open(f"/proc/{pid}/oom_score_adj", "w") as f:
            f.write(str(value))
        return True
    except OSError as e:       # lowering the score needs CAP_SYS_RESOURCE
        log.info("cannot set oom_score_adj=%d: %s", value, e)
        return False


def raise_nofile(n: int) -> int:
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = n if hard == resource.RLIM_INFINITY else min(n, hard)
    try:
        resource.setrlimit(resource.RLIMIT_NOFILE, (want, max(hard, want) if hard != resource.RLIM_INFINITY else hard))
    except (ValueError, OSError):
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (min(n, hard), hard))
        except (ValueError, OSError) as e:
            log.info("cannot raise RLIMIT_NOFILE to %d: %s", n, e)
    return resource.getrlimit(resource.RLIMIT_NOFILE)[0]


def kernel_tunables(protect: bool, root: str = "/proc/sys") -> list[str]:
    """The mismatched settings (after trying to fix them when not protected)."""
    bad = []
    for key, want in TUNABLES.items():
        path = os.path.join(root, key)
        try:
            cur = int(open(path).read().strip())
        except (OSError, ValueError):
            continue
        if cur == want:
            continue
        if protect:
            bad.append(f"{key.replace('/', '.')}: want {want}, have {cur}")
            continue
        try:
            with open(path, "w") as f:
                f.write(str(want))
        except OSError:
            bad.append(f"{key.replace('/', '.')}: want {want}, have {cur} (not permitted to set)")
    if protect and bad:
        raise SystemExit("kubelet: --protect-kernel-defaults is set and the kernel settings differ: " + "; ".join(bad))
    return bad


def bootstrap_client_cert(kubeconfig_path: str, bootstrap_path: str, cert_dir: str, node_name: str,
                          timeout: float = 300.0) -> bool:
    """False when --kubeconfig already exists (nothing to do), True after bootstrapping."""
    if os.path.exists(kubeconfig_path):
        return False
    import asyncio
    from ..kubeadm import tls_bootstrap
    kc = yaml.safe_load(open(bootstrap_path))
    ctx_name = kc.get("current-context")
    ctx = next((c["context"] for c in kc.get("contexts") or [] if c["name"] == ctx_name), None) or \
        (kc.get("contexts") or [{}])[0].get("context", {})
    cluster = next(c["cluster"] for c in kc["clusters"] if not ctx.get("cluster") or c["name"] == ctx["cluster"])
    user = next((u["user"] for u in kc.get("users") or [] if u["name"] == ctx.get("user")), None) or \
        (kc.get("users") or [{}])[0].get("user", {})
    token = user.get("token")
    if not token:
        raise SystemExit(f"kubelet: the bootstrap kubeconfig {bootstrap_path} has no token")
    if cluster.get("certificate-authority-data"):
        ca = base64.b64decode(cluster["certificate-authority-data"])
    else:
        ca = open(cluster["certificate-authority"], "rb").read()
    os.makedirs(cert_dir, exist_ok=True)
    log.info("bootstrapping the client certificate of system:node:%s through %s", node_name, cluster["server"])
    cert, _key = asyncio.run(tls_bootstrap(cluster["server"], ca, token, node_name, cert_dir, timeout))
    crt_path, key_path = os.path.join(cert_dir, "kubelet-client.crt"), os.path.join(cert_dir, "kubelet-client.key")
    with open(crt_path, "wb") as f:
        f.write(cert)
    user_name = f"system:node:{node_name}"
    out = {"apiVersion": "v1", "kind": "Config", "current-context": "default-context",
           "clusters": [{"name": "default-cluster", "cluster": {"server": cluster["server"],
                                                                "certificate-authority-data": base64.b64encode(ca).decode()}}],
           "users": [{"name": user_name, "user": {"client-certificate": crt_path, "client-key": key_path}}],
           "contexts": [{"name": "default-context", "context": {"cluster": "default-cluster", "user": user_name}}]}
    os.makedirs(os.path.dirname(os.path.abspath(kubeconfig_path)), exist_ok=True)
    tmp = kubeconfig_path + ".tmp"
    with open(tmp, "w") as f:
        yaml.safe_dump(out, f, sort_keys=False)
    os.chmod(tmp, 0o600)
    os.replace(tmp, kubeconfig_path)
    return True
