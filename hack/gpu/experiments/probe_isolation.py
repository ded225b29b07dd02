"""Probe which device-isolation mechanisms an (unprivileged) node offers.

Prints one JSON object: identity, capabilities, LSMs, user-namespace sysctls, whether an
unprivileged user+mount namespace can hide /dev/dri nodes and bind one back, whether a PID
namespace can mount its own /proc, the Landlock ABI, cgroup-v2 delegation, and whether the
GPU opens from inside such a namespace. Every experiment runs in a forked child so this
process is never changed.   python hack/gpu/experiments/probe_isolation.py > gpurun_out/iso_probe.json
"""
from __future__ import annotations

import ctypes
import errno
import glob
import json
import os
import platform
import subprocess
import sys

libc = ctypes.CDLL(None, use_errno=True)
CLONE_NEWNS, CLONE_NEWUSER, CLONE_NEWPID = 0x00020000, 0x10000000, 0x20000000
MS_BIND, MS_REC, MS_PRIVATE = 4096, 16384, 1 << 18
SYS_landlock_create_ruleset = 444


def _read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.strerror}>"


def _status():
    out = {}
    for line in _read("/proc/self/status").splitlines():
        k, _, v = line.partition(":")
        if k in ("Uid", "Gid", "Groups", "CapInh", "CapPrm", "CapEff", "CapBnd", "CapAmb", "NoNewPrivs", "Seccomp"):
            out[k] = v.strip()
    return out


def _child(fn):
    """Run fn() in a forked child; its return (a JSON-able value) comes back over a pipe."""
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        try:
            res = fn()
        except Exception as e:  # noqa: BLE001
            res = {"error": repr(e)}
        os.write(w, json.dumps(res).encode())
        os._exit(0)
    os.close(w)
    data = b""
    while True:
        chunk = os.read(r, 65536)
        if not chunk:
            break
        data += chunk
    os.waitpid(pid, 0)
    return json.loads(data or b"null")


def _err():
    e = ctypes.get_errno()
    return f"{errno.errorcode.get(e, e)}"


def _enter_userns(extra=0):
    uid, gid = os.getuid(), os.getgid()
    if libc.unshare(CLONE_NEWUSER | CLONE_NEWNS | extra) != 0:
        return "unshare " + _err()
    try:
        with open("/proc/self/setgroups", "w") as f:
            f.write("deny")
        with open("/proc/self/uid_map", "w") as f:
            f.write(f"0 {uid} 1")
        with open("/proc/self/gid_map", "w") as f:
            f.write(f"0 {gid} 1")
    except OSError as e:
        return f"idmap {e.strerror}"
    if libc.mount(None, b"/", None, MS_REC | MS_PRIVATE, None) != 0:
        return "rprivate " + _err()
    return None


def userns_dev():
    res = {}
    err = _enter_userns()
    if err:
        return {"ok": False, "error": err}
    nodes = sorted(glob.glob("/dev/dri/renderD*"))
    res["render_nodes"] = nodes
    keep = nodes[:1]
    fds = [os.open(k, os.O_PATH) for k in keep]
    if libc.mount(b"tmpfs", b"/dev/dri", b"tmpfs", 0, b"mode=755,size=64k") != 0:
        return {"ok": False, "error": "tmpfs on /dev/dri " + _err()}
    for k, fd in zip(keep, fds):
        t = "/dev/dri/" + os.path.basename(k)
        open(t, "w").close()
        if libc.mount(f"/proc/self/fd/{fd}".encode(), t.encode(), None, MS_BIND, None) != 0:
            return {"ok": False, "error": "bind " + _err()}
    res["visible_after"] = sorted(os.listdir("/dev/dri"))
    for k in keep:
        try:
            os.close(os.open(k, os.O_RDWR))
            res["open_kept"] = "ok"
        except OSError as e:
            res["open_kept"] = e.strerror
    if len(nodes) > 1:
        try:
            os.open(nodes[1], os.O_RDWR)
            res["open_hidden"] = "OPENED (isolation broken)"
        except OSError as e:
            res["open_hidden"] = errno.errorcode.get(e.errno, e.errno)
    if libc.mount(b"/dev/null", b"/dev/kfd", None, MS_BIND, None) != 0:
        res["hide_kfd"] = "bind " + _err()
    else:
        try:
            fd = os.open("/dev/kfd", os.O_RDWR)
            st = os.fstat(fd)
            res["hide_kfd"] = f"kfd now rdev {os.major(st.st_rdev)}:{os.minor(st.st_rdev)}"
            os.close(fd)
        except OSError as e:
            res["hide_kfd"] = e.strerror
    try:
        os.mknod("/tmp/amdkube-probe-node", 0o600 | 0o020000, os.makedev(226, 129))
        res["mknod"] = "ALLOWED"
        os.unlink("/tmp/amdkube-probe-node")
    except OSError as e:
        res["mknod"] = errno.errorcode.get(e.errno, e.errno)
    # a process of the same uid outside the namespace: /proc/<pid>/root reaches the host /dev
    if len(nodes) > 1:
        try:
            os.close(os.open(f"/proc/{os.getppid()}/root{nodes[1]}", os.O_RDWR))
            res["proc_root_escape"] = "OPENED via /proc/<ppid>/root"
        except OSError as e:
            res["proc_root_escape"] = errno.errorcode.get(e.errno, e.errno)
    res["ok"] = True
    return res


def pidns_proc():
    err = _enter_userns(CLONE_NEWPID)
    if err:
        return {"ok": False, "error": err}
    pid = os.fork()
    if pid == 0:
        rc = libc.mount(b"proc", b"/proc", b"proc", 0, None)
        e = ctypes.get_errno()
        os._exit(0 if rc == 0 else min(e, 250))
    _, st = os.waitpid(pid, 0)
    code = os.waitstatus_to_exitcode(st)
    return {"ok": code == 0, "mount_proc": "ok" if code == 0 else errno.errorcode.get(code, code)}


def landlock():
    libc.syscall.restype = ctypes.c_long
    v = libc.syscall(SYS_landlock_create_ruleset, None, ctypes.c_size_t(0), ctypes.c_uint32(1))
    return {"abi": int(v), "errno": None if v >= 0 else _err()}


def cgroup():
    cg = _read("/proc/self/cgroup")
    path = cg.split("::", 1)[-1] if "::" in cg else None
    res = {"self": cg, "controllers": _read("/sys/fs/cgroup/cgroup.controllers")}
    if path:
        d = "/sys/fs/cgroup" + path
        res["dir"] = d
        res["writable"] = os.access(d, os.W_OK)
        res["subtree_control"] = _read(d + "/cgroup.subtree_control")
        try:
            t = os.path.join(d, "amdkube-probe")
            os.mkdir(t)
            res["mkdir_child"] = "ok"
            os.rmdir(t)
        except OSError as e:
            res["mkdir_child"] = e.strerror
    return res


def gpu_in_userns(binary):
    def run():
        err = _enter_userns()
        if err:
            return {"error": err}
        nodes = sorted(glob.glob("/dev/dri/renderD*"))
        keep = nodes[:1]
        fds = [os.open(k, os.O_PATH) for k in keep]
        libc.mount(b"tmpfs", b"/dev/dri", b"tmpfs", 0, b"mode=755,size=64k")
        for k, fd in zip(keep, fds):
            t = "/dev/dri/" + os.path.basename(k)
            open(t, "w").close()
            libc.mount(f"/proc/self/fd/{fd}".encode(), t.encode(), None, MS_BIND, None)
        env = {k: v for k, v in os.environ.items() if not k.endswith("_VISIBLE_DEVICES")}
        p = subprocess.run([binary], env=env, capture_output=True, text=True, timeout=60)
        return {"rc": p.returncode, "out": p.stdout[-600:], "err": p.stderr[-600:]}
    return _child(run)


def main():
    out = {"uname": platform.release(), "status": _status(), "lsm": _read("/sys/kernel/security/lsm"),
           "sysctl": {k: _read("/proc/sys/" + k) for k in (
               "kernel/unprivileged_userns_clone", "user/max_user_namespaces",
               "kernel/apparmor_restrict_unprivileged_userns", "kernel/yama/ptrace_scope",
               "kernel/unprivileged_bpf_disabled")},
           "dev": {p: (lambda s: f"{oct(s.st_mode)} {s.st_uid}:{s.st_gid} {os.major(s.st_rdev)}:{os.minor(s.st_rdev)}")(os.stat(p))
                   for p in ["/dev/kfd"] + sorted(glob.glob("/dev/dri/*")) if os.path.exists(p)},
           "in_container": os.path.exists("/.dockerenv") or "kubepods" in _read("/proc/1/cgroup"),
           "proc_mounts_masked": [l.split()[1] for l in _read("/proc/self/mounts").splitlines() if l.split()[1].startswith("/proc/")],
           }
    out["userns_dev"] = _child(userns_dev)
    out["pidns_proc"] = _child(pidns_proc)
    out["landlock"] = landlock()
    out["cgroup"] = cgroup()
    vadd = os.path.join(os.path.dirname(__file__), "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")
    if len(sys.argv) > 1 and sys.argv[1] == "--gpu" and os.path.exists(vadd):
        out["gpu_in_userns"] = gpu_in_userns(os.path.abspath(vadd))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
