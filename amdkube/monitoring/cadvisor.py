"""The cAdvisor part of the kubelet, MI355X-node edition (vendor/github.com/google/cadvisor:
container/libcontainer/helpers.go cgroup readers, fs/fs.go, utils/sysinfo; pkg/volume/
metrics_du.go, metrics_statfs.go; pkg/kubelet/stats summary providers).

  * cgroup v2 container stats: cpu.stat usage, memory.current, working set (current −
    inactive_file), anon (rss), page faults (pgfault / pgmajfault), io.stat bytes, pids.current;
  * the process-group fallback for containers without a cgroup leaf (unprivileged rocshim):
    /proc/<pid>/stat CPU ticks, statm RSS, minor/major faults, /proc/<pid>/io bytes;
  * filesystem capacity (statvfs) and directory usage (du: bytes and inodes, cached for
    `ttl` seconds because walking volumes is costly — cAdvisor's housekeeping interval);
  * network counters from a /proc/<pid>/net/dev (the node's, or a pod sandbox's own netns);
  * rlimit (pid_max, running processes) and machine info.
"""
from __future__ import annotations

import os
import threading
import time

CLK_TCK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
PAGE = os.sysconf("SC_PAGE_SIZE") if hasattr(os, "sysconf") else 4096
_VIRTUAL_IF = ("lo", "veth", "cbr", "akb", "docker", "virbr", "tmp", "kube-ipvs")


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def _kv(text: str) -> dict[str, int]:
    out = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2 and parts[1].lstrip("-").isdigit():
            out[parts[0]] = int(parts[1])
    return out


def cgroup_stats(cg: str) -> dict | None:
    """Stats of one cgroup-v2 directory, or None when it does not exist."""
    if not cg or not os.path.isdir(cg):
        return None
    cpu = _kv(_read(os.path.join(cg, "cpu.stat")))
    mem_cur = _read(os.path.join(cg, "memory.current")).strip()
    mstat = _kv(_read(os.path.join(cg, "memory.stat")))
    usage = int(mem_cur) if mem_cur.isdigit() else 0
    io_r = io_w = 0
    for line in _read(os.path.join(cg, "io.stat")).splitlines():
        for tok in line.split()[1:]:
            k, _, v = tok.partition("=")
            if k == "rbytes" and v.isdigit():
                io_r += int(v)
            elif k == "wbytes" and v.isdigit():
                io_w += int(v)
    pids = _read(os.path.join(cg, "pids.current")).strip()
    return {"cpu_ns": cpu.get("usage_usec", 0) * 1000, "usage_bytes": usage,
            "working_set_bytes": max(0, usage - mstat.get("inactive_file", 0)), "rss_bytes": mstat.get("anon", 0),
            "page_faults": mstat.get("pgfault", 0), "major_page_faults": mstat.get("pgmajfault", 0),
            "io_read_bytes": io_r, "io_write_bytes": io_w, "pids": int(pids) if pids.isdigit() else 0}


def process_stats(pids: list[int]) -> dict:
    """The same numbers summed over a process group (no cgroup of its own)."""
    cpu = rss = minflt = majflt = rb = wb = 0
    n = 0
    for pid in pids:
        st = _read(f"/proc/{pid}/stat")
        if not st:
            continue
        fields = st[st.rfind(")") + 2:].split()
        try:
            minflt += int(fields[7])
            majflt += int(fields[9])
            cpu += (int(fields[11]) + int(fields[12])) * (10 ** 9 // CLK_TCK)
            rss += int(fields[21]) * PAGE
        except (IndexError, ValueError):
            continue
        io = _kv(_read(f"/proc/{pid}/io").replace(":", ""))
        rb += io.get("read_bytes", 0)
        wb += io.get("write_bytes", 0)
        n += 1
    return {"cpu_ns": cpu, "usage_bytes": rss, "working_set_bytes": rss, "rss_bytes": rss, "page_faults": minflt,
            "major_page_faults": majflt, "io_read_bytes": rb, "io_write_bytes": wb, "pids": n}


def fs_stats(path: str) -> dict:
    """statvfs → the summary API's FsStats."""
    try:
        st = os.statvfs(path)
    except OSError:
        return {}
    cap, avail = st.f_blocks * st.f_frsize, st.f_bavail * st.f_frsize
    return {"capacityBytes": cap, "availableBytes": avail, "usedBytes": cap - st.f_bfree * st.f_frsize,
            "inodes": st.f_files, "inodesFree": st.f_ffree, "inodesUsed": st.f_files - st.f_ffree}


def du(path: str) -> tuple[int, int]:
    """Bytes (allocated blocks, like du) and inodes under `path`, not crossing mounts."""
    total = inodes = 0
    try:
        root_dev = os.lstat(path).st_dev
    except OSError:
        return 0, 0
    stack = [path]
    while stack:
        d = stack.pop()
        try:
            it = os.scandir(d)
        except OSError:
            continue
        with it:
            for e in it:
                try:
                    st = e.stat(follow_symlinks=False)
                except OSError:
                    continue
                inodes += 1
                total += st.st_blocks * 512
                if e.is_dir(follow_symlinks=False) and st.st_dev == root_dev:
                    stack.append(e.path)
    return total, inodes + 1


class DuCache:
    """metrics_cached.go: a directory's usage is re-measured at most every `ttl` seconds."""

    def __init__(self, ttl: float = 10.0):
        self.ttl = ttl
        self._c: dict[str, tuple[float, int, int]] = {}
        self._lock = threading.Lock()

    def get(self, path: str) -> tuple[int, int]:
        now = time.monotonic()
        with self._lock:
            hit = self._c.get(path)
        if hit is not None and now - hit[0] < self.ttl:
            return hit[1], hit[2]
        b, i = du(path)
        with self._lock:
            self._c[path] = (now, b, i)
            if len(self._c) > 4096:
                for k in [k for k, v in self._c.items() if now - v[0] > self.ttl]:
                    del self._c[k]
        return b, i

    def forget(self, prefix: str):
        with self._lock:
            for k in [k for k in self._c if k.startswith(prefix)]:
                del self._c[k]


def net_dev(path: str = "/proc/net/dev") -> dict[str, dict]:
    out = {}
    for line in _read(path).splitlines()[2:]:
        name, _, rest = line.partition(":")
        f = rest.split()
        if len(f) < 16:
            continue
        out[name.strip()] = {"rxBytes": int(f[0]), "rxErrors": int(f[2]), "txBytes": int(f[8]), "txErrors": int(f[10])}
    return out


def network_stats(path: str = "/proc/net/dev", prefer: str | None = None) -> dict:
    """NetworkStats: the default interface (eth0 in a pod, the first physical one on the node)
    at the top level and every interface in `interfaces`."""
    devs = net_dev(path)
    ifaces = [{"name": k, **v} for k, v in sorted(devs.items()) if not k.startswith(_VIRTUAL_IF)]
    if not ifaces:
        return {}
    main = next((i for i in ifaces if i["name"] == prefer), ifaces[0])
    return {**main, "interfaces": ifaces}


def rlimit() -> dict:
    pid_max = _read("/proc/sys/kernel/pid_max").strip()
    try:
        cur = sum(1 for e in os.listdir("/proc") if e.isdigit())
    except OSError:
        cur = 0
    return {"maxpid": int(pid_max) if pid_max.isdigit() else 0, "curproc": cur}


def machine_info() -> dict:
    import psutil
    return {"num_cores": psutil.cpu_count(), "memory_capacity": psutil.virtual_memory().total,
            "machine_id": _read("/etc/machine-id").strip(), "boot_id": _read("/proc/sys/kernel/random/boot_id").strip(),
            "system_uuid": _read("/sys/class/dmi/id/product_uuid").strip(), "kernel_version": os.uname().release}
