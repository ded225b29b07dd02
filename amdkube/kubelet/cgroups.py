"""The kubelet's cgroup manager: internal cgroup names and the cgroupfs / systemd drivers.

Reference: pkg/kubelet/cm/cgroup_manager_linux.go —
* internal names are slash paths (`/kubepods/burstable/pod<uid>`);
* ConvertCgroupNameToSystemd (:60-105): every component becomes one `-`-joined slice name
  (dashes inside a component turn into `_`, a component already in slice form contributes its
  last segment), `/` is `-.slice`; with outputToCgroupFs the slice is expanded the way
  libcontainer's systemd.ExpandSlice does (`a-b-c.slice` ->
  `a.slice/a-b.slice/a-b-c.slice/`);
* ConvertCgroupFsNameToSystemd (:111) is the basename; RevertFromSystemdToCgroupStyleName
  (:166-175) undoes the conversion;
* NewCgroupManager (:214) picks the driver; the systemd one needs systemd to be the init system
  (libcontainer's UseSystemd: /run/systemd/system exists), else the reference panics — here it
  is a clear error at kubelet start.
The systemd driver creates each cgroup as a transient slice unit over D-Bus
(StartTransientUnit with MemoryMax / CPUWeight / CPUQuotaPerSecUSec, as libcontainer's
systemd manager sets MemoryLimit / CPUShares / CPUQuotaPerSecUSec), updates it with
SetUnitProperties and removes it with StopUnit; the cgroup v2 files are also written
directly, so a limit holds even on a systemd that does not know a property.
Runtime side: rocshim (--cgroup-driver) places each container in a transient scope inside its
pod's slice (runtime/rocshim.py).
"""
from __future__ import annotations

import logging
import os
import time

log = logging.getLogger("amdkube.kubelet.cgroups")

SYSTEMD_SUFFIX = ".slice"
CGROUPFS, SYSTEMD = "cgroupfs", "systemd"
SYSTEMD_DEST = "org.freedesktop.systemd1"
SYSTEMD_PATH = "/org/freedesktop/systemd1"
SYSTEMD_MANAGER = "org.freedesktop.systemd1.Manager"
SYSTEMD_PRIVATE_SOCKET = "/run/systemd/private"
SYSTEM_BUS_SOCKET = "/run/dbus/system_bus_socket"


class CgroupError(RuntimeError):
    pass


def is_systemd_style_name(name: str) -> bool:
    return name.endswith(SYSTEMD_SUFFIX)


def expand_slice(slice_name: str) -> str:
    """libcontainer systemd.ExpandSlice: `test-a-b.slice` -> `test.slice/test-a.slice/test-a-b.slice/`."""
    if len(slice_name) < len(SYSTEMD_SUFFIX) or not slice_name.endswith(SYSTEMD_SUFFIX) or "/" in slice_name:
        raise CgroupError(f"invalid slice name: {slice_name}")
    base = slice_name[:-len(SYSTEMD_SUFFIX)]
    if base == "-":
        return "/"
    path, prefix = "", ""
    for comp in base.split("-"):
        if not comp:
            raise CgroupError(f"invalid slice name: {slice_name}")
        path += prefix + comp + SYSTEMD_SUFFIX + "/"
        prefix += comp + "-"
    return path


def to_systemd(name: str, output_to_cgroupfs: bool = False) -> str:
    """ConvertCgroupNameToSystemd."""
    if name and name != "/":
        parts = []
        for part in name.split("/"):
            if not part:
                continue
            if is_systemd_style_name(part):
                part = part[:-len(SYSTEMD_SUFFIX)]
                part = part[part.rfind("-") + 1:]
            else:
                part = part.replace("-", "_")
            parts.append(part)
        result = "-".join(parts)
    else:
        result = "-"
    if not is_systemd_style_name(result):
        result += SYSTEMD_SUFFIX
    return expand_slice(result) if output_to_cgroupfs else result


def cgroupfs_to_systemd(path: str) -> str:
    """ConvertCgroupFsNameToSystemd: the expanded path's last component."""
    return os.path.basename(path.rstrip("/")) if path.rstrip("/") else path


def revert_from_systemd(name: str) -> str:
    """RevertFromSystemdToCgroupStyleName."""
    n = cgroupfs_to_systemd(name)
    if n.endswith(SYSTEMD_SUFFIX):
        n = n[:-len(SYSTEMD_SUFFIX)]
    return n.replace("-", "/").replace("_", "-")


RUNTIME_DEFAULT_ROOT = "/sys/fs/cgroup/amdkube"      # rocshim's cgroupfs-driver tree


def cgroup2_mount_of(path: str, mountinfo: str = "/proc/self/mountinfo") -> str | None:
    """The cgroup2 mount point `path` lies in (the deepest one), or None."""
    path = os.path.abspath(path)
    best = None
    try:
        with open(mountinfo) as f:
            lines = f.read().splitlines()
    except OSError:
        return None
    for line in lines:
        left, _, right = line.partition(" - ")
        fields = left.split()
        if len(fields) < 5 or not right.startswith("cgroup2 "):
            continue
        mp = fields[4].replace("\\040", " ")
        if (path == mp or path.startswith(mp.rstrip("/") + "/")) and (best is None or len(mp) > len(best)):
            best = mp
    return best


def systemd_cgroup_root(root: str, mountinfo: str = "/proc/self/mountinfo") -> str:
    """The cgroup root the systemd driver works under. systemd lays slices out from the cgroup2
    mount, so a root inside that mount is only meaningful as the mount itself: the runtime's
    cgroupfs default is remapped to it (as rocshim does), any other sub-directory is refused at
    start instead of every pods-cgroup create waiting out a directory systemd never makes. A
    root outside every cgroup2 mount (a test tree fed by a stand-in systemd) is kept."""
    mount = cgroup2_mount_of(root, mountinfo)
    if mount is None or os.path.abspath(root) == mount:
        return root
    if os.path.abspath(root) == RUNTIME_DEFAULT_ROOT:
        return mount
    raise CgroupError(f"--cgroup-driver=systemd: --cgroup-root {root} is not the cgroup2 mount {mount}; "
                      f"systemd creates slices from the mount, so the root must be {mount}")


def use_systemd(run_dir: str = "/run/systemd/system") -> bool:
    """libcontainer UseSystemd / sd_booted: systemd is the init system."""
    return os.path.isdir(run_dir)


def systemd_connection(timeout: float = 10.0):
    """go-systemd's dbus.New: root talks to systemd's private socket directly, others go
    through the system bus (AMDKUBE_SYSTEMD_BUS overrides the socket path)."""
    from ..utils.dbus import Connection
    override = os.environ.get("AMDKUBE_SYSTEMD_BUS")
    if override:
        return Connection(override, bus=os.environ.get("AMDKUBE_SYSTEMD_BUS_KIND", "bus") == "bus", timeout=timeout).connect()
    if os.geteuid() == 0 and os.path.exists(SYSTEMD_PRIVATE_SOCKET):
        return Connection(SYSTEMD_PRIVATE_SOCKET, bus=False, timeout=timeout).connect()
    return Connection(SYSTEM_BUS_SOCKET, bus=True, timeout=timeout).connect()


def unit_properties(resources: dict) -> list:
    """Resource limits as systemd unit properties (cgroup v2 names)."""
    props = []
    if resources.get("memory"):
        props.append(("MemoryMax", ("t", int(resources["memory"]))))
    if resources.get("cpu_weight"):
        props.append(("CPUWeight", ("t", int(resources["cpu_weight"]))))
    if resources.get("cpu_quota") and resources.get("cpu_period"):
        # systemd takes the quota per second of wall time
        props.append(("CPUQuotaPerSecUSec", ("t", int(resources["cpu_quota"]) * 1_000_000 // int(resources["cpu_period"]))))
    return props


class SystemdUnits:
    """The systemd manager calls the cgroup drivers need."""

    def __init__(self, connect=systemd_connection):
        import threading
        self._connect = connect
        self._conn = None
        # rocshim and the kubelet call from worker threads (asyncio.to_thread): one call at a
        # time on the shared connection, and one reconnect
        self._lock = threading.RLock()

    def _call(self, member: str, sig: str, *args):
        from ..utils.dbus import DBusError
        with self._lock:
            for attempt in (0, 1):
                if self._conn is None:
                    self._conn = self._connect()
                try:
                    return self._conn.call(SYSTEMD_DEST, SYSTEMD_PATH, SYSTEMD_MANAGER, member, sig, *args)
                except (OSError, DBusError) as e:
                    if isinstance(e, DBusError) and e.name != "org.freedesktop.DBus.Error.Disconnected":
                        raise
                    self.close()                   # a restarted systemd: reconnect once
                    if attempt:
                        raise

    def close(self):
        with self._lock:
            if self._conn is not None:
                self._conn.close()
                self._conn = None

    def start_transient(self, unit: str, properties: list) -> str:
        """StartTransientUnit(name, "replace", properties, aux=[]) -> the job's object path."""
        (job,) = self._call("StartTransientUnit", "ssa(sv)a(sa(sv))", unit, "replace", properties, [])
        return job

    def set_properties(self, unit: str, properties: list):
        self._call("SetUnitProperties", "sba(sv)", unit, True, properties)

    def stop(self, unit: str) -> str:
        (job,) = self._call("StopUnit", "ss", unit, "replace")
        return job


def _write_limits(path: str, resources: dict):
    for fname, val in (("memory.max", resources.get("memory")), ("cpu.weight", resources.get("cpu_weight")),
                       ("cpu.max", f"{resources['cpu_quota']} {resources['cpu_period']}"
                        if resources.get("cpu_quota") and resources.get("cpu_period") else None)):
        if val:
            with open(os.path.join(path, fname), "w") as f:
                f.write(str(val))


class CgroupManager:
    """Create / update / destroy cgroups by internal name under `root` (the cgroup v2 mount)."""

    def __init__(self, driver: str = CGROUPFS, root: str = "/sys/fs/cgroup", units: SystemdUnits | None = None,
                 wait_s: float = 5.0):
        if driver not in (CGROUPFS, SYSTEMD):
            raise CgroupError(f"invalid cgroup driver {driver!r} (cgroupfs or systemd)")
        self.driver, self.root, self.wait_s = driver, root, wait_s
        self.units = units if units is not None or driver == CGROUPFS else SystemdUnits()

    def name(self, internal: str) -> str:
        """cgroupManagerImpl.Name: the driver's literal name, in cgroupfs form."""
        return to_systemd(internal, True) if self.driver == SYSTEMD else internal

    def cgroup_name(self, literal: str) -> str:
        """cgroupManagerImpl.CgroupName: a literal cgroupfs name back to the internal one."""
        return revert_from_systemd(literal) if self.driver == SYSTEMD else literal

    def path(self, internal: str) -> str:
        return os.path.join(self.root, self.name(internal).strip("/"))

    def exists(self, internal: str) -> bool:
        return os.path.isdir(self.path(internal))

    def _await_dir(self, path: str):
        deadline = time.monotonic() + self.wait_s
        while not os.path.isdir(path):
            if time.monotonic() > deadline:
                raise CgroupError(f"systemd did not create {path} within {self.wait_s:.0f}s")
            time.sleep(0.01)

    def create(self, internal: str, resources: dict | None = None):
        resources = resources or {}
        path = self.path(internal)
        if self.driver == SYSTEMD:
            unit = to_systemd(internal)
            props = [("Description", ("s", f"amdkube cgroup {internal}")), ("MemoryAccounting", ("b", True)),
                     ("CPUAccounting", ("b", True))] + unit_properties(resources)
            try:
                self.units.start_transient(unit, props)
            except Exception as e:
                if "already exists" not in str(e) and "UnitExists" not in str(e):
                    raise CgroupError(f"systemd: creating {unit}: {e}") from e
                self.units.set_properties(unit, unit_properties(resources))
            self._await_dir(path)
        else:
            os.makedirs(path, exist_ok=True)
        _write_limits(path, resources)

    def update(self, internal: str, resources: dict):
        if self.driver == SYSTEMD and unit_properties(resources):
            self.units.set_properties(to_systemd(internal), unit_properties(resources))
        _write_limits(self.path(internal), resources)

    def destroy(self, internal: str):
        if self.driver == SYSTEMD:
            try:
                self.units.stop(to_systemd(internal))
            except Exception as e:
                log.debug("systemd: stopping %s: %r", to_systemd(internal), e)
        try:
            os.rmdir(self.path(internal))
        except OSError:
            pass

    def pids(self, internal: str) -> list[int]:
        out = []
        for dirpath, _dirs, files in os.walk(self.path(internal)):
            if "cgroup.procs" in files:
                try:
                    with open(os.path.join(dirpath, "cgroup.procs")) as f:
                        out += [int(x) for x in f.read().split()]
                except (OSError, ValueError):
                    pass
        return out


def scope_name(runtime_prefix: str, container_id: str) -> str:
    """The transient scope a runtime puts a container in (docker-<id>.scope, crio-<id>.scope)."""
    return f"{runtime_prefix}-{container_id}.scope"
