"""Mount interface (pkg/util/mount): the volume plugins' only way to touch the host mount table.

`SysMounter` drives mount(8)/umount(8) and reads /proc/self/mountinfo; `FakeMounter`
(pkg/util/mount/fake.go) keeps an in-memory table and a log of actions so plugins, the volume
manager and their tests run without privileges. `is_likely_not_mount_point` is the reference's
fast check (device of the path differs from its parent's); `get_mount_refs` lists the other
mount points of the same source (the device-global mount's per-pod bind mounts).
"""
from __future__ import annotations

import os
import subprocess
from dataclasses import dataclass, field


@dataclass
class MountPoint:
    device: str
    path: str
    type: str
    opts: list[str] = field(default_factory=list)
    root: str = "/"          # mountinfo field 4: the part of the source filesystem mounted here


def parse_mountinfo(text: str) -> list[MountPoint]:
    """/proc/self/mountinfo: `id parent major:minor root mountpoint opts ... - fstype source superopts`."""
    out = []
    for line in text.splitlines():
        pre, sep, post = line.partition(" - ")
        if not sep:
            continue
        f = pre.split()
        g = post.split()
        if len(f) < 6 or len(g) < 2:
            continue
        unesc = lambda s: s.replace("\\040", " ").replace("\\011", "\t").replace("\\012", "\n").replace("\\134", "\\")  # noqa: E731
        out.append(MountPoint(device=unesc(g[1]), path=unesc(f[4]), type=g[0], opts=f[5].split(","), root=unesc(f[3])))
    return out


class MountError(RuntimeError):
    pass


def unmount_under(base: str, mountinfo: str = "/proc/self/mountinfo") -> int:
    """Unmount every mount point below `base`, deepest first (test-harness hygiene: a kubelet
    stopped with volumes set up leaves their mounts behind, like the reference's)."""
    try:
        with open(mountinfo) as f:
            table = parse_mountinfo(f.read())
    except OSError:
        return 0
    root = os.path.realpath(base).rstrip("/") + "/"
    n = 0
    for mp in sorted((mp for mp in table if mp.path.startswith(root)), key=lambda mp: -len(mp.path)):
        if subprocess.run(["umount", "-l", mp.path], capture_output=True).returncode == 0:
            n += 1
    return n


class SysMounter:
    def __init__(self, mountinfo: str = "/proc/self/mountinfo"):
        self.mountinfo = mountinfo

    def list(self) -> list[MountPoint]:
        with open(self.mountinfo) as f:
            return parse_mountinfo(f.read())

    def mount(self, source: str, target: str, fstype: str = "", options: list[str] | None = None):
        cmd = ["mount"]
        if fstype:
            cmd += ["-t", fstype]
        opts = list(options or [])
        bind = "bind" in opts
        if opts:
            # mount(8) ignores most options on a bind: the reference binds first, then remounts
            cmd += ["-o", "bind" if bind else ",".join(opts)]
        cmd += [source, target]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            raise MountError(f"mount failed: {' '.join(cmd)}: {r.stderr.strip() or r.stdout.strip()}")
        extra = [o for o in opts if o != "bind"]
        if bind and extra:
            cmd2 = ["mount", "-o", ",".join(["bind", "remount", *extra]), source, target]
            r = subprocess.run(cmd2, capture_output=True, text=True, timeout=60)
            if r.returncode != 0:
                raise MountError(f"mount failed: {' '.join(cmd2)}: {r.stderr.strip()}")

    def unmount(self, target: str):
        r = subprocess.run(["umount", target], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            raise MountError(f"unmount failed: {target}: {r.stderr.strip()}")

    def is_likely_not_mount_point(self, path: str) -> bool:
        st = os.stat(path)                      # raises FileNotFoundError like the reference
        parent = os.stat(os.path.dirname(os.path.abspath(path.rstrip("/"))) or "/")
        return st.st_dev == parent.st_dev

    def is_mount_point(self, path: str) -> bool:
        p = os.path.realpath(path)
        return any(mp.path == p for mp in self.list())

    def get_mount_refs(self, path: str) -> list[str]:
        return mount_refs(self.list(), path)


def mount_refs(table: list[MountPoint], path: str) -> list[str]:
    p = os.path.realpath(path)
    src = next((mp for mp in table if mp.path == p), None)
    if src is None:
        return []
    return [mp.path for mp in table if mp.path != p and mp.device == src.device and mp.root == src.root]


class FakeMounter:
    """In-memory mount table (pkg/util/mount/fake.go): every mount/unmount is logged as
    (action, target, source, fstype, options)."""

    def __init__(self, mounts: list[MountPoint] | None = None):
        self.mounts: list[MountPoint] = list(mounts or [])
        self.log: list[tuple] = []
        self.fail: dict[str, str] = {}        # target or source -> error message (fault injection)

    def list(self) -> list[MountPoint]:
        return list(self.mounts)

    def mount(self, source: str, target: str, fstype: str = "", options: list[str] | None = None):
        for k in (target, source):
            if k in self.fail:
                raise MountError(self.fail[k])
        opts = list(options or [])
        dev, root = source, "/"
        if "bind" in opts:     # a bind mount shares the source mount's device
            src = next((mp for mp in self.mounts if mp.path == os.path.realpath(source)), None)
            if src is not None:
                dev, root = src.device, src.root
        self.mounts.append(MountPoint(dev, os.path.realpath(target), fstype or "none", opts, root))
        self.log.append(("mount", target, source, fstype, opts))

    def unmount(self, target: str):
        p = os.path.realpath(target)
        for i in range(len(self.mounts) - 1, -1, -1):
            if self.mounts[i].path == p:
                del self.mounts[i]
                self.log.append(("unmount", target, "", "", []))
                return
        self.log.append(("unmount", target, "", "", []))

    def is_likely_not_mount_point(self, path: str) -> bool:
        os.stat(path)
        return not self.is_mount_point(path)

    def is_mount_point(self, path: str) -> bool:
        p = os.path.realpath(path)
        return any(mp.path == p for mp in self.mounts)

    def get_mount_refs(self, path: str) -> list[str]:
        return mount_refs(self.mounts, path)

    def actions(self, kind: str | None = None) -> list[tuple]:
        return [a for a in self.log if kind is None or a[0] == kind]


class NoopMounter:
    """An unprivileged kubelet cannot mount: nothing is ever a mount point, mounting fails.
    Volume types that only need a directory (emptyDir on disk, hostPath, local, rendered
    secret/configMap content) still work; tmpfs-backed media degrade to plain directories."""
    privileged = False

    def list(self) -> list[MountPoint]:
        return []

    def mount(self, source, target, fstype="", options=None):
        raise MountError(f"mount of {source} at {target} needs a privileged kubelet (running as uid {os.geteuid()})")

    def unmount(self, target):
        pass

    def is_likely_not_mount_point(self, path):
        os.stat(path)
        return True

    def is_mount_point(self, path):
        return False

    def get_mount_refs(self, path):
        return []


class FakeExec:
    """Records commands the plugins run (iscsiadm, rbd, mkfs, ...); `responses` maps a command
    prefix (tuple of argv words) to (returncode, output)."""

    def __init__(self, responses: dict[tuple, tuple[int, str]] | None = None):
        self.responses = dict(responses or {})
        self.calls: list[list[str]] = []

    def run(self, argv: list[str], timeout: float = 60.0) -> tuple[int, str]:
        self.calls.append(list(argv))
        best = None
        for k, v in self.responses.items():
            if tuple(argv[:len(k)]) == k and (best is None or len(k) > len(best[0])):
                best = (k, v)
        return best[1] if best else (0, "")


class SysExec:
    def run(self, argv: list[str], timeout: float = 60.0) -> tuple[int, str]:
        try:
            r = subprocess.run(argv, capture_output=True, text=True, timeout=timeout)
        except FileNotFoundError as e:
            return 127, str(e)
        except subprocess.TimeoutExpired:
            return 124, f"{argv[0]}: timed out after {timeout}s"
        return r.returncode, (r.stdout + r.stderr)
