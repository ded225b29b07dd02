"""Node-local volume plugins: emptyDir, hostPath, local, secret, configMap, downwardAPI,
projected, gitRepo (pkg/volume/empty_dir, host_path, local, secret, configmap, downwardapi,
projected, git_repo).

* emptyDir: a directory under the pod (mode 0777); medium "Memory" mounts a tmpfs (sizeLimit
  becomes the tmpfs size), medium "HugePages" a hugetlbfs with the page size of the pod's
  hugepages-<size> request. Teardown unmounts the medium and deletes the contents.
* hostPath: the host path itself, after the `type` checks (DirectoryOrCreate, Directory,
  FileOrCreate, File, Socket, CharDevice, BlockDevice).
* local (PersistentVolume only): the PV's path, which must exist on this node.
* secret / configMap / downwardAPI / projected: content rendered by the kubelet (atomic writes,
  items and modes) into a tmpfs-backed directory (the reference wraps them in a Memory emptyDir
  so secrets never reach the disk); re-rendered on every reconcile (RequiresRemount).
* gitRepo: clone + checkout into an emptyDir.
"""
from __future__ import annotations

import asyncio
import os
import shutil
import stat

from ..api.quantity import Quantity
from . import VolumeError, VolumePlugin, unmount_and_remove
from .mount import MountError, NoopMounter


async def _tmpfs(host, dir: str, size: str | None = None, what: str = ""):
    """Mount a tmpfs at `dir` (once). An unprivileged kubelet keeps a plain directory."""
    os.makedirs(dir, mode=0o777, exist_ok=True)
    if isinstance(host.mounter, NoopMounter) or host.mounter.is_mount_point(dir):
        return
    opts = [f"size={size}"] if size else []
    try:
        await asyncio.to_thread(host.mounter.mount, "tmpfs", dir, "tmpfs", opts)
    except MountError as e:
        raise VolumeError(f"{what}: {e}")


class EmptyDirPlugin(VolumePlugin):
    name = "kubernetes.io/empty-dir"
    source_key = "emptyDir"
    supports_pv = False

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("emptyDir")
        medium = src.get("medium") or ""
        if medium == "Memory":
            size = None
            if src.get("sizeLimit"):
                size = str(Quantity(src["sizeLimit"]).value())
            await _tmpfs(self.host, dir, size, f"emptyDir {spec.name()}")
        elif medium == "HugePages":
            os.makedirs(dir, mode=0o777, exist_ok=True)
            if not isinstance(self.host.mounter, NoopMounter) and not self.host.mounter.is_mount_point(dir):
                page = hugepage_size(pod)
                try:
                    await asyncio.to_thread(self.host.mounter.mount, "nodev", dir, "hugetlbfs", [f"pagesize={page}"])
                except MountError as e:
                    raise VolumeError(f"emptyDir {spec.name()}: {e}")
        elif medium:
            raise VolumeError(f"emptyDir {spec.name()}: unknown storage medium {medium!r}")
        else:
            if not os.path.isdir(dir):
                os.makedirs(dir, exist_ok=True)
                os.chmod(dir, 0o777)
        return dir

    async def tear_down(self, dir):
        # rename-then-delete (empty_dir.go teardownDefault): the path is free immediately
        m = self.host.mounter
        if m.is_mount_point(dir):
            await unmount_and_remove(m, dir)
            return
        if os.path.isdir(dir):
            doomed = f"{dir}.deleting~{os.getpid()}"
            os.rename(dir, doomed)
            await asyncio.to_thread(shutil.rmtree, doomed, True)


def hugepage_size(pod: dict) -> str:
    """The single hugepages-<size> resource the pod asks for (reference: all containers must
    agree)."""
    sizes = set()
    for c in (pod.get("spec") or {}).get("containers") or []:
        res = c.get("resources") or {}
        for k in list((res.get("limits") or {})) + list((res.get("requests") or {})):
            if k.startswith("hugepages-"):
                sizes.add(k[len("hugepages-"):])
    if len(sizes) != 1:
        raise VolumeError("hugePages medium needs exactly one hugepages-<size> resource in the pod" if not sizes
                          else f"pod requests several huge page sizes: {sorted(sizes)}")
    return sizes.pop()


_CHECKS = {"Directory": stat.S_ISDIR, "File": stat.S_ISREG, "Socket": stat.S_ISSOCK,
           "CharDevice": stat.S_ISCHR, "BlockDevice": stat.S_ISBLK}


class HostPathPlugin(VolumePlugin):
    name = "kubernetes.io/host-path"
    source_key = "hostPath"
    access_modes = ("ReadWriteOnce",)

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        hp = spec.source("hostPath")
        p, typ = hp.get("path", ""), hp.get("type") or ""
        if typ == "DirectoryOrCreate":
            os.makedirs(p, mode=0o755, exist_ok=True)
        elif typ == "FileOrCreate":
            os.makedirs(os.path.dirname(p) or "/", exist_ok=True)
            if not os.path.exists(p):
                open(p, "a").close()
        elif typ:
            check = _CHECKS.get(typ)
            try:
                ok = check is not None and check(os.stat(p).st_mode)
            except OSError:
                ok = False
            if not ok:
                raise VolumeError(f"hostPath type check failed: {p} is not a {typ}")
        if spec.pv is not None and not os.path.exists(p):
            os.makedirs(p, exist_ok=True)    # host-path provisioner volumes
        return p

    async def tear_down(self, dir):
        pass        # nothing of the host path belongs to the pod


class LocalPlugin(VolumePlugin):
    name = "kubernetes.io/local-volume"
    source_key = "local"
    supports_inline = False
    access_modes = ("ReadWriteOnce",)

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        p = spec.source("local").get("path", "")
        if not os.path.exists(p):
            raise VolumeError(f"local volume {spec.name()}: path {p} does not exist on this node")
        return p

    async def tear_down(self, dir):
        pass


class _Rendered(VolumePlugin):
    """Kubelet-rendered content in a memory-backed directory, re-rendered every reconcile."""
    requires_remount = True
    supports_pv = False

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        ctx = self.host.pod_context
        if ctx is None:
            raise VolumeError(f"{self.name}: no pod context to render volume {spec.name()}")
        await _tmpfs(self.host, dir, None, f"volume {spec.name()}")
        await self.render(ctx, spec, pod, dir, f"volume {spec.name()}")
        return dir

    async def render(self, ctx, spec, pod, dir, what):
        raise NotImplementedError


class SecretPlugin(_Rendered):
    name = "kubernetes.io/secret"
    source_key = "secret"

    async def render(self, ctx, spec, pod, dir, what):
        await ctx._projection(pod, dir, "secrets", spec.source("secret"), 0o644, what)


class ConfigMapPlugin(_Rendered):
    name = "kubernetes.io/configmap"
    source_key = "configMap"

    async def render(self, ctx, spec, pod, dir, what):
        await ctx._projection(pod, dir, "configmaps", spec.source("configMap"), 0o644, what)


class DownwardAPIPlugin(_Rendered):
    name = "kubernetes.io/downward-api"
    source_key = "downwardAPI"

    async def render(self, ctx, spec, pod, dir, what):
        src = spec.source("downwardAPI")
        await ctx._downward(pod, dir, src.get("items"), src.get("defaultMode", 0o644))


class ProjectedPlugin(_Rendered):
    name = "kubernetes.io/projected"
    source_key = "projected"

    async def render(self, ctx, spec, pod, dir, what):
        src = spec.source("projected")
        dm = src.get("defaultMode", 0o644)
        for s in src.get("sources") or []:
            if "secret" in s:
                await ctx._projection(pod, dir, "secrets", s["secret"], dm, what)
            elif "configMap" in s:
                await ctx._projection(pod, dir, "configmaps", s["configMap"], dm, what)
            elif "downwardAPI" in s:
                await ctx._downward(pod, dir, s["downwardAPI"].get("items"), dm)


class GitRepoPlugin(VolumePlugin):
    name = "kubernetes.io/git-repo"
    source_key = "gitRepo"
    supports_pv = False

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        ctx = self.host.pod_context
        if ctx is None:
            raise VolumeError("gitRepo needs the kubelet pod context")
        return await ctx._git_repo(dir, spec.source("gitRepo"), f"volume {spec.name()}")

    async def tear_down(self, dir):
        if os.path.isdir(dir):
            await asyncio.to_thread(shutil.rmtree, dir, True)


def plugins() -> list[VolumePlugin]:
    return [EmptyDirPlugin(), HostPathPlugin(), LocalPlugin(), SecretPlugin(), ConfigMapPlugin(), DownwardAPIPlugin(),
            ProjectedPlugin(), GitRepoPlugin()]
