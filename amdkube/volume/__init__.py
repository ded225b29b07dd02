"""Volume plugin framework (pkg/volume: plugins.go VolumePluginMgr / VolumePlugin, volume.go
Mounter / Unmounter / Attacher / Detacher, util/operationexecutor naming rules).

A plugin recognises a `Spec` (a pod volume or a PersistentVolume) by its source key and sets
the volume up in the pod's directory `<root>/pods/<uid>/volumes/<escaped plugin name>/<volume>`.
Attachable plugins additionally attach the volume to the node (device path), mount the device
once at a node-global path `<root>/plugins/<plugin>/...`, and bind it into every pod that uses
it; their volumes have node-unique names (`<plugin>/<volume name>`) so two pods share one
attachment. Plugins whose content the kubelet renders (secret, configMap, downwardAPI,
projected) ask to be re-set-up on every reconcile (RequiresRemount).

Plugins are asynchronous: blocking host work (mount(8), iscsiadm, a FlexVolume driver, git)
runs in a thread so one slow volume never stalls the kubelet's event loop.
"""
from __future__ import annotations

import asyncio
import hashlib
import os

from .mount import FakeExec, FakeMounter, MountError, NoopMounter, SysExec, SysMounter   # noqa: F401


def escape_plugin_name(name: str) -> str:
    """kubernetes.io/empty-dir → kubernetes.io~empty-dir (util/strings EscapeQualifiedNameForDisk)."""
    return name.replace("/", "~")


def unescape_plugin_name(name: str) -> str:
    return name.replace("~", "/")


class VolumeError(RuntimeError):
    pass


class Spec:
    """volume.Spec: exactly one of `volume` (pod spec.volumes[i]) or `pv` (a PersistentVolume
    reached through a claim); `read_only` is the claim reference's readOnly."""

    def __init__(self, volume: dict | None = None, pv: dict | None = None, read_only: bool = False):
        self.volume, self.pv, self.read_only = volume, pv, read_only

    def name(self) -> str:
        if self.volume is not None:
            return self.volume["name"]
        return (self.pv.get("metadata") or {}).get("name", "")

    def _src(self) -> dict:
        return self.volume if self.volume is not None else (self.pv.get("spec") or {})

    def has(self, key: str) -> bool:
        return self._src().get(key) is not None

    def source(self, key: str) -> dict:
        return self._src().get(key) or {}

    def source_read_only(self, key: str) -> bool:
        return bool(self.read_only or self.source(key).get("readOnly"))

    def mount_options(self) -> list[str]:
        """PV spec.mountOptions (or the legacy volume.beta.kubernetes.io/mount-options annotation)."""
        if self.pv is None:
            return []
        opts = list((self.pv.get("spec") or {}).get("mountOptions") or [])
        ann = ((self.pv.get("metadata") or {}).get("annotations") or {}).get("volume.beta.kubernetes.io/mount-options")
        if ann:
            opts += [o.strip() for o in ann.split(",") if o.strip()]
        return opts

    def access_modes(self) -> list[str]:
        return list(((self.pv or {}).get("spec") or {}).get("accessModes") or [])


class VolumeHost:
    """What plugins may use from the kubelet (volume.VolumeHost)."""

    def __init__(self, root_dir: str, node_name: str = "", client=None, mounter=None, executor=None,
                 pod_context=None, node_ip: str = "127.0.0.1", plugins_dir: str | None = None):
        self.root_dir = root_dir
        self.node_name = node_name
        self.client = client
        self.mounter = mounter or SysMounter()
        self.exec = executor or SysExec()
        self.pod_context = pod_context     # kubelet PodContext: renders secret/configMap/downward content
        self.node_ip = node_ip
        self.flex_dir = plugins_dir or os.path.join(root_dir, "volumeplugins")
        self.dev_root = "/"          # where /dev/disk/by-path etc. are looked up (tests: a fake tree)
        self.sys_root = "/sys"
        self.attach_poll = 1.0       # seconds between device-appearance checks
        self.cloud = None            # the cloud provider (attachable cloud volumes: cinder)

    def pod_dir(self, uid: str) -> str:
        return os.path.join(self.root_dir, "pods", uid)

    def pod_volume_dir(self, uid: str, plugin: str, name: str) -> str:
        return os.path.join(self.root_dir, "pods", uid, "volumes", escape_plugin_name(plugin), name)

    def plugin_dir(self, plugin: str) -> str:
        return os.path.join(self.root_dir, "plugins", escape_plugin_name(plugin))

    async def run(self, argv: list[str], timeout: float = 60.0) -> tuple[int, str]:
        return await asyncio.to_thread(self.exec.run, argv, timeout)

    async def secret(self, ns: str, name: str) -> dict:
        if self.client is None:
            raise VolumeError(f"no API client to fetch secret {ns}/{name}")
        obj = await self.client.get_or_none("secrets", name, ns)
        if obj is None:
            raise VolumeError(f'secret "{name}" not found')
        import base64
        return {k: base64.b64decode(v).decode(errors="replace") for k, v in (obj.get("data") or {}).items()}


class VolumePlugin:
    """Base plugin. Subclasses set `name`, `source_key` and override set_up/tear_down; attachable
    ones set `attachable = True` and implement the attach/device-mount half."""
    name = ""
    source_key = ""
    attachable = False
    requires_remount = False
    supports_pv = True            # may appear in a PersistentVolume
    supports_inline = True        # may appear directly in a pod's volumes
    access_modes = ("ReadWriteOnce", "ReadOnlyMany", "ReadWriteMany")

    def init(self, host: VolumeHost):
        self.host = host

    def can_support(self, spec: Spec) -> bool:
        if spec.pv is not None and not self.supports_pv or spec.volume is not None and not self.supports_inline:
            return False
        return bool(self.source_key) and spec.has(self.source_key)

    def volume_name(self, spec: Spec) -> str:
        """GetVolumeName: unique per volume (not per pod) for attachable plugins."""
        return spec.name()

    def unique_name(self, spec: Spec, pod_uid: str) -> str:
        if self.attachable:
            return f"{self.name}/{self.volume_name(spec)}"
        return f"{self.name}/{pod_uid}-{spec.name()}"    # GetUniqueVolumeNameForNonAttachableVolume

    # ------------------------------------------------------------ per-pod half
    async def set_up(self, spec: Spec, pod: dict, dir: str, device_mount_path: str | None = None, fs_group=None):
        raise NotImplementedError

    async def tear_down(self, dir: str):
        """Default: unmount if something is mounted there, then remove the directory."""
        await unmount_and_remove(self.host.mounter, dir)

    # ------------------------------------------------------- attachable half
    async def attach(self, spec: Spec, node: str) -> str:
        return ""

    async def wait_for_attach(self, spec: Spec, device_path: str, pod: dict | None, timeout: float) -> str:
        return device_path

    def device_mount_path(self, spec: Spec) -> str:
        return os.path.join(self.host.plugin_dir(self.name), "mounts", self.volume_name(spec).replace("/", "~"))

    async def mount_device(self, spec: Spec, device_path: str, device_mount_path: str):
        pass

    async def unmount_device(self, device_mount_path: str):
        await unmount_and_remove(self.host.mounter, device_mount_path)

    async def detach(self, volume_name: str, node: str):
        pass


async def unmount_and_remove(mounter, dir: str):
    """util.UnmountPath: unmount while something is mounted at `dir`, then remove it."""
    if not os.path.lexists(dir):
        return
    try:
        while mounter.is_mount_point(dir):
            await asyncio.to_thread(mounter.unmount, dir)
    except MountError as e:
        raise VolumeError(str(e))
    try:
        os.rmdir(dir)
    except OSError:
        import shutil
        if mounter.is_mount_point(dir):
            raise VolumeError(f"{dir} is still mounted")
        shutil.rmtree(dir, ignore_errors=True)


async def bind_mount(mounter, source: str, target: str, read_only: bool = False):
    os.makedirs(target, mode=0o750, exist_ok=True)
    if mounter.is_mount_point(target):
        return
    opts = ["bind"] + (["ro"] if read_only else [])
    try:
        await asyncio.to_thread(mounter.mount, source, target, "", opts)
    except MountError as e:
        raise VolumeError(str(e))


async def format_and_mount(host: VolumeHost, device: str, target: str, fstype: str, options: list[str]):
    """mount.SafeFormatAndMount: mount; if the device has no filesystem (blkid says nothing and
    it is not read-only), mkfs it first — never reformat a device that has one."""
    fstype = fstype or "ext4"
    os.makedirs(target, mode=0o750, exist_ok=True)
    try:
        await asyncio.to_thread(host.mounter.mount, device, target, fstype, options)
        return
    except MountError as first:
        rc, out = await host.run(["blkid", "-p", "-s", "TYPE", "-o", "value", device])
        if rc == 2 and "ro" not in options:        # blkid: no recognisable filesystem
            mk = ["mkfs." + fstype] + (["-F", "-m0"] if fstype.startswith("ext") else []) + [device]
            rc2, out2 = await host.run(mk, timeout=600)
            if rc2 != 0:
                raise VolumeError(f"format of {device} as {fstype} failed: {out2.strip()}")
            try:
                await asyncio.to_thread(host.mounter.mount, device, target, fstype, options)
                return
            except MountError as e:
                raise VolumeError(str(e))
        raise VolumeError(str(first))


class PluginMgr:
    """VolumePluginMgr: exactly one plugin must claim a spec."""

    def __init__(self, plugins: list[VolumePlugin], host: VolumeHost):
        self.host = host
        self.plugins: dict[str, VolumePlugin] = {}
        for p in plugins:
            self.add(p)

    def add(self, p: VolumePlugin):
        if p.name in self.plugins:
            raise ValueError(f"volume plugin {p.name!r} was registered more than once")
        p.init(self.host)
        self.plugins[p.name] = p

    def refresh(self):
        """Probe dynamic plugins (FlexVolume drivers dropped into the plugin directory)."""
        from .flex import probe
        for p in probe(self.host.flex_dir):
            if p.name not in self.plugins:
                p.init(self.host)
                self.plugins[p.name] = p

    def find_by_spec(self, spec: Spec) -> VolumePlugin:
        found = [p for p in self.plugins.values() if p.can_support(spec)]
        if not found and os.path.isdir(self.host.flex_dir):
            self.refresh()
            found = [p for p in self.plugins.values() if p.can_support(spec)]
        if not found:
            raise VolumeError(f"no volume plugin matched volume {spec.name()!r}")
        if len(found) > 1:
            raise VolumeError(f"multiple volume plugins matched: {', '.join(sorted(p.name for p in found))}")
        return found[0]

    def find_by_name(self, name: str) -> VolumePlugin:
        p = self.plugins.get(name)
        if p is None and name.startswith("flexvolume-"):
            self.refresh()
            p = self.plugins.get(name)
        if p is None:
            raise VolumeError(f"no volume plugin named {name!r}")
        return p


def sha256_name(*parts: str) -> str:
    return hashlib.sha256("".join(parts).encode()).hexdigest()


def default_plugins() -> list[VolumePlugin]:
    """ProbeVolumePlugins of the reference kubelet (cmd/kubelet/app/plugins.go), MI355X build."""
    from . import csi, local, network
    from . import cinder, vendor
    return [*local.plugins(), *network.plugins(), csi.CSIPlugin(), *cinder.plugins(), *vendor.plugins()]
