"""FlexVolume (pkg/volume/flexvolume): out-of-tree volume drivers as executables.

A driver lives at `<volume plugin dir>/<vendor>~<driver>/<driver>` and is probed when it
appears (probe.go); `init` must answer Success and may report `capabilities.attach: false`.
The plugin name is `flexvolume-<vendor>/<driver>` and it claims `flexVolume` sources whose
`driver` is `<vendor>/<driver>`. Calls (driver-call.go):

  init | getvolumename <json> | attach <json> <node> | waitforattach <device> <json> |
  mountdevice <mount dir> <device> <json> | mount <mount dir> <json> | unmount <mount dir> |
  unmountdevice <mount dir> | detach <volume name> <node> | isattached <json> <node>

The JSON options hold kubernetes.io/fsType, kubernetes.io/readwrite (ro|rw),
kubernetes.io/pvOrVolumeName, the pod's name/namespace/uid/serviceAccount.name (mount), the
fsGroup, kubernetes.io/secret/<key> (base64, from secretRef) and the source's `options`. The
reply is JSON: {"status": "Success"|"Failure"|"Not supported", "message", "device",
"volumeName", "attached", "capabilities"}. A "Not supported" command is remembered and the
default behaviour runs instead (mount: bind the device mount; attach: no-op; unmount: unmount).
"""
from __future__ import annotations

import asyncio
import base64
import json
import os

from . import VolumeError, VolumePlugin, bind_mount, unmount_and_remove

NOT_SUPPORTED = "Not supported"


class DriverNotSupported(VolumeError):
    pass


def probe(plugin_dir: str) -> list["FlexVolumePlugin"]:
    """probe.go: every `<vendor>~<driver>/<driver>` executable whose init succeeds."""
    out = []
    if not os.path.isdir(plugin_dir):
        return out
    for d in sorted(os.listdir(plugin_dir)):
        if d.startswith("."):
            continue
        drv = d.split("~")[-1]
        exe = os.path.join(plugin_dir, d, drv)
        if not (os.path.isfile(exe) and os.access(exe, os.X_OK)):
            continue
        p = FlexVolumePlugin(d.replace("~", "/"), exe)
        try:
            p.capabilities = p._call_sync("init")
        except VolumeError:
            continue
        out.append(p)
    return out


def _parse(cmd: str, out: bytes) -> dict:
    try:
        st = json.loads(out.decode(errors="replace") or "null")
    except ValueError:
        raise VolumeError(f"flexvolume {cmd}: unparsable driver output {out[:200]!r}")
    if not isinstance(st, dict):
        raise VolumeError(f"flexvolume {cmd}: driver output is not an object")
    if st.get("status") == NOT_SUPPORTED:
        raise DriverNotSupported(NOT_SUPPORTED)
    if st.get("status") != "Success":
        raise VolumeError(f"{cmd} command failed, status: {st.get('status')}, reason: {st.get('message', '')}")
    return st


class FlexVolumePlugin(VolumePlugin):
    source_key = "flexVolume"
    access_modes = ("ReadWriteOnce", "ReadOnlyMany")

    def __init__(self, driver: str, exe: str, timeout: float = 120.0):
        self.driver, self.exe, self.timeout = driver, exe, timeout
        self.name = "flexvolume-" + driver
        self.unsupported: set[str] = set()
        self.capabilities: dict = {}

    @property
    def attachable(self):
        caps = self.capabilities.get("capabilities") or {}
        return bool(caps.get("attach", True))

    def can_support(self, spec):
        return spec.has("flexVolume") and spec.source("flexVolume").get("driver") == self.driver

    # ---------------------------------------------------------------- calls
    def _call_sync(self, cmd: str, *args: str) -> dict:
        import subprocess
        try:
            r = subprocess.run([self.exe, cmd, *args], capture_output=True, timeout=self.timeout)
        except (OSError, subprocess.TimeoutExpired) as e:
            raise VolumeError(f"flexvolume {self.driver} {cmd}: {e}")
        return _parse(cmd, r.stdout or r.stderr)

    async def call(self, cmd: str, *args: str, timeout: float | None = None) -> dict:
        if cmd in self.unsupported:
            raise DriverNotSupported(NOT_SUPPORTED)
        try:
            proc = await asyncio.create_subprocess_exec(self.exe, cmd, *args, stdout=asyncio.subprocess.PIPE,
                                                        stderr=asyncio.subprocess.STDOUT)
        except OSError as e:
            raise VolumeError(f"flexvolume {self.driver} {cmd}: {e}")
        try:
            out, _ = await asyncio.wait_for(proc.communicate(), timeout or self.timeout)
        except asyncio.TimeoutError:
            proc.kill()
            await proc.wait()
            raise VolumeError(f"flexvolume {self.driver} {cmd}: Timeout")
        try:
            return _parse(cmd, out)
        except DriverNotSupported:
            self.unsupported.add(cmd)
            raise

    async def options(self, spec, pod: dict | None = None, extra: dict | None = None) -> str:
        src = spec.source("flexVolume")
        o = {"kubernetes.io/fsType": src.get("fsType", ""),
             "kubernetes.io/readwrite": "ro" if spec.source_read_only("flexVolume") else "rw",
             "kubernetes.io/pvOrVolumeName": spec.name()}
        o.update(extra or {})
        ref = src.get("secretRef") or {}
        if ref.get("name") and pod is not None:
            ns = ((pod.get("metadata") or {}).get("namespace")) or "default"
            obj = await self.host.client.get_or_none("secrets", ref["name"], ns) if self.host.client else None
            if obj is None:
                raise VolumeError(f"flexvolume {self.driver}: secret {ns}/{ref['name']} not found")
            for k, v in (obj.get("data") or {}).items():
                o[f"kubernetes.io/secret/{k}"] = v      # still base64, as the reference passes it
        o.update(src.get("options") or {})
        return json.dumps(o, sort_keys=True)

    # ----------------------------------------------------------- plugin api
    def volume_name(self, spec):
        # getvolumename is a TODO in the reference too: the PV / volume name is used
        return spec.name()

    def device_mount_path(self, spec):
        return os.path.join(self.host.plugin_dir("kubernetes.io/flexvolume"), self.driver, "mounts", self.volume_name(spec))

    async def attach(self, spec, node):
        try:
            return (await self.call("attach", await self.options(spec), node)).get("device", "")
        except DriverNotSupported:
            return ""

    async def wait_for_attach(self, spec, device_path, pod, timeout):
        try:
            return (await self.call("waitforattach", device_path, await self.options(spec), timeout=timeout)).get("device", "")
        except DriverNotSupported:
            return device_path

    async def mount_device(self, spec, device_path, device_mount_path):
        if os.path.isdir(device_mount_path) and self.host.mounter.is_mount_point(device_mount_path):
            return
        os.makedirs(device_mount_path, mode=0o750, exist_ok=True)
        try:
            await self.call("mountdevice", device_mount_path, device_path, await self.options(spec))
        except DriverNotSupported:
            if device_path:
                from . import format_and_mount
                await format_and_mount(self.host, device_path, device_mount_path, spec.source("flexVolume").get("fsType", ""),
                                       ["ro"] if spec.source_read_only("flexVolume") else [])
        except VolumeError:
            try:
                os.rmdir(device_mount_path)
            except OSError:
                pass
            raise

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        if os.path.isdir(dir) and self.host.mounter.is_mount_point(dir):
            return dir
        os.makedirs(dir, mode=0o750, exist_ok=True)
        md = (pod or {}).get("metadata") or {}
        extra = {"kubernetes.io/pod.name": md.get("name", ""), "kubernetes.io/pod.namespace": md.get("namespace", ""),
                 "kubernetes.io/pod.uid": md.get("uid", ""),
                 "kubernetes.io/serviceAccount.name": ((pod or {}).get("spec") or {}).get("serviceAccountName", "")}
        if fs_group is not None:
            extra["kubernetes.io/fsGroup"] = str(fs_group)
        try:
            await self.call("mount", dir, await self.options(spec, pod, extra))
        except DriverNotSupported:
            # mounterDefaults: bind the device mount
            await bind_mount(self.host.mounter, device_mount_path or self.device_mount_path(spec), dir,
                             spec.source_read_only("flexVolume"))
        except VolumeError:
            try:
                os.rmdir(dir)
            except OSError:
                pass
            raise
        return dir

    async def tear_down(self, dir):
        if not os.path.lexists(dir):
            return
        try:
            await self.call("unmount", dir)
        except DriverNotSupported:
            await unmount_and_remove(self.host.mounter, dir)
            return
        if os.path.lexists(dir):
            os.rmdir(dir)

    async def unmount_device(self, device_mount_path):
        if not os.path.lexists(device_mount_path):
            return
        if self.host.mounter.is_mount_point(device_mount_path):
            try:
                await self.call("unmountdevice", device_mount_path)
            except DriverNotSupported:
                await unmount_and_remove(self.host.mounter, device_mount_path)
                return
        if os.path.lexists(device_mount_path):
            os.rmdir(device_mount_path)

    async def detach(self, volume_name, node):
        try:
            await self.call("detach", volume_name, node)
        except DriverNotSupported:
            pass

    async def is_attached(self, spec, node) -> bool | None:
        try:
            return bool((await self.call("isattached", await self.options(spec), node)).get("attached"))
        except DriverNotSupported:
            return None


def secret_option(data: dict[str, str]) -> dict[str, str]:
    """The kubernetes.io/secret/<key> options a driver receives for decoded secret data."""
    return {f"kubernetes.io/secret/{k}": base64.b64encode(v.encode()).decode() for k, v in data.items()}
