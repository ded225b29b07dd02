"""Network and block volume plugins (pkg/volume/nfs, cephfs, glusterfs, quobyte, azure_file,
iscsi, fc, rbd).

File-system protocols mount straight into the pod directory:
  * nfs        `mount -t nfs <server>:<path>` (+ro, PV mountOptions)
  * cephfs     `mount -t ceph <mon,...>:<path> -o name=<user>,secret=<key>|secretfile=<file>`
  * glusterfs  `mount -t glusterfs <ip>:<path>` with the other endpoint IPs as
               backup-volfile-servers and a per-pod log file (endpoints from the pod's namespace)
  * quobyte    `mount -t quobyte <registry>/<volume>` (user/group options)
  * azureFile  `mount -t cifs //<account>.file.core.windows.net/<share>` with the account
               name/key from the secret

Block protocols are attachable: WaitForAttach makes the device appear on the node, the device
is formatted if blank and mounted once at a node-global path, and every pod bind-mounts it:
  * iscsi  iscsiadm discovery + login per portal (CHAP from the secret), device
           /dev/disk/by-path/ip-<portal>-iscsi-<iqn>-lun-<lun>; logout when unmounted
  * fc     SCSI host rescan, device /dev/disk/by-path/*-fc-0x<wwn>-lun-<lun> or
           /dev/disk/by-id/{scsi-,wwn-}<wwid>
  * rbd    `rbd map <pool>/<image> --id <user> -m <mons> --key=<key>`; `rbd unmap` when unmounted
"""
from __future__ import annotations

import asyncio
import glob
import json
import os
import time

from . import VolumeError, VolumePlugin, bind_mount, format_and_mount, unmount_and_remove
from .mount import MountError


async def _mount(host, source, dir, fstype, opts, what):
    os.makedirs(dir, mode=0o750, exist_ok=True)
    if host.mounter.is_mount_point(dir):
        return dir
    try:
        await asyncio.to_thread(host.mounter.mount, source, dir, fstype, opts)
    except MountError as e:
        try:
            os.rmdir(dir)
        except OSError:
            pass
        raise VolumeError(f"{what}: {e}")
    return dir


async def _secret(host, pod, ref: dict | None, default_ns: str | None = None) -> dict:
    if not ref or not ref.get("name"):
        return {}
    ns = ref.get("namespace") or default_ns or ((pod or {}).get("metadata") or {}).get("namespace") or "default"
    return await host.secret(ns, ref["name"])


class NFSPlugin(VolumePlugin):
    name = "kubernetes.io/nfs"
    source_key = "nfs"

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("nfs")
        opts = (["ro"] if spec.source_read_only("nfs") else []) + spec.mount_options()
        return await _mount(self.host, f"{src.get('server', '')}:{src.get('path', '')}", dir, "nfs", opts,
                            f"nfs volume {spec.name()}")


class CephFSPlugin(VolumePlugin):
    name = "kubernetes.io/cephfs"
    source_key = "cephfs"

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("cephfs")
        mons = src.get("monitors") or []
        if not mons:
            raise VolumeError(f"cephfs volume {spec.name()}: no monitors")
        user = src.get("user") or "admin"
        opts = [f"name={user}"]
        if src.get("secretRef"):
            sec = await _secret(self.host, pod, src["secretRef"])
            key = sec.get("key") or next(iter(sec.values()), "")
            opts.append(f"secret={key}")
        else:
            opts.append(f"secretfile={src.get('secretFile') or f'/etc/ceph/{user}.secret'}")
        if spec.source_read_only("cephfs"):
            opts.append("ro")
        return await _mount(self.host, f"{','.join(mons)}:{src.get('path') or '/'}", dir, "ceph", opts + spec.mount_options(),
                            f"cephfs volume {spec.name()}")


class GlusterfsPlugin(VolumePlugin):
    name = "kubernetes.io/glusterfs"
    source_key = "glusterfs"

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("glusterfs")
        ns = src.get("endpointsNamespace") or ((pod or {}).get("metadata") or {}).get("namespace") or "default"
        ep = await self.host.client.get_or_none("endpoints", src.get("endpoints", ""), ns) if self.host.client else None
        ips = [a["ip"] for s in ((ep or {}).get("subsets") or []) for a in s.get("addresses") or []]
        if not ips:
            raise VolumeError(f"glusterfs volume {spec.name()}: endpoints {ns}/{src.get('endpoints')} has no addresses")
        logdir = os.path.join(self.host.plugin_dir(self.name), spec.name())
        os.makedirs(logdir, exist_ok=True)
        uid = ((pod or {}).get("metadata") or {}).get("uid", "")
        opts = [f"log-file={os.path.join(logdir, f'{uid}-glusterfs.log')}", "log-level=ERROR"]
        if len(ips) > 1:
            opts.append("backup-volfile-servers=" + ":".join(ips[1:]))
        if spec.source_read_only("glusterfs"):
            opts.append("ro")
        return await _mount(self.host, f"{ips[0]}:{src.get('path', '')}", dir, "glusterfs", opts + spec.mount_options(),
                            f"glusterfs volume {spec.name()}")


class QuobytePlugin(VolumePlugin):
    name = "kubernetes.io/quobyte"
    source_key = "quobyte"

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("quobyte")
        opts = ["allow-usermapping-in-volumename"]
        if src.get("user"):
            opts.append(f"user={src['user']}")
        if src.get("group"):
            opts.append(f"group={src['group']}")
        if spec.source_read_only("quobyte"):
            opts.append("ro")
        return await _mount(self.host, f"{src.get('registry', '')}/{src.get('volume', '')}", dir, "quobyte",
                            opts + spec.mount_options(), f"quobyte volume {spec.name()}")


class AzureFilePlugin(VolumePlugin):
    name = "kubernetes.io/azure-file"
    source_key = "azureFile"

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("azureFile")
        sec = await _secret(self.host, pod, {"name": src.get("secretName"), "namespace": src.get("secretNamespace")})
        acct, key = sec.get("azurestorageaccountname"), sec.get("azurestorageaccountkey")
        if not acct or not key:
            raise VolumeError(f"azureFile volume {spec.name()}: secret {src.get('secretName')} lacks the storage account")
        opts = ["vers=3.0", f"username={acct}", f"password={key}", "dir_mode=0777", "file_mode=0777"]
        if spec.source_read_only("azureFile"):
            opts.append("ro")
        return await _mount(self.host, f"//{acct}.file.core.windows.net/{src.get('shareName', '')}", dir, "cifs",
                            opts + spec.mount_options(), f"azureFile volume {spec.name()}")


# ---------------------------------------------------------------------------- block
class _Block(VolumePlugin):
    """Attachable block plugin: devices are made visible in wait_for_attach, mounted once at a
    global path and bind-mounted into pods."""
    attachable = True
    access_modes = ("ReadWriteOnce", "ReadOnlyMany")

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        if not device_mount_path:
            raise VolumeError(f"{self.name}: volume {spec.name()} is not mounted on the node")
        await bind_mount(self.host.mounter, device_mount_path, dir, spec.source_read_only(self.source_key))
        return dir

    async def mount_device(self, spec, device_path, device_mount_path):
        if os.path.isdir(device_mount_path) and self.host.mounter.is_mount_point(device_mount_path):
            return
        src = spec.source(self.source_key)
        opts = (["ro"] if spec.source_read_only(self.source_key) else []) + spec.mount_options()
        await format_and_mount(self.host, device_path, device_mount_path, src.get("fsType") or "ext4", opts)
        self._save(device_mount_path, spec)

    def _save(self, device_mount_path, spec):
        """The global mount's source, kept next to it so teardown after a restart can log out /
        unmap without the pod spec (persistISCSI / rbd's json)."""
        with open(device_mount_path.rstrip("/") + ".json", "w") as f:
            json.dump({"source": spec.source(self.source_key), "name": spec.name()}, f)

    def _load(self, device_mount_path) -> dict:
        try:
            with open(device_mount_path.rstrip("/") + ".json") as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    async def _wait_device(self, patterns: list[str], timeout: float, what: str) -> str:
        deadline = time.monotonic() + timeout
        while True:
            for p in patterns:
                hits = sorted(glob.glob(os.path.join(self.host.dev_root, p.lstrip("/"))))
                if hits:
                    return hits[0]
            if time.monotonic() >= deadline:
                raise VolumeError(f"{what}: device did not appear ({', '.join(patterns)})")
            await asyncio.sleep(min(self.host.attach_poll, max(0.01, deadline - time.monotonic())))


class ISCSIPlugin(_Block):
    name = "kubernetes.io/iscsi"
    source_key = "iscsi"

    def _disk(self, spec) -> dict:
        src = spec.source("iscsi")
        portal = src.get("targetPortal", "")
        if portal and ":" not in portal:
            portal += ":3260"
        portals = [portal] + [p if ":" in p else p + ":3260" for p in src.get("portals") or []]
        iface = src.get("iscsiInterface") or "default"
        if src.get("initiatorName"):
            iface = f"{portal}:{spec.name()}"
        return {"portals": portals, "iqn": src.get("iqn", ""), "lun": str(src.get("lun", 0)), "iface": iface,
                "initiator": src.get("initiatorName", "")}

    def volume_name(self, spec):
        d = self._disk(spec)
        return f"{d['portals'][0]}:{d['iqn']}:{d['lun']}"

    def device_mount_path(self, spec):
        d = self._disk(spec)
        return os.path.join(self.host.plugin_dir(self.name), f"iface-{d['iface']}",
                            f"{d['portals'][0]}-{d['iqn']}-lun-{d['lun']}")

    async def _iscsiadm(self, *args, ok_codes=(0,)):
        rc, out = await self.host.run(["iscsiadm", *args])
        if rc not in ok_codes:
            raise VolumeError(f"iscsiadm {' '.join(args)} failed ({rc}): {out.strip()}")
        return out

    async def wait_for_attach(self, spec, device_path, pod, timeout):
        d = self._disk(spec)
        src = spec.source("iscsi")
        chap = {}
        if src.get("chapAuthDiscovery") or src.get("chapAuthSession"):
            sec = await _secret(self.host, pod, src.get("secretRef"))
            if not sec:
                raise VolumeError(f"iscsi volume {spec.name()}: CHAP enabled but no secret")
            chap = sec
        if d["initiator"]:
            # a dedicated iface bound to the requested initiator name (cloneIface)
            await self._iscsiadm("-m", "iface", "-I", d["iface"], "-o", "new", ok_codes=(0, 15))
            await self._iscsiadm("-m", "iface", "-I", d["iface"], "-o", "update", "-n", "iface.initiatorname",
                                 "-v", d["initiator"])
        for tp in d["portals"]:
            await self._iscsiadm("-m", "discoverydb", "-t", "sendtargets", "-p", tp, "-I", d["iface"], "-o", "new",
                                 ok_codes=(0, 15))
            if src.get("chapAuthDiscovery"):
                await self._iscsiadm("-m", "discoverydb", "-t", "sendtargets", "-p", tp, "-I", d["iface"], "-o", "update",
                                     "-n", "discovery.sendtargets.auth.authmethod", "-v", "CHAP")
                for k in ("username", "password", "username_in", "password_in"):
                    if f"discovery.sendtargets.auth.{k}" in chap:
                        await self._iscsiadm("-m", "discoverydb", "-t", "sendtargets", "-p", tp, "-I", d["iface"], "-o",
                                             "update", "-n", f"discovery.sendtargets.auth.{k}",
                                             "-v", chap[f"discovery.sendtargets.auth.{k}"])
            await self._iscsiadm("-m", "discoverydb", "-t", "sendtargets", "-p", tp, "-I", d["iface"], "--discover")
            if src.get("chapAuthSession"):
                await self._iscsiadm("-m", "node", "-p", tp, "-T", d["iqn"], "-I", d["iface"], "-o", "update",
                                     "-n", "node.session.auth.authmethod", "-v", "CHAP")
                for k in ("username", "password", "username_in", "password_in"):
                    if f"node.session.auth.{k}" in chap:
                        await self._iscsiadm("-m", "node", "-p", tp, "-T", d["iqn"], "-I", d["iface"], "-o", "update",
                                             "-n", f"node.session.auth.{k}", "-v", chap[f"node.session.auth.{k}"])
            await self._iscsiadm("-m", "node", "-p", tp, "-T", d["iqn"], "-I", d["iface"], "--login", ok_codes=(0, 15))
        pats = [f"/dev/disk/by-path/ip-{tp}-iscsi-{d['iqn']}-lun-{d['lun']}" for tp in d["portals"]] + \
            [f"/dev/disk/by-path/pci-*-ip-{tp}-iscsi-{d['iqn']}-lun-{d['lun']}" for tp in d["portals"]]
        return await self._wait_device(pats, timeout, f"iscsi volume {spec.name()}")

    async def unmount_device(self, device_mount_path):
        info = self._load(device_mount_path)
        await unmount_and_remove(self.host.mounter, device_mount_path)
        src = info.get("source") or {}
        if src:
            from . import Spec
            d = self._disk(Spec(volume={"name": info.get("name", ""), "iscsi": src}))
            for tp in d["portals"]:
                await self._iscsiadm("-m", "node", "-p", tp, "-T", d["iqn"], "-I", d["iface"], "--logout", ok_codes=(0, 21))
                await self._iscsiadm("-m", "node", "-p", tp, "-T", d["iqn"], "-I", d["iface"], "-o", "delete", ok_codes=(0, 21))
        try:
            os.unlink(device_mount_path.rstrip("/") + ".json")
        except OSError:
            pass


class FCPlugin(_Block):
    name = "kubernetes.io/fc"
    source_key = "fc"

    def volume_name(self, spec):
        src = spec.source("fc")
        if src.get("wwids"):
            return ",".join(src["wwids"])
        return f"{','.join(src.get('targetWWNs') or [])}:{src.get('lun', 0)}"

    def device_mount_path(self, spec):
        src = spec.source("fc")
        if src.get("wwids"):
            leaf = src["wwids"][0]
        else:
            leaf = f"{(src.get('targetWWNs') or [''])[0]}-lun-{src.get('lun', 0)}"
        return os.path.join(self.host.plugin_dir(self.name), leaf)

    async def wait_for_attach(self, spec, device_path, pod, timeout):
        src = spec.source("fc")
        # rescan every SCSI host so newly zoned LUNs show up (fc_util.go rescaning)
        for scan in glob.glob(os.path.join(self.host.sys_root, "class", "scsi_host", "host*", "scan")):
            try:
                with open(scan, "w") as f:
                    f.write("- - -")
            except OSError:
                pass
        if src.get("wwids"):
            pats = [p for w in src["wwids"] for p in (f"/dev/disk/by-id/scsi-{w}", f"/dev/disk/by-id/wwn-{w}")]
        elif src.get("targetWWNs") and src.get("lun") is not None:
            pats = [f"/dev/disk/by-path/*-fc-0x{w}-lun-{src['lun']}" for w in src["targetWWNs"]]
        else:
            raise VolumeError(f"fc volume {spec.name()}: targetWWNs+lun or wwids required")
        return await self._wait_device(pats, timeout, f"fc volume {spec.name()}")


class RBDPlugin(_Block):
    name = "kubernetes.io/rbd"
    source_key = "rbd"

    def volume_name(self, spec):
        src = spec.source("rbd")
        return f"{src.get('pool') or 'rbd'}-image-{src.get('image', '')}"

    def device_mount_path(self, spec):
        return os.path.join(self.host.plugin_dir(self.name), "rbd", self.volume_name(spec))

    async def wait_for_attach(self, spec, device_path, pod, timeout):
        src = spec.source("rbd")
        pool, image = src.get("pool") or "rbd", src.get("image", "")
        user = src.get("user") or "admin"
        argv = ["rbd", "map", f"{pool}/{image}", "--id", user, "-m", ",".join(src.get("monitors") or [])]
        if src.get("secretRef"):
            sec = await _secret(self.host, pod, src["secretRef"])
            key = sec.get("key") or next(iter(sec.values()), "")
            argv.append(f"--key={key}")
        else:
            argv.append(f"--keyring={src.get('keyring') or '/etc/ceph/keyring'}")
        # already mapped? (rbd showmapped) — the reference checks /dev/rbd/<pool>/<image>
        link = os.path.join(self.host.dev_root, "dev", "rbd", pool, image)
        if os.path.exists(link):
            return os.path.realpath(link)
        rc, out = await self.host.run(argv, timeout=timeout)
        if rc != 0:
            raise VolumeError(f"rbd: map of {pool}/{image} failed: {out.strip()}")
        dev = out.strip().splitlines()[-1].strip() if out.strip() else ""
        if dev.startswith("/dev/"):
            return dev
        return await self._wait_device([f"/dev/rbd/{pool}/{image}"], timeout, f"rbd volume {spec.name()}")

    async def unmount_device(self, device_mount_path):
        info = self._load(device_mount_path)
        dev = None
        for mp in self.host.mounter.list():
            if mp.path == os.path.realpath(device_mount_path):
                dev = mp.device
        await unmount_and_remove(self.host.mounter, device_mount_path)
        if dev is None and info.get("source"):
            s = info["source"]
            dev = os.path.join("/dev/rbd", s.get("pool") or "rbd", s.get("image", ""))
        if dev:
            rc, out = await self.host.run(["rbd", "unmap", dev])
            if rc != 0:
                raise VolumeError(f"rbd: unmap of {dev} failed: {out.strip()}")
        try:
            os.unlink(device_mount_path.rstrip("/") + ".json")
        except OSError:
            pass


def plugins() -> list[VolumePlugin]:
    return [NFSPlugin(), CephFSPlugin(), GlusterfsPlugin(), QuobytePlugin(), AzureFilePlugin(), ISCSIPlugin(), FCPlugin(),
            RBDPlugin()]

