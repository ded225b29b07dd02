"""Vendor storage backends spoken over their REST APIs (reference: pkg/volume/flocker,
pkg/volume/storageos, pkg/volume/portworx, pkg/volume/scaleio — plugin, util and client files).

None of them is attachable through the attach/detach controller in v1.9: the kubelet's SetUp
asks the backend for the volume on this node, mounts it once at a node-global path and
bind-mounts it into the pod (Portworx mounts straight into the pod directory itself). Each
has a dynamic provisioner for its StorageClass provisioner name, used by the PV controller
(`controllers/volumes.py`), which also deletes provisioned volumes on reclaim.

  * flocker   — control service `/v1/configuration/datasets`, `/v1/state/datasets`,
                `/v1/state/nodes` (TLS with the cluster CA and an API-user certificate from
                FLOCKER_CONTROL_SERVICE_*): find the dataset (by datasetUUID or metadata name),
                make this node (matched by host IP) its primary and wait until the state shows
                it here, then bind-mount the dataset's state path.
  * storageos — `/v1/namespaces/{ns}/volumes[/{name}[/mount|/unmount]]` with basic auth
                (API address and credentials from the volume's secretRef, default
                tcp://localhost:5705): the volume's device file lives under
                /var/lib/storageos/volumes/<id>; a regular file is bound to a loop device
                (`losetup --find --show`), formatted if blank and mounted at the global path.
  * portworx  — the openstorage REST API `/v1/osd-volumes` on the node (port 9001): attach
                and mount are `PUT /v1/osd-volumes/{id}` actions; the driver mounts the volume
                at the pod directory.
  * scaleIO   — the gateway REST API (`/api/login` token, `types/Volume/instances`,
                `instances/Volume::{id}/action/addMappedSdc|removeMappedSdc|removeVolume`,
                `types/Sdc/instances`): the volume is mapped to this node's SDC (GUID from the
                `scaleio.sdcGuid` node label or `drv_cfg --query_guid`) and appears as
                /dev/disk/by-id/emc-vol-<mdm id>-<volume id>.
No such backend exists offline: the request shapes follow the vendors' public API
documentation and are tested against in-repo fakes (tests/fake_storage.py), so parity with the
real services is unpinned.
"""
from __future__ import annotations

import asyncio
import base64
import glob
import hashlib
import json
import os
import time

from . import VolumeError, VolumePlugin, bind_mount, format_and_mount, unmount_and_remove

GIB = 1 << 30


def _http():
    """A requests session whose transport failures surface as VolumeError (FailedMount events
    name the unreachable backend instead of a raw connection traceback)."""
    import requests

    class Session(requests.Session):
        def request(self, method, url, *a, **kw):
            try:
                return super().request(method, url, *a, **kw)
            except requests.RequestException as e:
                raise VolumeError(f"storage backend at {url.split('?', 1)[0]} is unreachable: {e.__class__.__name__}") from e
    return Session()


def _raise(r, what: str):
    if r.status_code >= 400:
        raise VolumeError(f"{what}: HTTP {r.status_code}: {r.text[:200]}")


class _Vendor(VolumePlugin):
    """Shared per-pod bookkeeping: what a pod directory holds, so teardown (which only gets the
    directory) can release the backend volume when its last pod on this node goes."""

    def _rec_path(self, dir: str) -> str:
        return os.path.join(self.host.plugin_dir(self.name), "pods", hashlib.sha256(dir.encode()).hexdigest()[:32] + ".json")

    def _record(self, dir: str, rec: dict):
        p = self._rec_path(dir)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            json.dump(rec, f)

    def _recall(self, dir: str) -> dict:
        try:
            with open(self._rec_path(dir)) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    def _forget(self, dir: str):
        try:
            os.unlink(self._rec_path(dir))
        except OSError:
            pass

    def global_path(self, key: str) -> str:
        return os.path.join(self.host.plugin_dir(self.name), "mounts", key.replace("/", "~"))

    def _users(self, global_path: str) -> int:
        """Pods on this node that still bind the global mount."""
        d = os.path.join(self.host.plugin_dir(self.name), "pods")
        n = 0
        for f in glob.glob(os.path.join(d, "*.json")):
            try:
                with open(f) as fh:
                    n += json.load(fh).get("global") == global_path
            except (OSError, ValueError):
                pass
        return n

    async def _mount_global(self, device: str, gp: str, fstype: str, ro: bool):
        if not (os.path.isdir(gp) and self.host.mounter.is_mount_point(gp)):
            await format_and_mount(self.host, device, gp, fstype or "ext4", ["ro"] if ro else [])

    async def tear_down(self, dir: str):
        rec = self._recall(dir)
        await unmount_and_remove(self.host.mounter, dir)
        self._forget(dir)
        gp = rec.get("global")
        if rec and (not gp or self._users(gp) == 0):
            if gp:
                await unmount_and_remove(self.host.mounter, gp)
            await self.release(rec)

    async def release(self, rec: dict):
        pass


# ------------------------------------------------------------------------------ flocker
class FlockerClient:
    def __init__(self, host_ip: str, http=None):
        env = os.environ.get
        self.base = (f"{env('FLOCKER_CONTROL_SERVICE_PROTOCOL', 'https')}://{env('FLOCKER_CONTROL_SERVICE_HOST', 'localhost')}:"
                     f"{env('FLOCKER_CONTROL_SERVICE_PORT', '4523')}/v1")
        self.host_ip = host_ip
        self.http = http or _http()
        if self.base.startswith("https"):
            self.http.verify = env("FLOCKER_CONTROL_SERVICE_CA_FILE", "/etc/flocker/cluster.crt")
            self.http.cert = (env("FLOCKER_CONTROL_SERVICE_CLIENT_CERT_FILE", "/etc/flocker/apiuser.crt"),
                              env("FLOCKER_CONTROL_SERVICE_CLIENT_KEY_FILE", "/etc/flocker/apiuser.key"))

    def _get(self, path):
        r = self.http.get(self.base + path, timeout=30)
        _raise(r, f"flocker GET {path}")
        return r.json()

    def _post(self, path, body):
        r = self.http.post(self.base + path, json=body, timeout=30)
        _raise(r, f"flocker POST {path}")
        return r.json()

    def primary_uuid(self) -> str:
        for n in self._get("/state/nodes"):
            if n.get("host") == self.host_ip:
                return n["uuid"]
        raise VolumeError(f"flocker: no node with host {self.host_ip} in the cluster state")

    def dataset_id(self, name: str) -> str:
        for d in self._get("/configuration/datasets"):
            if (d.get("metadata") or {}).get("name") == name and not d.get("deleted"):
                return d["dataset_id"]
        raise VolumeError(f"flocker: no dataset named {name!r}")

    def state(self, dataset_id: str) -> dict | None:
        return next((d for d in self._get("/state/datasets") if d.get("dataset_id") == dataset_id), None)

    def move(self, dataset_id: str, primary: str):
        self._post(f"/configuration/datasets/{dataset_id}", {"primary": primary})

    def create(self, name: str, size: int, primary: str) -> str:
        return self._post("/configuration/datasets", {"primary": primary, "maximum_size": size, "metadata": {"name": name}})["dataset_id"]

    def delete(self, dataset_id: str):
        r = self.http.delete(f"{self.base}/configuration/datasets/{dataset_id}", timeout=30)
        if r.status_code != 404:
            _raise(r, "flocker delete dataset")


class FlockerPlugin(_Vendor):
    name = "kubernetes.io/flocker"
    source_key = "flocker"
    wait_timeout, wait_tick = 120.0, 0.5

    def volume_name(self, spec) -> str:
        src = spec.source("flocker")
        return src.get("datasetUUID") or src.get("datasetName") or ""

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("flocker")
        c = FlockerClient(self.host.node_ip)

        def ready() -> str:
            ds = src.get("datasetUUID") or c.dataset_id(src.get("datasetName", ""))
            me = c.primary_uuid()
            st = c.state(ds)
            if st is None or st.get("primary") != me:
                c.move(ds, me)
                end = time.monotonic() + self.wait_timeout
                while True:
                    st = c.state(ds)
                    if st is not None and st.get("primary") == me and st.get("path"):
                        break
                    if time.monotonic() > end:
                        raise VolumeError(f"timed out waiting for dataset {ds} to move to primary {me}")
                    time.sleep(self.wait_tick)
            return os.path.join(self.host.dev_root, st["path"].lstrip("/"))
        path = await asyncio.to_thread(ready)
        await bind_mount(self.host.mounter, path, dir, spec.source_read_only("flocker"))
        self._record(dir, {"path": path})
        return dir


class FlockerProvisioner:
    provisioner = "kubernetes.io/flocker"
    source_key = "flocker"

    async def aprovision(self, client, name, gib, params, tags, pvc_name):
        def go():
            c = FlockerClient(os.environ.get("FLOCKER_PRIMARY_HOST", ""))
            nodes = c._get("/state/nodes")
            if not nodes:
                raise VolumeError("flocker: the cluster has no nodes")
            primary = next((n["uuid"] for n in nodes if n.get("host") == c.host_ip), nodes[0]["uuid"])
            return c.create(name, gib * GIB, primary)
        ds = await asyncio.to_thread(go)
        return {"datasetUUID": ds}, {}

    async def adelete(self, client, src: dict):
        await asyncio.to_thread(FlockerClient("").delete, src["datasetUUID"])


# ---------------------------------------------------------------------------- storageos
def _b64(s: str) -> str:
    return base64.b64decode(s).decode() if s else ""


async def _secret_data(client, ns: str, name: str) -> dict:
    if not name or client is None:
        return {}
    obj = await client.get_or_none("secrets", name, ns)
    if obj is None:
        raise VolumeError(f'secret "{ns}/{name}" not found')
    return {k: _b64(v) for k, v in (obj.get("data") or {}).items()}


class StorageOSClient:
    def __init__(self, cfg: dict, http=None):
        addr = cfg.get("apiAddress") or "tcp://localhost:5705"
        self.base = addr.replace("tcp://", "http://", 1).rstrip("/") + "/v" + str(cfg.get("apiVersion") or "1").lstrip("v")
        self.auth = (cfg.get("apiUsername") or "storageos", cfg.get("apiPassword") or "storageos")
        self.http = http or _http()

    def call(self, method, path, body=None, ok404=False):
        r = self.http.request(method, self.base + path, json=body, auth=self.auth, timeout=30)
        if ok404 and r.status_code == 404:
            return None
        _raise(r, f"storageos {method} {path}")
        return r.json() if r.content else {}

    def volume(self, ns, name):
        return self.call("GET", f"/namespaces/{ns}/volumes/{name}", ok404=True)

    def create(self, ns, name, gib, pool="", fstype="", description="", labels=None):
        return self.call("POST", f"/namespaces/{ns}/volumes", {"name": name, "size": gib, "pool": pool, "fsType": fstype,
                                                              "description": description, "labels": labels or {}})

    def mount(self, ns, name, client, mountpoint, fstype):
        self.call("POST", f"/namespaces/{ns}/volumes/{name}/mount",
                  {"name": name, "namespace": ns, "client": client, "mountpoint": mountpoint, "fsType": fstype})

    def unmount(self, ns, name, client):
        self.call("POST", f"/namespaces/{ns}/volumes/{name}/unmount", {"name": name, "namespace": ns, "client": client})

    def delete(self, ns, name):
        self.call("DELETE", f"/namespaces/{ns}/volumes/{name}", ok404=True)


class StorageOSPlugin(_Vendor):
    name = "kubernetes.io/storageos"
    source_key = "storageos"
    device_dir = "/var/lib/storageos/volumes"

    def volume_name(self, spec) -> str:
        src = spec.source("storageos")
        return f"{src.get('volumeNamespace') or 'default'}.{src.get('volumeName', '')}"

    async def _cfg(self, src, pod) -> dict:
        ref = src.get("secretRef") or {}
        ns = ref.get("namespace") or ((pod or {}).get("metadata") or {}).get("namespace") or "default"
        return await _secret_data(self.host.client, ns, ref.get("name", ""))

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("storageos")
        vns, vname = src.get("volumeNamespace") or ((pod or {}).get("metadata") or {}).get("namespace") or "default", src.get("volumeName", "")
        cfg = await self._cfg(src, pod)
        api = StorageOSClient(cfg)
        vol = await asyncio.to_thread(api.volume, vns, vname)
        if vol is None:
            raise VolumeError(f"storageos volume {vns}/{vname} not found")
        dev = os.path.join(self.host.dev_root, self.device_dir.lstrip("/"), vol["id"])
        if not os.path.exists(dev):
            raise VolumeError(f"storageos volume {vns}/{vname}: device {dev} is not present on this node")
        if os.path.isfile(dev):                 # a file-backed volume: bind it to a loop device
            rc, out = await self.host.run(["losetup", "-j", dev])
            loop = out.split(":", 1)[0].strip() if rc == 0 and out.strip() else ""
            if not loop:
                rc, out = await self.host.run(["losetup", "--find", "--show", dev])
                if rc != 0:
                    raise VolumeError(f"losetup {dev}: {out.strip()}")
                loop = out.strip()
            dev = loop
        gp = self.global_path(f"{vns}.{vname}")
        fstype = src.get("fsType") or vol.get("fsType") or "ext4"
        await self._mount_global(dev, gp, fstype, spec.source_read_only("storageos"))
        await asyncio.to_thread(api.mount, vns, vname, self.host.node_name, gp, fstype)
        await bind_mount(self.host.mounter, gp, dir, spec.source_read_only("storageos"))
        self._record(dir, {"global": gp, "ns": vns, "name": vname, "cfg": {k: cfg[k] for k in ("apiAddress",) if k in cfg},
                           "secret": (src.get("secretRef") or {}), "pod_ns": ((pod or {}).get("metadata") or {}).get("namespace"),
                           "device": dev})
        return dir

    async def release(self, rec):
        ref = rec.get("secret") or {}
        cfg = await _secret_data(self.host.client, ref.get("namespace") or rec.get("pod_ns") or "default", ref.get("name", ""))
        await asyncio.to_thread(StorageOSClient(cfg).unmount, rec["ns"], rec["name"], self.host.node_name)
        if (rec.get("device") or "").startswith("/dev/loop"):
            await self.host.run(["losetup", "-d", rec["device"]])


class StorageOSProvisioner:
    provisioner = "kubernetes.io/storageos"
    source_key = "storageos"

    async def _cfg(self, client, params):
        p = {k.lower(): v for k, v in params.items()}
        return await _secret_data(client, p.get("adminsecretnamespace", "default"), p.get("adminsecretname", "")), p

    async def aprovision(self, client, name, gib, params, tags, pvc_name):
        cfg, p = await self._cfg(client, params)
        ns = tags.get("kubernetes.io/created-for/pvc/namespace", "default")
        labels = {k: v for k, v in tags.items()}
        vol = await asyncio.to_thread(StorageOSClient(cfg).create, ns, name, gib, p.get("pool", ""), p.get("fstype", "ext4"),
                                      p.get("description", "Kubernetes volume"), labels)
        src = {"volumeName": vol.get("name", name), "volumeNamespace": ns, "fsType": vol.get("fsType") or p.get("fstype", "ext4")}
        if p.get("adminsecretname"):
            src["secretRef"] = {"name": p["adminsecretname"], "namespace": p.get("adminsecretnamespace", "default")}
        return src, {}

    async def adelete(self, client, src):
        ref = src.get("secretRef") or {}
        cfg = await _secret_data(client, ref.get("namespace", "default"), ref.get("name", ""))
        await asyncio.to_thread(StorageOSClient(cfg).delete, src.get("volumeNamespace", "default"), src["volumeName"])


# ----------------------------------------------------------------------------- portworx
def portworx_endpoint() -> str:
    return os.environ.get("AMDKUBE_PORTWORX_ENDPOINT", "http://127.0.0.1:9001").rstrip("/")


class PortworxClient:
    ON, OFF = 1, 2          # openstorage api.ParamOn / ParamOff

    def __init__(self, base: str, http=None):
        self.base, self.http = base, http or _http()

    def call(self, method, path, body=None):
        r = self.http.request(method, self.base + "/v1/osd-volumes" + path, json=body, timeout=60)
        _raise(r, f"portworx {method} {path or '/'}")
        out = r.json() if r.content else {}
        if isinstance(out, dict) and out.get("error"):
            raise VolumeError(f"portworx: {out['error']}")
        return out

    def inspect(self, vid: str) -> dict | None:
        vols = self.call("GET", f"/{vid}")
        return vols[0] if vols else None

    def attach(self, vid: str) -> str:
        return self.call("PUT", f"/{vid}", {"action": {"attach": self.ON}}).get("device_path", "")

    def mount(self, vid: str, path: str):
        self.call("PUT", f"/{vid}", {"action": {"mount": self.ON, "mount_path": path}})

    def unmount(self, vid: str, path: str):
        self.call("PUT", f"/{vid}", {"action": {"mount": self.OFF, "mount_path": path}})

    def detach(self, vid: str):
        self.call("PUT", f"/{vid}", {"action": {"attach": self.OFF}})

    def create(self, name: str, size: int, spec: dict, labels: dict) -> str:
        return self.call("POST", "", {"locator": {"name": name, "volume_labels": labels},
                                      "spec": {"size": size, **spec}, "source": {}})["id"]

    def delete(self, vid: str):
        self.call("DELETE", f"/{vid}")


class PortworxPlugin(_Vendor):
    name = "kubernetes.io/portworx-volume"
    source_key = "portworxVolume"

    def volume_name(self, spec) -> str:
        return spec.source("portworxVolume").get("volumeID", "")

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        vid = self.volume_name(spec)
        px = PortworxClient(portworx_endpoint())
        os.makedirs(dir, mode=0o750, exist_ok=True)

        def go():
            vol = px.inspect(vid)
            if vol is None:
                raise VolumeError(f"portworx volume {vid} not found")
            if not vol.get("attached_on"):
                px.attach(vid)
            if dir not in (vol.get("attach_path") or []):
                px.mount(vid, dir)
        await asyncio.to_thread(go)
        self._record(dir, {"id": vid})
        return dir

    async def tear_down(self, dir: str):
        rec = self._recall(dir)
        if rec:
            px = PortworxClient(portworx_endpoint())

            def go():
                px.unmount(rec["id"], dir)
                vol = px.inspect(rec["id"]) or {}
                if not vol.get("attach_path"):
                    px.detach(rec["id"])
            await asyncio.to_thread(go)
        self._forget(dir)
        await unmount_and_remove(self.host.mounter, dir)


class PortworxProvisioner:
    provisioner = "kubernetes.io/portworx-volume"
    source_key = "portworxVolume"

    async def _endpoint(self, client) -> str:
        """The provisioner reaches Portworx through its kube-system service (portworx_util.go)."""
        if os.environ.get("AMDKUBE_PORTWORX_ENDPOINT") or client is None:
            return portworx_endpoint()
        svc = await client.get_or_none("services", "portworx-service", "kube-system")
        if svc is None or not (svc.get("spec") or {}).get("clusterIP"):
            raise VolumeError("portworx: service kube-system/portworx-service not found")
        return f"http://{svc['spec']['clusterIP']}:9001"

    async def aprovision(self, client, name, gib, params, tags, pvc_name):
        p = {k.lower(): v for k, v in params.items()}
        spec = {"format": p.get("fs", "ext4"), "ha_level": int(p.get("repl", 1)),
                "block_size": int(p.get("block_size", 32)) * 1024, "shared": str(p.get("shared", "false")).lower() == "true"}
        px = PortworxClient(await self._endpoint(client))
        vid = await asyncio.to_thread(px.create, name, gib * GIB, spec, {**tags, "pvc": pvc_name})
        return {"volumeID": vid, "fsType": spec["format"]}, {}

    async def adelete(self, client, src):
        px = PortworxClient(await self._endpoint(client))
        await asyncio.to_thread(px.delete, src["volumeID"])


# ------------------------------------------------------------------------------ scaleio
class ScaleIOClient:
    def __init__(self, gateway: str, user: str, password: str, verify: bool = True, http=None):
        self.base, self.http = gateway.rstrip("/"), http or _http()
        self.http.verify = verify
        r = self.http.get(self.base + "/login", auth=(user, password), timeout=30)
        _raise(r, "scaleio login")
        self.auth = (user, r.json() if r.headers.get("Content-Type", "").startswith("application/json") else r.text.strip('"'))

    def call(self, method, path, body=None, ok404=False):
        r = self.http.request(method, self.base + path, json=body, auth=self.auth, timeout=60)
        if ok404 and r.status_code in (404, 500) and "Could not find" in r.text:
            return None
        _raise(r, f"scaleio {method} {path}")
        return r.json() if r.content else {}

    def system_id(self, name: str) -> str:
        for s in self.call("GET", "/types/System/instances"):
            if not name or s.get("name") == name or s.get("id") == name:
                return s["id"]
        raise VolumeError(f"scaleio: system {name!r} not found")

    def pool_id(self, system: str, domain: str, pool: str) -> str:
        pds = self.call("GET", f"/instances/System::{self.system_id(system)}/relationships/ProtectionDomain")
        pd = next((d for d in pds if d.get("name") == domain), None)
        if pd is None:
            raise VolumeError(f"scaleio: protection domain {domain!r} not found")
        sps = self.call("GET", f"/instances/ProtectionDomain::{pd['id']}/relationships/StoragePool")
        sp = next((s for s in sps if s.get("name") == pool), None)
        if sp is None:
            raise VolumeError(f"scaleio: storage pool {pool!r} not found in {domain!r}")
        return sp["id"]

    def volume_id(self, name: str) -> str | None:
        return self.call("POST", "/types/Volume/instances/action/queryIdByKey", {"name": name}, ok404=True)

    def volume(self, vid: str) -> dict:
        return self.call("GET", f"/instances/Volume::{vid}")

    def sdc_id(self, guid: str) -> str:
        for s in self.call("GET", "/types/Sdc/instances"):
            if s.get("sdcGuid", "").lower() == guid.lower():
                return s["id"]
        raise VolumeError(f"scaleio: no SDC with GUID {guid}")

    def map(self, vid: str, sdc: str, multiple: bool):
        self.call("POST", f"/instances/Volume::{vid}/action/addMappedSdc",
                  {"sdcId": sdc, "allowMultipleMappings": "TRUE" if multiple else "FALSE"})

    def unmap(self, vid: str, sdc: str):
        self.call("POST", f"/instances/Volume::{vid}/action/removeMappedSdc", {"sdcId": sdc})

    def create(self, name: str, kb: int, pool_id: str, thin: bool) -> str:
        return self.call("POST", "/types/Volume/instances", {"name": name, "volumeSizeInKb": str(kb), "storagePoolId": pool_id,
                                                            "volumeType": "ThinProvisioned" if thin else "ThickProvisioned"})["id"]

    def delete(self, vid: str):
        self.call("POST", f"/instances/Volume::{vid}/action/removeVolume", {"removeMode": "ONLY_ME"})


async def _scaleio_client(client, src_or_params: dict, ns: str) -> ScaleIOClient:
    ref = src_or_params.get("secretRef") or {}
    name = ref.get("name") if isinstance(ref, dict) else ref
    sec = await _secret_data(client, (ref.get("namespace") if isinstance(ref, dict) else None) or ns, name or "")
    if not sec.get("username"):
        raise VolumeError("scaleio: the secretRef must hold username and password")
    ssl = str(src_or_params.get("sslEnabled", "false")).lower() == "true"
    return await asyncio.to_thread(ScaleIOClient, src_or_params["gateway"], sec["username"], sec.get("password", ""), ssl)


class ScaleIOPlugin(_Vendor):
    name = "kubernetes.io/scaleio"
    source_key = "scaleIO"
    sdc_root = "/opt/emc/scaleio/sdc/bin"
    attach_timeout = 30.0

    def volume_name(self, spec) -> str:
        return spec.source("scaleIO").get("volumeName", "")

    async def _sdc_guid(self) -> str:
        if self.host.client is not None:
            node = await self.host.client.get_or_none("nodes", self.host.node_name)
            g = (((node or {}).get("metadata") or {}).get("labels") or {}).get("scaleio.sdcGuid")
            if g:
                return g
        rc, out = await self.host.run([os.path.join(self.sdc_root, "drv_cfg"), "--query_guid"])
        if rc != 0 or not out.strip():
            raise VolumeError(f"scaleio: cannot find this node's SDC GUID (drv_cfg: {out.strip()})")
        return out.strip()

    async def set_up(self, spec, pod, dir, device_mount_path=None, fs_group=None):
        src = spec.source("scaleIO")
        ns = ((pod or {}).get("metadata") or {}).get("namespace") or "default"
        sio = await _scaleio_client(self.host.client, src, ns)
        guid = await self._sdc_guid()
        ro = spec.source_read_only("scaleIO")

        def attach() -> str:
            vid = sio.volume_id(src.get("volumeName", ""))
            if not vid:
                raise VolumeError(f"scaleio volume {src.get('volumeName')!r} not found")
            sdc = sio.sdc_id(guid)
            if sdc not in {x.get("sdcId") for x in sio.volume(vid).get("mappedSdcInfo") or []}:
                sio.map(vid, sdc, multiple=ro)
            return vid
        vid = await asyncio.to_thread(attach)
        pat = os.path.join(self.host.dev_root, "dev/disk/by-id", f"emc-vol-*-{vid}")
        end = time.monotonic() + self.attach_timeout
        while not glob.glob(pat):
            if time.monotonic() > end:
                raise VolumeError(f"scaleio volume {vid}: device did not appear ({pat})")
            await asyncio.sleep(min(self.host.attach_poll, 0.5))
        dev = sorted(glob.glob(pat))[0]
        gp = self.global_path(src.get("volumeName", vid))
        await self._mount_global(dev, gp, src.get("fsType") or "xfs", ro)
        await bind_mount(self.host.mounter, gp, dir, ro)
        self._record(dir, {"global": gp, "vid": vid, "guid": guid, "ns": ns,
                           "src": {k: src.get(k) for k in ("gateway", "secretRef", "sslEnabled")}})
        return dir

    async def release(self, rec):
        sio = await _scaleio_client(self.host.client, rec["src"], rec["ns"])
        await asyncio.to_thread(lambda: sio.unmap(rec["vid"], sio.sdc_id(rec["guid"])))


class ScaleIOProvisioner:
    provisioner = "kubernetes.io/scaleio"
    source_key = "scaleIO"

    async def aprovision(self, client, name, gib, params, tags, pvc_name):
        p = dict(params)
        for k in ("gateway", "system", "protectionDomain", "storagePool", "secretRef"):
            if not p.get(k):
                raise VolumeError(f"scaleio storage class: parameter {k} is required")
        sio = await _scaleio_client(client, p, p.get("secretNamespace", "default"))
        gib8 = -(-gib // 8) * 8                  # ScaleIO allocates in 8 GiB units
        thin = p.get("storageMode", "ThinProvisioned") == "ThinProvisioned"
        vname = f"k8svol-{name[-20:]}"

        def go():
            return sio.create(vname, gib8 * 1024 * 1024, sio.pool_id(p["system"], p["protectionDomain"], p["storagePool"]), thin)
        await asyncio.to_thread(go)
        return {"gateway": p["gateway"], "system": p["system"], "protectionDomain": p["protectionDomain"],
                "storagePool": p["storagePool"], "storageMode": p.get("storageMode", "ThinProvisioned"),
                "secretRef": {"name": p["secretRef"], "namespace": p.get("secretNamespace", "default")},
                "sslEnabled": str(p.get("sslEnabled", "false")).lower() == "true", "volumeName": vname,
                "fsType": p.get("fsType", "xfs")}, {}

    async def adelete(self, client, src):
        sio = await _scaleio_client(client, src, "default")

        def go():
            vid = sio.volume_id(src["volumeName"])
            if vid:
                sio.delete(vid)
        await asyncio.to_thread(go)


def plugins() -> list[VolumePlugin]:
    return [FlockerPlugin(), StorageOSPlugin(), PortworxPlugin(), ScaleIOPlugin()]


def provisioners() -> list:
    return [FlockerProvisioner(), StorageOSProvisioner(), PortworxProvisioner(), ScaleIOProvisioner()]
