"""VMware vSphere cloud provider and the disks behind the vsphereVolume plugin (reference:
pkg/cloudprovider/providers/vsphere — vsphere.go, vsphere_util.go, vclib/{connection,
datacenter,virtualmachine,diskmanagers}.go; pkg/volume/vsphere_volume).

vCenter speaks the vim25 SOAP API at `https://<server>/sdk`. This client is a small SOAP
codec over `requests` (no govmomi): managed-object references travel as `<x type="T">id</x>`,
polymorphic data objects carry `xsi:type`, and the session is the `vmware_soap_session`
cookie from `SessionManager.Login` (re-login once when a call faults NotAuthenticated).

  * Instances: the node's VM is `<datacenter>/vm/<folder>/<node name>`
    (`SearchIndex.FindByInventoryPath`); its IPv4 addresses on the public network
    (`guest.net`, `[Network] public-network`, every network when unset) are both ExternalIP and
    InternalIP, as vsphere.go reports them. The instance ID is the VM's BIOS UUID
    (`config.uuid`, providerID `vsphere://<uuid>`) and only powered-on VMs exist.
    Existence by provider ID is `SearchIndex.FindByUuid`.
  * Volumes: `[datastore] kubevols/<name>.vmdk` disks. Attach is `ReconfigVM_Task` adding a
    VirtualDisk (independent_persistent, FlatVer2 backing) at the first free unit of the VM's
    SCSI controller; the guest sees it as `/dev/disk/by-id/wwn-0x<disk uuid>`
    (`VirtualDiskManager.QueryVirtualDiskUuid`). Detach removes the device whose backing file
    is the disk; create is `FileManager.MakeDirectory` + `VirtualDiskManager.CreateVirtualDisk_Task`
    (thin / zeroedthick / eagerzeroedthick, lsiLogic adapter), delete is `DeleteVirtualDisk_Task`.
    Tasks are polled through `PropertyCollector.RetrievePropertiesEx` on `info`.
Config (vsphere.conf INI): `[Global] user, password, port, insecure-flag, vm-uuid`,
`[VirtualCenter "<server>"]` (or `[Workspace] server`), `[Workspace] datacenter, folder,
default-datastore`, `[Disk] scsicontrollertype`, `[Network] public-network`.
"""
from __future__ import annotations

import configparser
import ipaddress
import json
import threading
import time
import xml.etree.ElementTree as ET
from typing import NamedTuple
from xml.sax.saxutils import escape

from . import Interface, off_loop

PROVIDER = "vsphere"
VOLUME_PROVISIONER = "kubernetes.io/vsphere-volume"
XSI = "http://www.w3.org/2001/XMLSchema-instance"
SOAP_NS = "http://schemas.xmlsoap.org/soap/envelope/"
SCSI_TYPES = ("ParaVirtualSCSIController", "VirtualLsiLogicController", "VirtualLsiLogicSASController", "VirtualBusLogicController")


class MoRef(NamedTuple):
    type: str
    value: str


class VSphereError(RuntimeError):
    def __init__(self, fault: str, msg: str):
        super().__init__(f"vSphere {fault}: {msg}")
        self.fault = fault


def _xml(name: str, v) -> str:
    if v is None:
        return ""
    if isinstance(v, MoRef):
        return f'<{name} type="{v.type}">{escape(v.value)}</{name}>'
    if isinstance(v, list):
        return "".join(_xml(name, i) for i in v)
    if isinstance(v, dict):
        t = v.get("@type")
        head = f'<{name} xsi:type="{t}">' if t else f"<{name}>"
        return head + "".join(_xml(k, x) for k, x in v.items() if k != "@type") + f"</{name}>"
    if isinstance(v, bool):
        v = "true" if v else "false"
    return f"<{name}>{escape(str(v))}</{name}>"


def envelope(op: str, this: MoRef, args: dict) -> str:
    return ('<?xml version="1.0" encoding="UTF-8"?><soapenv:Envelope xmlns:soapenv="http://schemas.xmlsoap.org/soap/envelope/" '
            'xmlns:xsd="http://www.w3.org/2001/XMLSchema" xmlns:xsi="http://www.w3.org/2001/XMLSchema-instance"><soapenv:Body>'
            f'<{op} xmlns="urn:vim25">{_xml("_this", this)}' + "".join(_xml(k, v) for k, v in args.items())
            + f"</{op}></soapenv:Body></soapenv:Envelope>")


def parse(el):
    """An element → text, MoRef (a leaf with a `type` attribute) or {tag: value} with repeated
    tags as lists and the xsi:type under '@type'."""
    kids = list(el)
    if not kids:
        if el.get("type") is not None:
            return MoRef(el.get("type"), (el.text or "").strip())
        return el.text or ""
    out = {}
    t = el.get(f"{{{XSI}}}type")
    if t:
        out["@type"] = t
    for k in kids:
        tag = k.tag.rsplit("}", 1)[-1]
        val = parse(k)
        if tag in out:
            out[tag] = out[tag] if isinstance(out[tag], list) else [out[tag]]
            out[tag].append(val)
        else:
            out[tag] = val
    return out


def as_list(v) -> list:
    if v is None or v == "":
        return []
    return v if isinstance(v, list) else [v]


def parse_config(cfg) -> dict:
    if isinstance(cfg, str):
        try:
            cfg = json.loads(cfg)
        except ValueError:
            cp = configparser.ConfigParser(interpolation=None, strict=False)
            cp.read_string(cfg)
            cfg = {s: dict(cp.items(s)) for s in cp.sections()}
    out = {"global": {}, "workspace": {}, "disk": {}, "network": {}, "vcenters": {}}
    for sec, vals in (cfg or {}).items():
        low = sec.lower()
        if low.startswith("virtualcenter"):
            out["vcenters"][sec.split(None, 1)[1].strip('"') if " " in sec else vals.get("server", "")] = {
                str(k).lower(): v for k, v in vals.items()}
        elif low in out:
            out[low] = {str(k).lower(): v for k, v in (vals or {}).items()}
    return out


class Client:
    """One vCenter session."""

    def __init__(self, url: str, user: str, password: str, http):
        self.url, self.user, self.password, self.http = url, user, password, http
        self.lock = threading.Lock()
        self.sc: dict | None = None
        self.logged_in = False

    def _post(self, op: str, this: MoRef, args: dict):
        r = self.http.post(self.url, data=envelope(op, this, args).encode(), timeout=60,
                           headers={"Content-Type": "text/xml; charset=utf-8", "SOAPAction": "urn:vim25/6.5"})
        body = ET.fromstring(r.content).find(f"{{{SOAP_NS}}}Body")
        fault = body.find(f"{{{SOAP_NS}}}Fault") if body is not None else None
        if fault is not None:
            detail = fault.find("detail")
            kind = ""
            if detail is not None and len(detail):
                kind = (detail[0].get(f"{{{XSI}}}type") or detail[0].tag.rsplit("}", 1)[-1]).removesuffix("Fault")
            raise VSphereError(kind or "Fault", fault.findtext("faultstring") or "")
        if r.status_code >= 400 or body is None or not len(body):
            raise VSphereError("HTTP", f"{op}: HTTP {r.status_code}")
        resp = body[0]
        rv = [parse(x) for x in resp if x.tag.rsplit("}", 1)[-1] == "returnval"]
        return rv[0] if len(rv) == 1 else (rv or None)

    def content(self) -> dict:
        if self.sc is None:
            self.sc = self._post("RetrieveServiceContent", MoRef("ServiceInstance", "ServiceInstance"), {})
        return self.sc

    def login(self):
        self._post("Login", self.content()["sessionManager"], {"userName": self.user, "password": self.password})
        self.logged_in = True

    def call(self, op: str, this: MoRef, **args):
        with self.lock:
            if not self.logged_in:
                self.login()
        try:
            return self._post(op, this, args)
        except VSphereError as e:
            if e.fault != "NotAuthenticated":
                raise
            with self.lock:
                self.login()
            return self._post(op, this, args)

    def props(self, obj: MoRef, paths: list[str]) -> dict:
        spec = {"propSet": {"type": obj.type, "pathSet": paths}, "objectSet": {"obj": obj, "skip": False}}
        rv = self.call("RetrievePropertiesEx", self.content()["propertyCollector"], specSet=spec, options={})
        out = {}
        for o in as_list((rv or {}).get("objects")):
            for p in as_list(o.get("propSet")):
                out[p["name"]] = p.get("val")
        return out

    def wait(self, task: MoRef, timeout: float = 300) -> dict:
        end, delay = time.monotonic() + timeout, 0.05
        while True:
            info = self.props(task, ["info"]).get("info") or {}
            if info.get("state") == "success":
                return info
            if info.get("state") == "error":
                err = info.get("error") or {}
                raise VSphereError("TaskError", err.get("localizedMessage") or str(err))
            if time.monotonic() > end:
                raise TimeoutError(f"vSphere task {task.value} did not finish in {timeout}s")
            time.sleep(delay)
            delay = min(delay * 2, 2.0)


class Instances:
    def __init__(self, vs: "VSphere"):
        self.vs = vs

    def vm(self, name: str) -> MoRef:
        path = "/".join(p for p in (self.vs.datacenter, "vm", self.vs.folder.strip("/"), name) if p)
        ref = self.vs.client.call("FindByInventoryPath", self.vs.client.content()["searchIndex"], inventoryPath="/" + path)
        if not isinstance(ref, MoRef):
            raise LookupError(f"no VM found for node {name} ({path})")
        return ref

    def _active(self, name: str) -> tuple[MoRef, dict]:
        ref = self.vm(name)
        p = self.vs.client.props(ref, ["config.uuid", "runtime.powerState", "guest.net"])
        if p.get("runtime.powerState") != "poweredOn":
            raise LookupError(f"VM {name} is {p.get('runtime.powerState') or 'not powered on'}")
        return ref, p

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        net = self.vs.public_network
        out = []
        for nic in as_list((self.vm_props(name).get("guest.net") or {}).get("GuestNicInfo")):
            if net and nic.get("network") != net:
                continue
            for ip in as_list(nic.get("ipAddress")):
                try:
                    if ipaddress.ip_address(ip).version != 4:
                        continue
                except ValueError:
                    continue
                for t in ("ExternalIP", "InternalIP"):
                    if {"type": t, "address": ip} not in out:
                        out.append({"type": t, "address": ip})
        return out

    def vm_props(self, name: str) -> dict:
        return self.vs.client.props(self.vm(name), ["guest.net"])

    @off_loop
    def instance_exists(self, name: str) -> bool:
        try:
            self._active(name)
            return True
        except LookupError:
            return False

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        uuid = pid.split("://", 1)[-1].strip("/")
        dc = self.vs.datacenter_ref()
        ref = self.vs.client.call("FindByUuid", self.vs.client.content()["searchIndex"], datacenter=dc, uuid=uuid, vmSearch=True)
        return isinstance(ref, MoRef)

    @off_loop
    def instance_id(self, name: str) -> str:
        return self._active(name)[1]["config.uuid"].lower()

    @off_loop
    def instance_type(self, name: str) -> str:
        return ""


def disk_path(datastore: str, name: str) -> str:
    return f"[{datastore}] kubevols/{name}.vmdk"


class Volumes:
    provisioner = VOLUME_PROVISIONER
    source_key = "vsphereVolume"

    def __init__(self, vs: "VSphere"):
        self.vs = vs

    @property
    def c(self) -> Client:
        return self.vs.client

    def _devices(self, vm: MoRef) -> list[dict]:
        return as_list((self.c.props(vm, ["config.hardware.device"]).get("config.hardware.device") or {}).get("VirtualDevice"))

    def _disk_of(self, devices: list[dict], path: str) -> dict | None:
        return next((d for d in devices if d.get("@type") == "VirtualDisk" and (d.get("backing") or {}).get("fileName") == path), None)

    def disk_uuid(self, path: str) -> str:
        u = self.c.call("QueryVirtualDiskUuid", self.c.content()["virtualDiskManager"], name=path, datacenter=self.vs.datacenter_ref())
        return str(u).replace(" ", "").replace("-", "").lower()

    def attach(self, node: str, path: str) -> str:
        vm = self.vs.instances_.vm(node)
        devices = self._devices(vm)
        if self._disk_of(devices, path) is None:
            want = self.vs.scsi_type
            ctrls = [d for d in devices if d.get("@type") in SCSI_TYPES]
            ctrl = next((d for d in ctrls if d.get("@type") == want), None) or (ctrls[0] if ctrls else None)
            if ctrl is None:
                raise VSphereError("NoController", f"VM {node} has no SCSI controller")
            used = {int(d.get("unitNumber", -1)) for d in devices if str(d.get("controllerKey")) == str(ctrl["key"])}
            unit = next((u for u in range(16) if u != 7 and u not in used), None)
            if unit is None:
                raise VSphereError("NoFreeUnit", f"SCSI controller {ctrl['key']} of VM {node} is full")
            spec = {"@type": "VirtualMachineConfigSpec", "deviceChange": {
                "@type": "VirtualDeviceConfigSpec", "operation": "add",
                "device": {"@type": "VirtualDisk", "key": -100, "backing": {
                    "@type": "VirtualDiskFlatVer2BackingInfo", "fileName": path, "diskMode": "independent_persistent"},
                    "controllerKey": ctrl["key"], "unitNumber": unit}}}
            self.c.wait(self.c.call("ReconfigVM_Task", vm, spec=spec))
        return self.device_candidates(path)[0]

    def detach(self, node: str, path: str):
        try:
            vm = self.vs.instances_.vm(node)
        except LookupError:
            return
        d = self._disk_of(self._devices(vm), path)
        if d is None:
            return
        spec = {"@type": "VirtualMachineConfigSpec", "deviceChange": {
            "@type": "VirtualDeviceConfigSpec", "operation": "remove",
            "device": {"@type": "VirtualDisk", "key": d["key"], "backing": d.get("backing"),
                       "controllerKey": d.get("controllerKey"), "unitNumber": d.get("unitNumber")}}}
        self.c.wait(self.c.call("ReconfigVM_Task", vm, spec=spec))

    def is_attached(self, node: str, path: str) -> bool:
        try:
            return self._disk_of(self._devices(self.vs.instances_.vm(node)), path) is not None
        except LookupError:
            return False

    def device_candidates(self, path: str, device_path: str = "") -> list[str]:
        """The attach result already names the disk's WWN path; only without one is vCenter asked."""
        if device_path.startswith("/dev/disk/by-id/wwn-0x"):
            return [device_path]
        return [f"/dev/disk/by-id/wwn-0x{self.disk_uuid(path)}"]

    def create(self, name: str, gib: int, disk_format: str = "thin", datastore: str = "") -> str:
        ds = datastore or self.vs.default_datastore
        if disk_format not in ("thin", "zeroedthick", "eagerzeroedthick"):
            raise ValueError(f"invalid vSphere diskformat {disk_format!r}: thin, zeroedthick or eagerzeroedthick")
        dc = self.vs.datacenter_ref()
        try:
            self.c.call("MakeDirectory", self.c.content()["fileManager"], name=f"[{ds}] kubevols", datacenter=dc,
                        createParentDirectories=True)
        except VSphereError as e:
            if e.fault != "FileAlreadyExists":
                raise
        path = disk_path(ds, name)
        spec = {"@type": "FileBackedVirtualDiskSpec", "diskType": disk_format, "adapterType": "lsiLogic",
                "capacityKb": gib * 1024 * 1024}
        self.c.wait(self.c.call("CreateVirtualDisk_Task", self.c.content()["virtualDiskManager"], name=path, datacenter=dc, spec=spec))
        return path

    def delete(self, path: str):
        try:
            self.c.wait(self.c.call("DeleteVirtualDisk_Task", self.c.content()["virtualDiskManager"], name=path,
                                    datacenter=self.vs.datacenter_ref()))
        except VSphereError as e:
            if e.fault not in ("FileNotFound", "NotFound"):
                raise

    def provision(self, name: str, gib: int, params: dict, tags: dict, pvc_name: str) -> tuple[dict, dict]:
        p = {str(k).lower(): v for k, v in params.items()}
        path = self.create(f"kubernetes-dynamic-{name}", gib, p.get("diskformat", "thin"), p.get("datastore", ""))
        return {"volumePath": path, "fsType": p.get("fstype", "ext4")}, {}

    def delete_source(self, src: dict):
        self.delete(src["volumePath"])


class VSphere(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        cfg = parse_config(config)
        g, ws = cfg["global"], cfg["workspace"]
        server = ws.get("server") or g.get("server") or next(iter(cfg["vcenters"]), "")
        if not server:
            raise ValueError("vsphere: a vCenter server is required ([VirtualCenter \"<server>\"] or [Workspace] server)")
        vc = cfg["vcenters"].get(server, {})
        port = vc.get("port") or g.get("port") or "443"
        scheme = g.get("scheme", "https")
        self.http = session or requests.Session()
        if str(vc.get("insecure-flag") or g.get("insecure-flag") or "").lower() in ("1", "true"):
            self.http.verify = False
        self.client = Client(f"{scheme}://{server}:{port}/sdk", vc.get("user") or g.get("user", ""),
                             vc.get("password") or g.get("password", ""), self.http)
        self.datacenter = ws.get("datacenter") or g.get("datacenter") or (vc.get("datacenters") or g.get("datacenters") or "").split(",")[0].strip()
        if not self.datacenter:
            raise ValueError("vsphere: a datacenter is required ([Workspace] datacenter)")
        self.folder = ws.get("folder") or g.get("working-dir", "")
        self.default_datastore = ws.get("default-datastore") or g.get("datastore", "")
        self.scsi_type = {"pvscsi": "ParaVirtualSCSIController", "lsilogic-sas": "VirtualLsiLogicSASController",
                          "lsilogic": "VirtualLsiLogicController", "buslogic": "VirtualBusLogicController"}.get(
            (cfg["disk"].get("scsicontrollertype") or "pvscsi").lower(), "ParaVirtualSCSIController")
        self.public_network = cfg["network"].get("public-network", "")
        self._dc: MoRef | None = None
        self.instances_ = Instances(self)
        self.volumes_ = Volumes(self)

    def datacenter_ref(self) -> MoRef:
        if self._dc is None:
            ref = self.client.call("FindByInventoryPath", self.client.content()["searchIndex"], inventoryPath="/" + self.datacenter)
            if not isinstance(ref, MoRef):
                raise LookupError(f"vsphere: datacenter {self.datacenter} not found")
            self._dc = ref
        return self._dc

    def instances(self):
        return self.instances_

    def volumes(self):
        return self.volumes_
