"""A small in-memory vCenter speaking the vim25 SOAP subset the vsphere provider uses:
RetrieveServiceContent, Login (session cookie checked on every later call), FindByInventoryPath,
FindByUuid, RetrievePropertiesEx (VM guest.net / config.uuid / runtime.powerState /
config.hardware.device, Task info), ReconfigVM_Task (add/remove VirtualDisk), MakeDirectory,
CreateVirtualDisk_Task, DeleteVirtualDisk_Task, QueryVirtualDiskUuid. Tasks are running on the
first poll and succeed on the next. Shapes follow the public vSphere Web Services API; no
vCenter exists offline."""
from __future__ import annotations

import itertools
import threading
import uuid
import xml.etree.ElementTree as ET
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from xml.sax.saxutils import escape

from amdkube.cloudprovider.vsphere import SOAP_NS, MoRef, _xml, as_list, parse


class FakeVCenter:
    USER, PASSWORD = "k8s@vsphere.local", "vc-pw"

    def __init__(self, dc="gpu-dc", folder="kubernetes"):
        self.dc, self.folder = dc, folder
        self.vms: dict[str, dict] = {}            # moref id -> vm
        self.disks: dict[str, str] = {}           # "[ds] path" -> uuid
        self.dirs: set[str] = set()
        self.tasks: dict[str, dict] = {}
        self.sessions: set[str] = set()
        self.logins = 0
        self._n = itertools.count(1)
        self.lock = threading.RLock()
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.port = self.httpd.server_address[1]

    def add_vm(self, name, nets, power="poweredOn", ctrl="ParaVirtualSCSIController"):
        mid = f"vm-{next(self._n)}"
        self.vms[mid] = {"name": name, "uuid": str(uuid.uuid4()).upper(), "power": power, "nets": nets,
                         "devices": [{"@type": ctrl, "key": "1000", "busNumber": "0"},
                                     {"@type": "VirtualDisk", "key": "2000", "controllerKey": "1000", "unitNumber": "0",
                                      "backing": {"@type": "VirtualDiskFlatVer2BackingInfo", "fileName": f"[ds1] {name}/{name}.vmdk"}}]}
        return mid

    def config(self, **extra):
        txt = (f'[Global]\nuser = {self.USER}\npassword = {self.PASSWORD}\nport = {self.port}\ninsecure-flag = 1\nscheme = http\n'
               f'[VirtualCenter "127.0.0.1"]\n[Workspace]\nserver = 127.0.0.1\ndatacenter = {self.dc}\nfolder = {self.folder}\n'
               f"default-datastore = ds1\n")
        for sec, kv in extra.items():
            txt += f"[{sec}]\n" + "".join(f"{k} = {v}\n" for k, v in kv.items())
        return txt

    def start(self):
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    # ------------------------------------------------------------------ SOAP
    def _handler(self):
        vc = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                req = ET.fromstring(self.rfile.read(int(self.headers.get("Content-Length") or 0)))
                op_el = req.find(f"{{{SOAP_NS}}}Body")[0]
                op = op_el.tag.rsplit("}", 1)[-1]
                args = {}
                for k in op_el:
                    args.setdefault(k.tag.rsplit("}", 1)[-1], []).append(parse(k))
                args = {k: v[0] if len(v) == 1 else v for k, v in args.items()}
                cookie = self.headers.get("Cookie", "")
                headers = {}
                with vc.lock:
                    if op not in ("RetrieveServiceContent", "Login") and not any(
                            c.strip().startswith("vmware_soap_session=") and c.split("=", 1)[1].strip('"') in vc.sessions
                            for c in cookie.split(";")):
                        out = vc._fault("NotAuthenticated", "The session is not authenticated.")
                    else:
                        try:
                            out = getattr(vc, "op_" + op)(args, headers)
                        except KeyError as e:
                            out = vc._fault("ManagedObjectNotFound", f"object {e} not found")
                body = ('<?xml version="1.0" encoding="UTF-8"?><soapenv:Envelope xmlns:soapenv="http://schemas.xmlsoap.org/soap/envelope/" '
                        'xmlns:xsi="http://www.w3.org/2001/XMLSchema-instance"><soapenv:Body>'
                        + (out if out.startswith("<soapenv:Fault") else f'<{op}Response xmlns="urn:vim25">{out}</{op}Response>')
                        + "</soapenv:Body></soapenv:Envelope>").encode()
                self.send_response(500 if b"soapenv:Fault" in body else 200)
                self.send_header("Content-Type", "text/xml")
                for k, v in headers.items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)
        return H

    @staticmethod
    def _fault(kind, msg):
        return (f"<soapenv:Fault><faultcode>ServerFaultCode</faultcode><faultstring>{escape(msg)}</faultstring>"
                f'<detail><{kind}Fault xmlns="urn:vim25" xsi:type="{kind}"/></detail></soapenv:Fault>')

    def _task(self, result=None, error=None):
        tid = f"task-{next(self._n)}"
        self.tasks[tid] = {"polls": 0, "result": result, "error": error}
        return _xml("returnval", MoRef("Task", tid))

    def op_RetrieveServiceContent(self, a, h):
        refs = {"rootFolder": ("Folder", "group-d1"), "propertyCollector": ("PropertyCollector", "propertyCollector"),
                "searchIndex": ("SearchIndex", "SearchIndex"), "sessionManager": ("SessionManager", "SessionManager"),
                "fileManager": ("FileManager", "FileManager"), "virtualDiskManager": ("VirtualDiskManager", "virtualDiskManager")}
        return "<returnval>" + "".join(_xml(k, MoRef(*v)) for k, v in refs.items()) + "</returnval>"

    def op_Login(self, a, h):
        if a.get("userName") != self.USER or a.get("password") != self.PASSWORD:
            return self._fault("InvalidLogin", "Cannot complete login due to an incorrect user name or password.")
        sid = uuid.uuid4().hex
        self.sessions.add(sid)
        self.logins += 1
        h["Set-Cookie"] = f'vmware_soap_session="{sid}"; Path=/; HttpOnly'
        return f"<returnval><key>{sid}</key><userName>{self.USER}</userName></returnval>"

    def op_FindByInventoryPath(self, a, h):
        path = a["inventoryPath"]
        if path == f"/{self.dc}":
            return _xml("returnval", MoRef("Datacenter", "datacenter-2"))
        for mid, vm in self.vms.items():
            if path == f"/{self.dc}/vm/{self.folder}/{vm['name']}":
                return _xml("returnval", MoRef("VirtualMachine", mid))
        return ""

    def op_FindByUuid(self, a, h):
        for mid, vm in self.vms.items():
            if vm["uuid"].lower() == a["uuid"].lower():
                return _xml("returnval", MoRef("VirtualMachine", mid))
        return ""

    def op_RetrievePropertiesEx(self, a, h):
        spec = a["specSet"]
        obj = spec["objectSet"]["obj"]
        paths = as_list(spec["propSet"]["pathSet"])
        props = []
        if obj.type == "Task":
            t = self.tasks[obj.value]
            t["polls"] += 1
            if t["polls"] < 2:
                info = {"@type": "TaskInfo", "key": obj.value, "state": "running"}
            elif t["error"]:
                info = {"@type": "TaskInfo", "key": obj.value, "state": "error",
                        "error": {"@type": "LocalizedMethodFault", "localizedMessage": t["error"]}}
            else:
                info = {"@type": "TaskInfo", "key": obj.value, "state": "success"}
            props.append(("info", info))
        else:
            vm = self.vms[obj.value]
            for p in paths:
                if p == "guest.net":
                    props.append((p, {"@type": "ArrayOfGuestNicInfo", "GuestNicInfo": [
                        {"@type": "GuestNicInfo", "network": n, "ipAddress": ips} for n, ips in vm["nets"]]}))
                elif p == "config.uuid":
                    props.append((p, vm["uuid"]))
                elif p == "runtime.powerState":
                    props.append((p, vm["power"]))
                elif p == "config.hardware.device":
                    props.append((p, {"@type": "ArrayOfVirtualDevice", "VirtualDevice": vm["devices"]}))
        return ("<returnval><objects>" + _xml("obj", obj) + "".join(_xml("propSet", {"name": n, "val": v}) for n, v in props)
                + "</objects></returnval>")

    def op_ReconfigVM_Task(self, a, h):
        vm = self.vms[a["_this"].value]
        for ch in as_list(a["spec"].get("deviceChange")):
            dev = ch["device"]
            path = dev["backing"]["fileName"]
            if ch["operation"] == "add":
                if path not in self.disks:
                    return self._task(error=f"File {path} was not found")
                if any(d.get("controllerKey") == dev["controllerKey"] and d.get("unitNumber") == dev["unitNumber"] for d in vm["devices"]):
                    return self._task(error="unit in use")
                vm["devices"].append({"@type": "VirtualDisk", "key": str(2000 + len(vm["devices"])), "controllerKey": dev["controllerKey"],
                                      "unitNumber": dev["unitNumber"], "backing": {"@type": "VirtualDiskFlatVer2BackingInfo",
                                                                                   "fileName": path, "diskMode": dev["backing"]["diskMode"]}})
            else:
                vm["devices"] = [d for d in vm["devices"] if d.get("key") != dev["key"]]
        return self._task()

    def op_MakeDirectory(self, a, h):
        if a["name"] in self.dirs:
            return self._fault("FileAlreadyExists", f"Cannot complete the operation because the file or folder {a['name']} already exists")
        self.dirs.add(a["name"])
        return ""

    def op_CreateVirtualDisk_Task(self, a, h):
        ds, rest = a["name"][1:].split("] ", 1)
        if f"[{ds}] {rest.rsplit('/', 1)[0]}" not in self.dirs:
            return self._task(error="parent directory missing")
        self.disks[a["name"]] = "60 00 C2 9" + uuid.uuid4().hex[:7] + " " + uuid.uuid4().hex[:16]
        self.last_spec = a["spec"]
        return self._task(result=a["name"])

    def op_DeleteVirtualDisk_Task(self, a, h):
        if a["name"] not in self.disks:
            return self._fault("FileNotFound", f"File {a['name']} was not found")
        if any(d.get("backing", {}).get("fileName") == a["name"] for vm in self.vms.values() for d in vm["devices"]):
            return self._task(error="disk is attached")
        del self.disks[a["name"]]
        return self._task()

    def op_QueryVirtualDiskUuid(self, a, h):
        if a["name"] not in self.disks:
            return self._fault("FileNotFound", f"File {a['name']} was not found")
        return f"<returnval>{self.disks[a['name']]}</returnval>"
