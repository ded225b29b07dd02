"""A small in-memory Azure (Azure AD token endpoint, instance metadata + managed identity,
Resource Manager for VMs, NICs, public IPs, load balancers, NSGs, route tables and managed
disks) for the provider tests. Resources are stored by lower-cased resource ID; PUTs on VMs and
disks answer with an Azure-AsyncOperation to poll, as the real service does. Bearer tokens are
checked on every ARM call."""
from __future__ import annotations

import itertools
import json
import re
import threading
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlsplit


class FakeAzure:
    def __init__(self, sub="sub-1", rg="mi355x-rg", location="eastus"):
        self.sub, self.rg, self.location = sub, rg, location
        self.lock = threading.RLock()
        self.res: dict[str, dict] = {}
        self.tokens: set[str] = set()
        self.token_calls = 0
        self.asyncops: dict[str, int] = {}
        self._ip = itertools.count(10)
        self._priv = itertools.count(100)
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"

    def rid(self, provider, kind, name):
        return f"/subscriptions/{self.sub}/resourceGroups/{self.rg}/providers/{provider}/{kind}/{name}"

    def get(self, rid):
        return self.res.get(rid.lower())

    def put(self, rid, obj):
        obj = dict(obj, id=rid, name=rid.rsplit("/", 1)[-1])
        self.res[rid.lower()] = obj
        return obj

    # ------------------------------------------------------------------ fixtures
    def add_vm(self, name, ip, public=None, size="Standard_ND96isr_MI355X_v6", fault_domain=1):
        nic_id = self.rid("Microsoft.Network", "networkInterfaces", f"{name}-nic")
        ipc = {"name": "ipconfig1", "id": nic_id + "/ipConfigurations/ipconfig1",
               "properties": {"primary": True, "privateIPAddress": ip, "loadBalancerBackendAddressPools": []}}
        if public:
            pip = self.put(self.rid("Microsoft.Network", "publicIPAddresses", f"{name}-pip"),
                           {"location": self.location, "properties": {"ipAddress": public}})
            ipc["properties"]["publicIPAddress"] = {"id": pip["id"]}
        self.put(nic_id, {"location": self.location, "properties": {"ipConfigurations": [ipc]}})
        return self.put(self.rid("Microsoft.Compute", "virtualMachines", name), {
            "location": self.location, "_fd": fault_domain,
            "properties": {"hardwareProfile": {"vmSize": size},
                           "networkProfile": {"networkInterfaces": [{"id": nic_id, "properties": {"primary": True}}]},
                           "storageProfile": {"dataDisks": []}}})

    def add_nsg(self, name="k8s-nsg"):
        return self.put(self.rid("Microsoft.Network", "networkSecurityGroups", name),
                        {"location": self.location, "properties": {"securityRules": [
                            {"name": "allow-ssh", "properties": {"priority": 500, "access": "Allow", "direction": "Inbound",
                                                                 "destinationPortRange": "22", "protocol": "Tcp",
                                                                 "sourceAddressPrefix": "*", "destinationAddressPrefix": "*"}}]}})

    def start(self):
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def config(self, **extra):
        return {"tenantId": "tenant-1", "subscriptionId": self.sub, "aadClientId": "client-1", "aadClientSecret": "secret-1",
                "resourceGroup": self.rg, "location": self.location, "vnetName": "k8s-vnet", "subnetName": "k8s-subnet",
                "securityGroupName": "k8s-nsg", "routeTableName": "k8s-routes",
                "resourceManagerEndpoint": self.url + "/", "activeDirectoryEndpoint": self.url + "/aad/",
                "instanceMetadataEndpoint": self.url + "/metadata/", **extra}

    # ------------------------------------------------------------------ HTTP
    def _handler(self):
        az = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=None, headers=None):
                data = json.dumps(body).encode() if body is not None else b""
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                for k, v in (headers or {}).items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def _token(self):
                az.token_calls += 1
                t = uuid.uuid4().hex
                az.tokens.add(t)
                return self._send(200, {"access_token": t, "expires_in": "3599", "token_type": "Bearer"})

            def _do(self, method):
                u = urlsplit(self.path)
                q = {k: v[0] for k, v in parse_qs(u.query).items()}
                n = int(self.headers.get("Content-Length") or 0)
                raw = self.rfile.read(n) if n else b""
                if u.path.startswith("/aad/") and u.path.endswith("/oauth2/token"):
                    form = {k: v[0] for k, v in parse_qs(raw.decode()).items()}
                    if form.get("client_secret") != "secret-1" or form.get("grant_type") != "client_credentials":
                        return self._send(401, {"error": "invalid_client"})
                    return self._token()
                if u.path.startswith("/metadata/"):
                    if self.headers.get("Metadata") != "true":
                        return self._send(400, {"error": "Metadata header required"})
                    if u.path == "/metadata/identity/oauth2/token":
                        return self._token()
                    if u.path == "/metadata/instance/compute":
                        return self._send(200, {"platformFaultDomain": "2", "location": az.location})
                    return self._send(404, {})
                if u.path.startswith("/asyncop/"):
                    return self._send(200, {"status": "Succeeded"})
                if self.headers.get("Authorization", "")[7:] not in az.tokens:
                    return self._send(401, {"error": {"code": "InvalidAuthenticationToken", "message": "bad token"}})
                if "api-version" not in q:
                    return self._send(400, {"error": {"code": "MissingApiVersionParameter", "message": "api-version"}})
                body = json.loads(raw) if raw else None
                with az.lock:
                    code, out, hdrs = az.arm(method, u.path, q, body)
                self._send(code, out, hdrs)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

            def do_PUT(self):
                self._do("PUT")

            def do_DELETE(self):
                self._do("DELETE")
        return H

    @staticmethod
    def _err(code, c, msg):
        return code, {"error": {"code": c, "message": msg}}, {}

    def _async(self):
        op = uuid.uuid4().hex
        return {"Azure-AsyncOperation": f"{self.url}/asyncop/{op}"}

    def arm(self, method, path, q, body):
        key = path.lower()
        mt = re.fullmatch(r"(/subscriptions/[^/]+/resourcegroups/[^/]+/providers/[^/]+/)([^/]+)", key)
        if mt and method == "GET":           # a collection
            pre = key + "/"
            return 200, {"value": [v for k, v in self.res.items() if k.startswith(pre) and k.count("/") == key.count("/") + 1]}, {}
        if method == "GET":
            obj = self.res.get(key)
            if obj is None:
                return self._err(404, "ResourceNotFound", path)
            obj = json.loads(json.dumps(obj))
            if "/virtualmachines/" in key:
                fd = obj.pop("_fd", 0)
                if q.get("$expand") == "instanceView":
                    obj["properties"]["instanceView"] = {"platformFaultDomain": fd}
            return 200, obj, {}
        if method == "DELETE":
            if key not in self.res:
                return self._err(404, "ResourceNotFound", path)
            if "/microsoft.compute/disks/" in key and self.res[key].get("managedBy"):
                return self._err(409, "OperationNotAllowed", "disk attached")
            if "/routetables/" in key and "/routes/" in key:
                t = self.res[key.split("/routes/")[0]]
                t["properties"]["routes"] = [r for r in t["properties"].get("routes") or [] if r["id"].lower() != key]
            del self.res[key]
            return 200, None, {}
        # PUT
        body = dict(body or {})
        if "/virtualmachines/" in key:
            vm = self.res.get(key)
            if vm is None:
                return self._err(404, "ResourceNotFound", path)
            new = (body.get("properties") or {}).get("storageProfile", {}).get("dataDisks")
            if new is not None:
                for d in self.res.values():
                    if d.get("managedBy", "").lower() == key:
                        d["managedBy"], d["properties"]["diskState"] = "", "Unattached"
                for dd in new:
                    disk = self.res.get(dd["managedDisk"]["id"].lower())
                    if disk is None:
                        return self._err(404, "NotFound", f"disk {dd['managedDisk']['id']}")
                    if disk.get("managedBy") and disk["managedBy"].lower() != key:
                        return self._err(409, "AttachDiskWhileBeingDetached", "disk attached elsewhere")
                    disk["managedBy"], disk["properties"]["diskState"] = vm["id"], "Attached"
                vm["properties"]["storageProfile"]["dataDisks"] = new
            return 200, vm, self._async()
        if "/microsoft.compute/disks/" in key:
            body.setdefault("properties", {})["diskState"] = "Unattached"
            body["managedBy"] = ""
            obj = self.put(path, body)
            return 201, obj, self._async()
        if "/publicipaddresses/" in key:
            old = self.res.get(key)
            body.setdefault("properties", {})["ipAddress"] = ((old or {}).get("properties") or {}).get("ipAddress") or f"52.0.0.{next(self._ip)}"
            return 200, self.put(path, body), {}
        if "/loadbalancers/" in key:
            for f in (body.get("properties") or {}).get("frontendIPConfigurations") or []:
                fp = f.setdefault("properties", {})
                f["id"] = f"{path}/frontendIPConfigurations/{f['name']}"
                if fp.get("subnet") and not fp.get("privateIPAddress"):
                    fp["privateIPAddress"] = f"10.240.0.{next(self._priv)}"
            for p in (body.get("properties") or {}).get("backendAddressPools") or []:
                p["id"] = f"{path}/backendAddressPools/{p['name']}"
                members = [ipc["id"] for nic in self.res.values() if "/networkinterfaces/" in nic["id"].lower()
                           for ipc in nic["properties"]["ipConfigurations"]
                           if any(x["id"].lower() == p["id"].lower() for x in ipc["properties"].get("loadBalancerBackendAddressPools") or [])]
                p["properties"] = {"backendIPConfigurations": [{"id": i} for i in members]}
            return 200, self.put(path, body), {}
        if "/networkinterfaces/" in key:
            obj = self.put(path, body)
            for lb in [v for v in self.res.values() if "/loadbalancers/" in v["id"].lower()]:
                for p in (lb.get("properties") or {}).get("backendAddressPools") or []:
                    members = [ipc["id"] for nic in self.res.values() if "/networkinterfaces/" in nic["id"].lower()
                               for ipc in nic["properties"]["ipConfigurations"]
                               if any(x["id"].lower() == p["id"].lower() for x in ipc["properties"].get("loadBalancerBackendAddressPools") or [])]
                    p["properties"] = {"backendIPConfigurations": [{"id": i} for i in members]}
            return 200, obj, {}
        if "/routetables/" in key and "/routes/" in key:
            tkey = key.split("/routes/")[0]
            t = self.res.get(tkey)
            if t is None:
                return self._err(404, "ResourceNotFound", "route table")
            r = self.put(path, body)
            t["properties"]["routes"] = [x for x in t["properties"].get("routes") or [] if x["id"].lower() != key] + [r]
            return 201, r, {}
        if "/routetables/" in key:
            body.setdefault("properties", {}).setdefault("routes", [])
            return 201, self.put(path, body), {}
        return 200, self.put(path, body), {}
