"""A small in-memory Compute Engine (compute/v1 REST: instances, disks, routes, addresses,
firewalls, HTTP health checks, target pools, forwarding rules, zonal/regional/global Operations)
and metadata server for the GCE provider tests. Mutations answer with a RUNNING Operation that
is DONE on the next poll, as the real API does for anything non-trivial; bearer tokens issued
by the metadata server are checked on every call."""
from __future__ import annotations

import itertools
import json
import re
import threading
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlsplit


class FakeGCE:
    def __init__(self, project="mi355x-proj", region="us-central1", zones=("us-central1-a", "us-central1-b")):
        self.project, self.region, self.zones = project, region, list(zones)
        self.lock = threading.RLock()
        self.instances: dict[tuple[str, str], dict] = {}
        self.disks: dict[tuple[str, str], dict] = {}
        self.routes: dict[str, dict] = {}
        self.addresses: dict[str, dict] = {}
        self.firewalls: dict[str, dict] = {}
        self.hcs: dict[str, dict] = {}
        self.pools: dict[str, dict] = {}
        self.rules: dict[str, dict] = {}
        self.ops: dict[str, dict] = {}
        self.tokens: set[str] = set()
        self.token_calls = 0
        self.self_name = None
        self._ip = itertools.count(10)
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"
        self.base = self.url + "/compute/v1/"

    def add_instance(self, name, ip, zone=None, external=None, mtype="a3-mi355x-8g", tags=("gke-node",)):
        zone = zone or self.zones[0]
        nic = {"networkIP": ip, "network": self.base + f"projects/{self.project}/global/networks/default",
               "accessConfigs": [{"natIP": external}] if external else []}
        inst = {"name": name, "zone": self.base + f"projects/{self.project}/zones/{zone}", "status": "RUNNING",
                "machineType": self.base + f"projects/{self.project}/zones/{zone}/machineTypes/{mtype}",
                "networkInterfaces": [nic], "tags": {"items": list(tags)}, "disks": [{"deviceName": "boot", "source": "boot"}]}
        self.instances[(zone, name)] = inst
        if self.self_name is None:
            self.self_name, self.self_zone = name, zone
        return inst

    def start(self):
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def config(self, **extra):
        return {"global": {"project-id": self.project, "network-name": "default", "multizone": "true",
                           "api-endpoint": self.base, "metadata-url": self.url + "/computeMetadata/v1/", **extra}}

    # ------------------------------------------------------------------ HTTP
    def _handler(self):
        g = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=None, text=None):
                data = text.encode() if text is not None else (json.dumps(body).encode() if body is not None else b"")
                self.send_response(code)
                self.send_header("Content-Type", "text/plain" if text is not None else "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def _do(self, method):
                u = urlsplit(self.path)
                q = {k: v[0] for k, v in parse_qs(u.query).items()}
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n)) if n else None
                if u.path.startswith("/computeMetadata/v1/"):
                    if self.headers.get("Metadata-Flavor") != "Google":
                        return self._send(403, text="Missing Metadata-Flavor")
                    code, text = g.metadata(u.path[len("/computeMetadata/v1/"):])
                    return self._send(code, text=text)
                tok = self.headers.get("Authorization", "")[7:]
                if tok not in g.tokens:
                    return self._send(401, {"error": {"code": 401, "message": "Invalid Credentials",
                                                      "errors": [{"reason": "authError"}]}})
                p = u.path[len("/compute/v1/"):]
                with g.lock:
                    code, out = g.route(method, p, q, body)
                self._send(code, out)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

            def do_PUT(self):
                self._do("PUT")

            def do_DELETE(self):
                self._do("DELETE")
        return H

    def metadata(self, path):
        inst = self.instances.get((getattr(self, "self_zone", ""), self.self_name)) or {}
        nic = (inst.get("networkInterfaces") or [{}])[0]
        if path == "instance/service-accounts/default/token":
            self.token_calls += 1
            t = uuid.uuid4().hex
            self.tokens.add(t)
            return 200, json.dumps({"access_token": t, "expires_in": 3599, "token_type": "Bearer"})
        table = {"project/project-id": self.project, "instance/zone": f"projects/123456/zones/{getattr(self, 'self_zone', '')}",
                 "instance/hostname": f"{self.self_name}.c.{self.project}.internal",
                 "instance/network-interfaces/0/ip": nic.get("networkIP", "")}
        if nic.get("accessConfigs"):
            table["instance/network-interfaces/0/access-configs/0/external-ip"] = nic["accessConfigs"][0]["natIP"]
        return (200, table[path]) if path in table else (404, "not found")

    # ------------------------------------------------------------------ REST
    def _op(self, scope):
        name = f"operation-{uuid.uuid4().hex[:12]}"
        link = self.base + f"projects/{self.project}/{scope}/operations/{name}"
        self.ops[name] = {"name": name, "status": "DONE", "selfLink": link}
        return 200, {"name": name, "status": "RUNNING", "selfLink": link}

    @staticmethod
    def _err(code, reason, msg):
        return code, {"error": {"code": code, "message": msg, "errors": [{"reason": reason, "message": msg}]}}

    def route(self, method, p, q, body):
        pre = f"projects/{self.project}/"
        if not p.startswith(pre):
            return self._err(404, "notFound", p)
        p = p[len(pre):]
        mt = re.fullmatch(r"(zones/[^/]+|regions/[^/]+|global)/operations/([^/]+)", p)
        if mt:
            return (200, self.ops[mt.group(2)]) if mt.group(2) in self.ops else self._err(404, "notFound", p)
        if p == f"regions/{self.region}" and method == "GET":
            return 200, {"name": self.region, "zones": [self.base + f"projects/{self.project}/zones/{z}" for z in self.zones]}
        # ---- instances
        mt = re.fullmatch(r"zones/([^/]+)/instances(?:/([^/]+))?(?:/(attachDisk|detachDisk))?", p)
        if mt:
            zone, name, verb = mt.groups()
            if name is None:
                return 200, {"items": [i for (z, _), i in self.instances.items() if z == zone]}
            inst = self.instances.get((zone, name))
            if inst is None:
                return self._err(404, "notFound", f"instance {name} not found")
            if verb is None:
                return 200, inst
            if verb == "attachDisk":
                dname = body["source"].rsplit("/", 1)[-1]
                d = self.disks[(zone, dname)]
                d.setdefault("users", []).append(self.base + f"projects/{self.project}/zones/{zone}/instances/{name}")
                inst["disks"].append({"deviceName": body["deviceName"], "source": d["selfLink"], "mode": body["mode"]})
                return self._op(f"zones/{zone}")
            dev = q["deviceName"]
            for dk in inst["disks"]:
                if dk["deviceName"] == dev:
                    d = self.disks.get((zone, dk["source"].rsplit("/", 1)[-1]))
                    if d:
                        d["users"] = [x for x in d.get("users", []) if not x.endswith(f"/instances/{name}")]
            inst["disks"] = [dk for dk in inst["disks"] if dk["deviceName"] != dev]
            return self._op(f"zones/{zone}")
        # ---- disks
        mt = re.fullmatch(r"zones/([^/]+)/disks(?:/([^/]+))?", p)
        if mt:
            zone, name = mt.groups()
            if method == "POST":
                if (zone, body["name"]) in self.disks:
                    return self._err(409, "alreadyExists", "disk exists")
                d = dict(body, zone=self.base + f"projects/{self.project}/zones/{zone}", status="READY",
                         selfLink=self.base + f"projects/{self.project}/zones/{zone}/disks/{body['name']}")
                self.disks[(zone, body["name"])] = d
                return self._op(f"zones/{zone}")
            d = self.disks.get((zone, name))
            if d is None:
                return self._err(404, "notFound", f"disk {name}")
            if method == "DELETE":
                if d.get("users"):
                    return self._err(400, "resourceInUseByAnotherResource", "in use")
                del self.disks[(zone, name)]
                return self._op(f"zones/{zone}")
            return 200, d
        # ---- global routes / firewalls / health checks
        mt = re.fullmatch(r"global/(routes|firewalls|httpHealthChecks)(?:/([^/]+))?", p)
        if mt:
            kind, name = mt.groups()
            table = {"routes": self.routes, "firewalls": self.firewalls, "httpHealthChecks": self.hcs}[kind]
            if name is None and method == "GET":
                items = list(table.values())
                if kind == "routes" and q.get("filter"):
                    f = dict(re.findall(r"\((\w+) eq ([^)]*)\)", q["filter"]))
                    items = [r for r in items if re.fullmatch(f["name"], r["name"]) and r["network"] == f["network"]
                             and r["description"] == f["description"]]
                return 200, {"items": items}
            if method == "POST":
                if body["name"] in table:
                    return self._err(409, "alreadyExists", f"{kind} {body['name']} exists")
                table[body["name"]] = dict(body, selfLink=self.base + f"projects/{self.project}/global/{kind}/{body['name']}")
                return self._op("global")
            if name not in table:
                return self._err(404, "notFound", f"{kind} {name}")
            if method == "PUT":
                table[name] = dict(body, selfLink=table[name]["selfLink"])
                return self._op("global")
            if method == "DELETE":
                if kind == "httpHealthChecks" and any(name in " ".join(tp.get("healthChecks") or []) for tp in self.pools.values()):
                    return self._err(400, "resourceInUseByAnotherResource", "health check in use")
                del table[name]
                return self._op("global")
            return 200, table[name]
        # ---- regional LB pieces
        mt = re.fullmatch(rf"regions/{self.region}/(addresses|forwardingRules|targetPools)(?:/([^/]+))?(?:/(addInstance|removeInstance))?", p)
        if mt:
            kind, name, verb = mt.groups()
            table = {"addresses": self.addresses, "forwardingRules": self.rules, "targetPools": self.pools}[kind]
            if name is None and method == "GET":
                return 200, {"items": list(table.values())}
            if method == "POST" and verb is None:
                if body["name"] in table:
                    return self._err(409, "alreadyExists", f"{kind} {body['name']} exists")
                obj = dict(body, selfLink=self.base + f"projects/{self.project}/regions/{self.region}/{kind}/{body['name']}")
                if kind == "addresses":
                    obj.setdefault("address", f"35.0.0.{next(self._ip)}")
                if kind == "forwardingRules" and self.pools.get(body["target"].rsplit("/", 1)[-1]) is None:
                    return self._err(400, "invalid", "target pool does not exist")
                table[body["name"]] = obj
                return self._op(f"regions/{self.region}")
            if name not in table:
                return self._err(404, "notFound", f"{kind} {name}")
            if verb == "addInstance":
                table[name]["instances"] = table[name].get("instances", []) + [i["instance"] for i in body["instances"]]
                return self._op(f"regions/{self.region}")
            if verb == "removeInstance":
                drop = {i["instance"] for i in body["instances"]}
                table[name]["instances"] = [i for i in table[name].get("instances", []) if i not in drop]
                return self._op(f"regions/{self.region}")
            if method == "DELETE":
                if kind == "targetPools" and any(r["target"].endswith("/" + name) for r in self.rules.values()):
                    return self._err(400, "resourceInUseByAnotherResource", "pool in use")
                del table[name]
                return self._op(f"regions/{self.region}")
            return 200, table[name]
        return self._err(404, "notFound", f"no route {method} {p}")
