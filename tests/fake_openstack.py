"""A small in-memory OpenStack (Keystone v3, Nova, Neutron, Octavia, Cinder) for the provider
tests: enough of each public REST API, with the reference's resource shapes, that
cloudprovider/openstack.py can be driven end to end. Runs on its own thread (the provider's
client is synchronous)."""
from __future__ import annotations

import itertools
import json
import re
import threading
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlsplit


class FakeOpenStack:
    def __init__(self, region="RegionOne", project="proj-1"):
        self.region, self.project = region, project
        self.lock = threading.RLock()
        self.servers: dict[str, dict] = {}
        self.ports: dict[str, dict] = {}
        self.routers: dict[str, dict] = {}
        self.fips: dict[str, dict] = {}
        self.lbs: dict[str, dict] = {}
        self.listeners: dict[str, dict] = {}
        self.pools: dict[str, dict] = {}
        self.members: dict[str, dict] = {}
        self.monitors: dict[str, dict] = {}
        self.volumes: dict[str, dict] = {}
        self.tokens: set[str] = set()
        self.auth_calls = 0
        self.fail_next: dict[str, int] = {}       # "METHOD path-regex" -> HTTP status (once)
        self.on_attach = None                     # fn(server, volume) when Nova attaches a volume
        self._vip = itertools.count(10)
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"

    # ------------------------------------------------------------------ fixtures
    def add_server(self, name, fixed_ip, floating_ip=None, az="nova", flavor="gpu.mi355x.8x"):
        sid = str(uuid.uuid4())
        addrs = {"private": [{"addr": fixed_ip, "version": 4, "OS-EXT-IPS:type": "fixed"}]}
        if floating_ip:
            addrs["private"].append({"addr": floating_ip, "version": 4, "OS-EXT-IPS:type": "floating"})
        self.servers[sid] = {"id": sid, "name": name, "status": "ACTIVE", "addresses": addrs,
                             "flavor": {"original_name": flavor}, "OS-EXT-AZ:availability_zone": az, "accessIPv4": ""}
        pid = str(uuid.uuid4())
        self.ports[pid] = {"id": pid, "device_id": sid, "fixed_ips": [{"ip_address": fixed_ip, "subnet_id": "subnet-1"}],
                           "allowed_address_pairs": []}
        return sid

    def add_router(self, rid="router-1"):
        self.routers[rid] = {"id": rid, "name": "k8s", "routes": []}

    def start(self):
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def config(self, **lb):
        return {"Global": {"auth-url": self.url + "/identity/v3", "username": "admin", "password": "secret",
                           "tenant-id": self.project, "domain-name": "Default", "region": self.region},
                "LoadBalancer": {"subnet-id": "subnet-1", "floating-network-id": "public-net", **lb},
                "Route": {"router-id": "router-1"}, "BlockStorage": {"bs-version": "v3"}}

    def catalog(self):
        def ep(url):
            return [{"interface": "public", "region_id": self.region, "region": self.region, "url": url}]
        return [{"type": "compute", "endpoints": ep(self.url + "/compute/v2.1")},
                {"type": "network", "endpoints": ep(self.url + "/network")},
                {"type": "load-balancer", "endpoints": ep(self.url + "/lb")},
                {"type": "volumev3", "endpoints": ep(self.url + f"/volume/v3/{self.project}")},
                {"type": "identity", "endpoints": ep(self.url + "/identity")}]

    # ------------------------------------------------------------------ HTTP
    def _handler(self):
        os_ = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=None, headers=None):
                data = json.dumps(body).encode() if body is not None else b""
                self.send_response(code)
                if body is not None:
                    self.send_header("Content-Type", "application/json")
                for k, v in (headers or {}).items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def _do(self, method):
                u = urlsplit(self.path)
                q = {k: v[0] for k, v in parse_qs(u.query).items()}
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n)) if n else None
                with os_.lock:
                    for pat, code in list(os_.fail_next.items()):
                        mth, _, rx = pat.partition(" ")
                        if mth == method and re.search(rx, u.path):
                            del os_.fail_next[pat]
                            return self._send(code, {"error": "injected"})
                    if u.path.endswith("/auth/tokens") and method == "POST":
                        os_.auth_calls += 1
                        pw = body["auth"]["identity"]["password"]["user"]["password"]
                        if pw != "secret":
                            return self._send(401, {"error": "bad credentials"})
                        tok = uuid.uuid4().hex
                        os_.tokens.add(tok)
                        return self._send(201, {"token": {"catalog": os_.catalog()}}, {"X-Subject-Token": tok})
                    if self.headers.get("X-Auth-Token") not in os_.tokens:
                        return self._send(401, {"error": "token"})
                    code, out = os_.route(method, u.path, q, body)
                return self._send(code, out)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

            def do_PUT(self):
                self._do("PUT")

            def do_DELETE(self):
                self._do("DELETE")
        return H

    def route(self, method, path, q, body):
        p = path
        # ---- nova
        if p == "/compute/v2.1/servers/detail":
            rx = re.compile(q["name"]) if "name" in q else None
            lst = [s for s in self.servers.values() if (rx is None or rx.search(s["name"]))
                   and s["status"] == q.get("status", s["status"])]
            return 200, {"servers": lst}
        mt = re.fullmatch(r"/compute/v2.1/servers/([^/]+)", p)
        if mt and method == "GET":
            s = self.servers.get(mt.group(1))
            return (200, {"server": s}) if s else (404, {"itemNotFound": {}})
        mt = re.fullmatch(r"/compute/v2.1/servers/([^/]+)/os-volume_attachments(?:/([^/]+))?", p)
        if mt:
            srv, vid = self.servers[mt.group(1)], (mt.group(2) or (body or {}).get("volumeAttachment", {}).get("volumeId"))
            v = self.volumes[vid]
            if method == "POST":
                dev = f"/dev/vd{chr(ord('b') + len([x for x in self.volumes.values() if x['attachments']]))}"
                v["attachments"] = [{"server_id": srv["id"], "device": dev, "volume_id": vid}]
                v["status"] = "in-use"
                if self.on_attach:
                    self.on_attach(srv, v)
                return 200, {"volumeAttachment": {"id": vid, "volumeId": vid, "serverId": srv["id"], "device": dev}}
            if method == "DELETE":
                v["attachments"], v["status"] = [], "available"
                return 202, None
        # ---- neutron
        mt = re.fullmatch(r"/network/v2.0/routers/([^/]+)", p)
        if mt:
            r = self.routers[mt.group(1)]
            if method == "PUT":
                r["routes"] = body["router"]["routes"]
            return 200, {"router": r}
        if p == "/network/v2.0/ports":
            return 200, {"ports": [x for x in self.ports.values() if x["device_id"] == q.get("device_id", x["device_id"])]}
        mt = re.fullmatch(r"/network/v2.0/ports/([^/]+)", p)
        if mt and method == "PUT":
            port = self.ports[mt.group(1)]
            port.update(body["port"])
            return 200, {"port": port}
        if p == "/network/v2.0/floatingips":
            if method == "GET":
                return 200, {"floatingips": [f for f in self.fips.values() if f["port_id"] == q.get("port_id", f["port_id"])]}
            fid = str(uuid.uuid4())
            f = {"id": fid, "port_id": body["floatingip"]["port_id"],
                 "floating_ip_address": body["floatingip"].get("floating_ip_address") or f"203.0.113.{next(self._vip)}",
                 "floating_network_id": body["floatingip"]["floating_network_id"]}
            self.fips[fid] = f
            return 201, {"floatingip": f}
        mt = re.fullmatch(r"/network/v2.0/floatingips/([^/]+)", p)
        if mt and method == "DELETE":
            self.fips.pop(mt.group(1), None)
            return 204, None
        # ---- octavia
        mt = re.fullmatch(r"/lb/v2/lbaas/(loadbalancers|listeners|pools|healthmonitors)(?:/([^/]+))?", p)
        if mt:
            kind, rid = mt.groups()
            table = {"loadbalancers": self.lbs, "listeners": self.listeners, "pools": self.pools,
                     "healthmonitors": self.monitors}[kind]
            single = kind[:-1]
            if method == "GET" and rid is None:
                flt = {k: v for k, v in q.items()}
                return 200, {kind: [x for x in table.values() if all(str(x.get(k)) == v for k, v in flt.items())]}
            if method == "GET":
                return (200, {single: table[rid]}) if rid in table else (404, {})
            if method == "POST":
                obj = dict(body[single], id=str(uuid.uuid4()), provisioning_status="ACTIVE")
                if kind == "loadbalancers":
                    obj.update(vip_address=f"10.0.1.{next(self._vip)}", vip_port_id=str(uuid.uuid4()))
                if kind == "healthmonitors":
                    self.pools[obj["pool_id"]]["healthmonitor_id"] = obj["id"]
                table[obj["id"]] = obj
                return 201, {single: obj}
            if method == "DELETE":
                table.pop(rid, None)
                return 204, None
        mt = re.fullmatch(r"/lb/v2/lbaas/pools/([^/]+)/members(?:/([^/]+))?", p)
        if mt:
            pool, mid = mt.groups()
            if method == "GET":
                return 200, {"members": [x for x in self.members.values() if x["pool_id"] == pool]}
            if method == "POST":
                obj = dict(body["member"], id=str(uuid.uuid4()), pool_id=pool)
                self.members[obj["id"]] = obj
                return 201, {"member": obj}
            if method == "DELETE":
                self.members.pop(mid, None)
                return 204, None
        # ---- cinder
        mt = re.fullmatch(rf"/volume/v3/{self.project}/volumes(?:/([^/]+))?", p)
        if mt:
            vid = mt.group(1)
            if method == "POST":
                v = dict(body["volume"], id=str(uuid.uuid4()), status="available", attachments=[])
                v.setdefault("availability_zone", "nova")
                self.volumes[v["id"]] = v
                return 202, {"volume": v}
            if method == "GET":
                return (200, {"volume": self.volumes[vid]}) if vid in self.volumes else (404, {})
            if method == "DELETE":
                self.volumes.pop(vid, None)
                return 202, None
        return 404, {"error": f"no route {method} {p}"}
