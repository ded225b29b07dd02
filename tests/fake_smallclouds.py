"""In-memory fakes of three small cloud APIs for the provider tests:
  * FakeCloudStack — the signed query API (signature checked on every call): listVirtualMachines,
    public IPs, load balancer rules and their instances, async jobs finished on the first poll;
  * FakeOVirt — the engine's `GET /vms?search=` XML with basic auth;
  * FakePhoton — Photon controller projects/VMs/subnets/disks and tasks (QUEUED, then COMPLETED).
Shapes follow the public API documentation; no real service exists offline."""
from __future__ import annotations

import base64
import itertools
import json
import threading
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qsl, urlsplit

from amdkube.cloudprovider.cloudstack import sign


class _Server:
    def _serve(self, handler_fn):
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _do(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n)) if n else None
                u = urlsplit(self.path)
                code, ctype, out = handler_fn(self.command, u.path, dict(parse_qsl(u.query)), body, self.headers)
                data = out if isinstance(out, bytes) else (out.encode() if isinstance(out, str) else json.dumps(out).encode())
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)
            do_GET = do_POST = do_DELETE = do_PUT = _do
        outer.lock = threading.RLock()
        outer.httpd = ThreadingHTTPServer(("127.0.0.1", 0), H)
        outer.url = f"http://127.0.0.1:{outer.httpd.server_address[1]}"

    def start(self):
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


class FakeCloudStack(_Server):
    KEY, SECRET = "ak-mi355x", "sk-secret"

    def __init__(self, zone="zone-mi355x"):
        self.zone = zone
        self.vms: dict[str, dict] = {}
        self.ips: dict[str, dict] = {}
        self.rules: dict[str, dict] = {}
        self.members: dict[str, set] = {}
        self.jobs: dict[str, dict] = {}
        self.calls: list[str] = []
        self._n = itertools.count(1)
        self._serve(self._handle)

    def add_vm(self, name, ip, public=None, offering="mi355x.8gpu", network="net-1"):
        vid = str(uuid.uuid4())
        self.vms[vid] = {"id": vid, "name": name, "zonename": self.zone, "serviceofferingname": offering,
                         "nic": [{"ipaddress": ip, "networkid": network}], **({"publicip": public} if public else {})}
        return vid

    def config(self):
        return f"[Global]\napi-url = {self.url}/client/api\napi-key = {self.KEY}\nsecret-key = {self.SECRET}\n"

    def _job(self, result):
        jid = str(uuid.uuid4())
        self.jobs[jid] = result
        return {"jobid": jid}

    def _handle(self, method, path, q, body, headers):
        sig = q.pop("signature", "")
        if q.get("apiKey") != self.KEY or sig != sign(q, self.SECRET):
            return 401, "application/json", {"errorresponse": {"errorcode": 401, "errortext": "unable to verify user credentials"}}
        cmd = q["command"]
        with self.lock:
            self.calls.append(cmd)
            resp = self._cmd(cmd, q)
        if "errorcode" in resp:
            return resp["errorcode"], "application/json", {cmd.lower() + "response": resp}
        return 200, "application/json", {cmd.lower() + "response": resp}

    def _cmd(self, cmd, q):
        if cmd == "listVirtualMachines":
            vms = [v for v in self.vms.values() if ("name" not in q or v["name"] == q["name"]) and ("id" not in q or v["id"] == q["id"])]
            return {"count": len(vms), "virtualmachine": vms} if vms else {}
        if cmd == "queryAsyncJobResult":
            return {"jobstatus": 1, "jobresult": self.jobs.pop(q["jobid"])}
        if cmd == "associateIpAddress":
            iid = str(uuid.uuid4())
            self.ips[iid] = {"id": iid, "ipaddress": f"203.0.113.{next(self._n)}", "associatednetworkid": q["networkid"]}
            return self._job({"ipaddress": self.ips[iid]})
        if cmd == "disassociateIpAddress":
            self.ips.pop(q["id"])
            return self._job({"success": True})
        if cmd == "listPublicIpAddresses":
            ips = [i for i in self.ips.values() if i["ipaddress"] == q.get("ipaddress")]
            return {"count": len(ips), "publicipaddress": ips} if ips else {}
        if cmd == "listLoadBalancerRules":
            rules = [r for r in self.rules.values() if q.get("keyword", "") in r["name"]]
            return {"count": len(rules), "loadbalancerrule": rules} if rules else {}
        if cmd == "createLoadBalancerRule":
            rid = str(uuid.uuid4())
            ip = self.ips.get(q["publicipid"]) or {"ipaddress": "?"}
            self.rules[rid] = {"id": rid, "name": q["name"], "algorithm": q["algorithm"], "publicipid": q["publicipid"],
                               "publicip": ip["ipaddress"], "publicport": q["publicport"], "privateport": q["privateport"],
                               "protocol": q["protocol"]}
            self.members[rid] = set()
            return self._job({"loadbalancer": self.rules[rid]})
        if cmd == "updateLoadBalancerRule":
            self.rules[q["id"]]["algorithm"] = q["algorithm"]
            return self._job({"loadbalancer": self.rules[q["id"]]})
        if cmd == "deleteLoadBalancerRule":
            self.rules.pop(q["id"])
            self.members.pop(q["id"], None)
            return self._job({"success": True})
        if cmd in ("assignToLoadBalancerRule", "removeFromLoadBalancerRule"):
            ids = set(q["virtualmachineids"].split(","))
            if cmd.startswith("assign"):
                self.members[q["id"]] |= ids
            else:
                self.members[q["id"]] -= ids
            return self._job({"success": True})
        if cmd == "listLoadBalancerRuleInstances":
            vms = [self.vms[i] for i in sorted(self.members.get(q["id"], ()))]
            return {"count": len(vms), "loadbalancerruleinstance": vms} if vms else {}
        return {"errorcode": 432, "errortext": f"unknown command {cmd}"}


class FakeOVirt(_Server):
    USER, PASSWORD = "admin@internal", "engine-pw"

    def __init__(self):
        self.vms: list[dict] = []
        self.searches: list[str] = []
        self._serve(self._handle)

    def add_vm(self, name, fqdn, ips=(), state="up"):
        vid = str(uuid.uuid4())
        self.vms.append({"id": vid, "name": name, "fqdn": fqdn, "ips": list(ips), "state": state})
        return vid

    def config(self):
        return f"[connection]\nuri = {self.url}/ovirt-engine/api\npassword = {self.PASSWORD}\n[filters]\nvms = cluster=gpu\n"

    def _handle(self, method, path, q, body, headers):
        want = "Basic " + base64.b64encode(f"{self.USER}:{self.PASSWORD}".encode()).decode()
        if headers.get("Authorization") != want:
            return 401, "text/plain", "unauthorized"
        if path != "/ovirt-engine/api/vms":
            return 404, "text/plain", "not found"
        self.searches.append(q.get("search", ""))
        parts = ["<vms>"]
        for v in self.vms:
            ips = "".join(f'<ip address="{a}" version="v4"/>' for a in v["ips"])
            gi = f"<guest_info><fqdn>{v['fqdn']}</fqdn><ips>{ips}</ips></guest_info>" if v["fqdn"] else ""
            parts.append(f'<vm href="/vms/{v["id"]}" id="{v["id"]}"><name>{v["name"]}</name>{gi}'
                         f"<status><state>{v['state']}</state></status></vm>")
        parts.append("</vms>")
        return 200, "application/xml", "".join(parts)


class FakePhoton(_Server):
    PROJECT, TOKEN = "proj-1", "photon-token"

    def __init__(self):
        self.vms: dict[str, dict] = {}
        self.disks: dict[str, dict] = {}
        self.tasks: dict[str, dict] = {}
        self._serve(self._handle)

    def add_vm(self, name, conns, flavor="mi355x-vm"):
        vid = str(uuid.uuid4())
        self.vms[vid] = {"id": vid, "name": name, "flavor": flavor, "conns": conns}
        return vid

    def config(self, **extra):
        lines = [f"[Global]", f"target = {self.url}", f"project = {self.PROJECT}", "username = k8s", "password = pw"]
        lines += [f"{k} = {v}" for k, v in extra.items()]
        return "\n".join(lines) + "\n"

    def _task(self, op, entity="", props=None):
        tid = str(uuid.uuid4())
        self.tasks[tid] = {"id": tid, "state": "QUEUED", "operation": op, "entity": {"id": entity},
                           "resourceProperties": props}
        return dict(self.tasks[tid])

    def _handle(self, method, path, q, body, headers):
        if path == "/auth/tokens" and method == "POST":
            return 200, "application/json", {"access_token": self.TOKEN}
        if headers.get("Authorization") != f"Bearer {self.TOKEN}":
            return 401, "application/json", {"code": "Unauthorized"}
        with self.lock:
            return self._route(method, path.strip("/").split("/"), body)

    def _route(self, method, seg, body):
        J = "application/json"
        if seg[:3] == ["projects", self.PROJECT, "vms"] and method == "GET":
            return 200, J, {"items": [{k: v for k, v in vm.items() if k != "conns"} for vm in self.vms.values()]}
        if seg[0] == "vms" and seg[1] not in self.vms:
            return 404, J, {"code": "VmNotFound"}
        if seg[0] == "vms" and len(seg) == 2:
            vm = self.vms[seg[1]]
            return 200, J, {k: v for k, v in vm.items() if k != "conns"}
        if seg[0] == "vms" and seg[2] == "subnets":
            return 200, J, self._task("GET_NETWORKS", seg[1], {"networkConnections": self.vms[seg[1]]["conns"]})
        if seg[0] == "vms" and seg[2] in ("attach_disk", "detach_disk"):
            d = self.disks.get(body["diskId"])
            if d is None:
                return 404, J, {"code": "DiskNotFound"}
            if seg[2] == "attach_disk":
                if d["vms"]:
                    return 400, J, {"code": "DiskAttached"}
                d["vms"] = [seg[1]]
            else:
                d["vms"] = [v for v in d["vms"] if v != seg[1]]
            return 200, J, self._task(seg[2].upper(), seg[1])
        if seg[:3] == ["projects", self.PROJECT, "disks"] and method == "POST":
            did = str(uuid.uuid4())
            self.disks[did] = {"id": did, "name": body["name"], "kind": body["kind"], "flavor": body["flavor"],
                               "capacityGb": body["capacityGb"], "state": "DETACHED", "vms": []}
            return 200, J, self._task("CREATE_DISK", did)
        if seg[0] == "disks":
            d = self.disks.get(seg[1])
            if d is None:
                return 404, J, {"code": "DiskNotFound"}
            if method == "DELETE":
                del self.disks[seg[1]]
                return 200, J, self._task("DELETE_DISK", seg[1])
            return 200, J, d
        if seg[0] == "tasks":
            t = self.tasks[seg[1]]
            t["state"] = "COMPLETED"
            return 200, J, t
        return 404, J, {"code": "NotFound"}
