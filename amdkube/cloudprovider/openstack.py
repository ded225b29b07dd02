"""The OpenStack cloud provider: the on-prem cloud MI355X fleets commonly sit in.

Reference: pkg/cloudprovider/providers/openstack — openstack.go (Keystone auth, nodeAddresses:
floating or "public"-network addresses are ExternalIP, the rest InternalIP, plus accessIPv4/v6;
servers found by `name=^<node>$`; providerID `openstack:///<server id>`), openstack_instances.go
(instance type from the flavor name/id/original_name), openstack_routes.go (Neutron router
extra routes with next hop = the node's address, plus an allowed-address-pair on the node's port,
each step unwound on failure), openstack_loadbalancer.go (LBaaS v2 / Octavia: a load balancer
on --subnet-id named after the service UID, one listener + pool per service port, node
InternalIP:nodePort members, optional health monitor, a floating IP on --floating-network-id),
openstack_volumes.go (Cinder volumes attached through Nova os-volume_attachments, device
/dev/disk/by-id/virtio-<id[:20]>).

This implementation speaks the public REST APIs directly (Keystone v3 password or token auth
with the service catalog; Nova v2.1; Neutron v2.0; Octavia v2 or Neutron LBaaS v2; Cinder
v3/v2) with `requests`; no SDK. Config: the reference's cloud.conf INI sections ([Global],
[LoadBalancer], [BlockStorage], [Route], [Metadata]) or the same keys as YAML/JSON.
"""
from __future__ import annotations

import asyncio
import configparser
import ipaddress
import json
import logging
import re
import threading
import time

from . import Interface, Route, Zone
from ..api import meta as m

log = logging.getLogger("amdkube.cloudprovider.openstack")
PROVIDER = "openstack"
METADATA_URL = "http://169.254.169.254/openstack/latest/meta_data.json"


class OpenStackError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"openstack: HTTP {status}: {msg}")
        self.status = status


def parse_config(cfg) -> dict:
    """cloud.conf (INI, gcfg sections) or a dict → {section: {key: value}} with lower-case sections."""
    if isinstance(cfg, str):
        try:
            data = json.loads(cfg)
        except ValueError:
            cp = configparser.ConfigParser(interpolation=None)
            cp.read_string(cfg)
            data = {s: dict(cp.items(s)) for s in cp.sections()}
        cfg = data
    out = {}
    for sec, vals in (cfg or {}).items():
        key = sec.lower().replace("_", "").replace("-", "")
        out[key] = {str(k).lower(): v for k, v in (vals or {}).items()} if isinstance(vals, dict) else vals
    return out


class Client:
    """Keystone v3 session + service catalog; JSON requests with one re-auth on 401."""

    def __init__(self, g: dict, session=None):
        import requests
        self.g = g
        self.auth_url = str(g.get("auth-url", "")).rstrip("/")
        if not self.auth_url:
            raise ValueError("openstack: [Global] auth-url is required")
        self.region = g.get("region", "")
        self.http = session or requests.Session()
        ca = g.get("ca-file")
        self.http.verify = ca if ca else True
        self.token, self.catalog, self.expires = None, [], 0.0
        self._lock = threading.Lock()

    def _auth_body(self) -> dict:
        g = self.g
        if g.get("application-credential-id"):
            ident = {"methods": ["application_credential"], "application_credential": {
                "id": g["application-credential-id"], "secret": g.get("application-credential-secret", "")}}
            return {"auth": {"identity": ident}}
        user = {"password": g.get("password", "")}
        if g.get("user-id"):
            user["id"] = g["user-id"]
        else:
            user["name"] = g.get("username", "")
            user["domain"] = {"id": g["domain-id"]} if g.get("domain-id") else {"name": g.get("domain-name", "Default")}
        body = {"auth": {"identity": {"methods": ["password"], "password": {"user": user}}}}
        if g.get("trust-id"):
            body["auth"]["scope"] = {"OS-TRUST:trust": {"id": g["trust-id"]}}
        elif g.get("tenant-id"):
            body["auth"]["scope"] = {"project": {"id": g["tenant-id"]}}
        elif g.get("tenant-name"):
            dom = {"id": g["domain-id"]} if g.get("domain-id") else {"name": g.get("domain-name", "Default")}
            body["auth"]["scope"] = {"project": {"name": g["tenant-name"], "domain": dom}}
        return body

    def authenticate(self):
        url = self.auth_url if self.auth_url.endswith("/v3") else self.auth_url + "/v3"
        r = self.http.post(url + "/auth/tokens", json=self._auth_body(), timeout=30)
        if r.status_code not in (200, 201):
            raise OpenStackError(r.status_code, f"keystone authentication failed: {r.text[:200]}")
        self.token = r.headers.get("X-Subject-Token")
        tok = r.json().get("token") or {}
        self.catalog = tok.get("catalog") or []
        self.expires = time.time() + 3000

    def endpoint(self, *types: str) -> str:
        with self._lock:
            if self.token is None or time.time() > self.expires:
                self.authenticate()
        for t in types:
            for svc in self.catalog:
                if svc.get("type") != t:
                    continue
                for ep in svc.get("endpoints") or []:
                    if ep.get("interface", "public") == "public" and (not self.region or
                                                                     self.region in (ep.get("region_id"), ep.get("region"))):
                        return ep["url"].rstrip("/")
        raise OpenStackError(404, f"no {'/'.join(types)} endpoint in region {self.region!r}")

    def call(self, service: tuple, method: str, path: str, body=None, ok=(200, 201, 202, 204), params=None):
        base = self.endpoint(*service)
        for attempt in (0, 1):
            r = self.http.request(method, base + path, json=body, params=params, timeout=60,
                                  headers={"X-Auth-Token": self.token or "", "Accept": "application/json"})
            if r.status_code == 401 and attempt == 0:
                with self._lock:
                    self.authenticate()
                continue
            break
        if r.status_code not in ok:
            raise OpenStackError(r.status_code, f"{method} {path}: {r.text[:300]}")
        return r.json() if r.content and r.headers.get("Content-Type", "").startswith("application/json") else None


COMPUTE, NETWORK, VOLUME = ("compute",), ("network",), ("volumev3", "volumev2", "volume", "block-storage")


def node_addresses(srv: dict) -> list[dict]:
    out: list[dict] = []

    def add(t, a):
        e = {"type": t, "address": a}
        if a and e not in out:
            out.append(e)
    for net, lst in sorted((srv.get("addresses") or {}).items()):
        for a in lst or []:
            add("ExternalIP" if a.get("OS-EXT-IPS:type") == "floating" or net == "public" else "InternalIP", a.get("addr"))
    for k in ("accessIPv4", "accessIPv6"):
        if srv.get(k):
            add("ExternalIP", srv[k])
    return out


class Instances:
    def __init__(self, os_):
        self.os = os_

    def server(self, name: str) -> dict:
        lst = self.os.client.call(COMPUTE, "GET", "/servers/detail",
                                  params={"name": f"^{re.escape(name)}$", "status": "ACTIVE"})["servers"]
        if not lst:
            raise LookupError(f"instance {name} not found")
        if len(lst) > 1:
            raise LookupError(f"multiple instances named {name}")
        self.os.servers[name] = lst[0]
        return lst[0]

    def server_by_id(self, sid: str) -> dict | None:
        try:
            return self.os.client.call(COMPUTE, "GET", f"/servers/{sid}")["server"]
        except OpenStackError as e:
            if e.status == 404:
                return None
            raise

    async def node_addresses(self, name: str) -> list[dict]:
        return node_addresses(await asyncio.to_thread(self.server, name))

    async def instance_exists(self, name: str) -> bool:
        try:
            await asyncio.to_thread(self.server, name)
            return True
        except LookupError:
            return False

    async def instance_exists_by_provider_id(self, provider_id: str) -> bool:
        return (await asyncio.to_thread(self.server_by_id, instance_id_from_provider_id(provider_id))) is not None

    async def instance_id(self, name: str) -> str:
        return f"{PROVIDER}:///{(await asyncio.to_thread(self.server, name))['id']}"

    async def instance_type(self, name: str) -> str:
        fl = (await asyncio.to_thread(self.server, name)).get("flavor") or {}
        for k in ("name", "id", "original_name"):
            if isinstance(fl.get(k), str):
                return fl[k]
        return ""


def instance_id_from_provider_id(pid: str) -> str:
    mt = re.fullmatch(rf"{PROVIDER}:///([^/]+)", pid or "")
    if not mt:
        raise ValueError(f'ProviderID "{pid}" didn\'t match expected format "openstack:///InstanceID"')
    return mt.group(1)


class Routes:
    """Neutron router extra routes (next hop = the node's InternalIP) + allowed-address-pairs."""
    named = False          # Neutron keeps no route names: any route to a cluster node is ours

    def __init__(self, os_, router_id: str):
        self.os, self.router_id = os_, router_id

    def _router(self) -> dict:
        return self.os.client.call(NETWORK, "GET", f"/v2.0/routers/{self.router_id}")["router"]

    def _put_routes(self, routes):
        self.os.client.call(NETWORK, "PUT", f"/v2.0/routers/{self.router_id}", {"router": {"routes": routes}})

    def _node_ip(self, node: str, v6: bool) -> tuple[str, dict]:
        srv = self.os.instances_.server(node)
        for a in node_addresses(srv):
            if a["type"] == "InternalIP" and (ipaddress.ip_address(a["address"]).version == 6) == v6:
                return a["address"], srv
        raise LookupError(f"node {node} has no internal IPv{6 if v6 else 4} address")

    def _port(self, srv: dict, ip: str) -> dict:
        for p in self.os.client.call(NETWORK, "GET", "/v2.0/ports", params={"device_id": srv["id"]})["ports"]:
            if any(f.get("ip_address") == ip for f in p.get("fixed_ips") or []):
                return p
        raise LookupError(f"no port with {ip} on server {srv['id']}")

    def list(self, cluster: str) -> list[Route]:
        ip_to_node = {}
        for srv in self.os.client.call(COMPUTE, "GET", "/servers/detail")["servers"]:
            for a in node_addresses(srv):
                ip_to_node.setdefault(a["address"], srv["name"])
        out = []
        for r in self._router().get("routes") or []:
            node = ip_to_node.get(r.get("nexthop"))
            if node:
                out.append(Route(f"{node}-{r['destination']}", node, r["destination"]))
        return out

    def create(self, cluster: str, name_hint: str, route: Route):
        v6 = ipaddress.ip_network(route.destination_cidr, strict=False).version == 6
        ip, srv = self._node_ip(route.target_node, v6)
        router = self._router()
        old = list(router.get("routes") or [])
        if any(r.get("destination") == route.destination_cidr and r.get("nexthop") == ip for r in old):
            return
        self._put_routes(old + [{"destination": route.destination_cidr, "nexthop": ip}])
        try:
            port = self._port(srv, ip)
            pairs = list(port.get("allowed_address_pairs") or [])
            if not any(p.get("ip_address") == route.destination_cidr for p in pairs):
                self.os.client.call(NETWORK, "PUT", f"/v2.0/ports/{port['id']}",
                                    {"port": {"allowed_address_pairs": pairs + [{"ip_address": route.destination_cidr}]}})
        except Exception:
            self._put_routes(old)                      # unwind the router change
            raise

    def delete(self, cluster: str, route: Route):
        v6 = ipaddress.ip_network(route.destination_cidr, strict=False).version == 6
        ip, srv = self._node_ip(route.target_node, v6)
        router = self._router()
        old = list(router.get("routes") or [])
        keep = [r for r in old if not (r.get("destination") == route.destination_cidr and r.get("nexthop") == ip)]
        if keep != old:
            self._put_routes(keep)
        port = self._port(srv, ip)
        pairs = [p for p in port.get("allowed_address_pairs") or [] if p.get("ip_address") != route.destination_cidr]
        if pairs != (port.get("allowed_address_pairs") or []):
            self.os.client.call(NETWORK, "PUT", f"/v2.0/ports/{port['id']}", {"port": {"allowed_address_pairs": pairs}})


def lb_name(svc: dict) -> str:
    """cloudprovider.GetLoadBalancerName: "a" + the service UID without dashes, at most 32 chars."""
    return ("a" + m.uid_of(svc).replace("-", ""))[:32]


class LoadBalancer:
    def __init__(self, os_, cfg: dict):
        self.os, self.cfg = os_, cfg
        self.timeout = float(cfg.get("provisioning-timeout", 300))

    # Octavia (load-balancer service) or Neutron's LBaaS v2 extension: same resource shapes
    def _svc(self):
        try:
            self.os.client.endpoint("load-balancer")
            return ("load-balancer",), "/v2/lbaas"
        except OpenStackError:
            return NETWORK, "/v2.0/lbaas"

    def _call(self, method, path, body=None, ok=(200, 201, 202, 204), params=None):
        svc, prefix = self._svc()
        return self.os.client.call(svc, method, prefix + path, body, ok, params)

    def _find(self, svc) -> dict | None:
        lst = self._call("GET", "/loadbalancers", params={"name": lb_name(svc)})["loadbalancers"]
        return lst[0] if lst else None

    def _wait_active(self, lb_id: str):
        deadline = time.monotonic() + self.timeout
        while True:
            lb = self._call("GET", f"/loadbalancers/{lb_id}")["loadbalancer"]
            st = lb.get("provisioning_status")
            if st == "ACTIVE":
                return lb
            if st == "ERROR" or time.monotonic() > deadline:
                raise OpenStackError(500, f"load balancer {lb_id} is {st}")
            time.sleep(1.0)

    def _floating(self, lb: dict) -> dict | None:
        lst = self.os.client.call(NETWORK, "GET", "/v2.0/floatingips", params={"port_id": lb["vip_port_id"]})["floatingips"]
        return lst[0] if lst else None

    def _status(self, lb: dict) -> dict:
        fip = self._floating(lb) if self.cfg.get("floating-network-id") else None
        return {"ingress": [{"ip": (fip or {}).get("floating_ip_address") or lb["vip_address"]}]}

    def get(self, cluster: str, svc: dict):
        lb = self._find(svc)
        return (self._status(lb), True) if lb else (None, False)

    def _members(self, nodes, port) -> set[tuple[str, int]]:
        out = set()
        for n in nodes:
            ip = next((a["address"] for a in (n.get("status") or {}).get("addresses") or [] if a.get("type") == "InternalIP"), None)
            if ip and port.get("nodePort"):
                out.add((ip, int(port["nodePort"])))
        return out

    def _sync_pool(self, lb_id: str, pool_id: str, want: set):
        have = {(mb["address"], mb["protocol_port"]): mb["id"]
                for mb in self._call("GET", f"/pools/{pool_id}/members")["members"]}
        for addr in sorted(want - set(have)):
            self._call("POST", f"/pools/{pool_id}/members", {"member": {"address": addr[0], "protocol_port": addr[1],
                                                                         "subnet_id": self.cfg.get("subnet-id", "")}})
            self._wait_active(lb_id)
        for addr in sorted(set(have) - want):
            self._call("DELETE", f"/pools/{pool_id}/members/{have[addr]}")
            self._wait_active(lb_id)

    def ensure(self, cluster: str, svc: dict, nodes: list[dict]) -> dict:
        spec = svc.get("spec") or {}
        ports = spec.get("ports") or []
        if any(p.get("protocol", "TCP") != "TCP" for p in ports):
            raise ValueError("only TCP LoadBalancer services are supported on OpenStack")
        if not self.cfg.get("subnet-id"):
            raise ValueError("openstack: [LoadBalancer] subnet-id is required for LoadBalancer services")
        lb = self._find(svc)
        if lb is None:
            lb = self._call("POST", "/loadbalancers", {"loadbalancer": {
                "name": lb_name(svc), "vip_subnet_id": self.cfg["subnet-id"],
                "description": f"Kubernetes external service {m.namespace_of(svc)}/{m.name_of(svc)}"}})["loadbalancer"]
        lb = self._wait_active(lb["id"])
        listeners = {ls["protocol_port"]: ls for ls in self._call("GET", "/listeners", params={"loadbalancer_id": lb["id"]})["listeners"]}
        method = self.cfg.get("lb-method", "ROUND_ROBIN")
        for i, p in enumerate(ports):
            ls = listeners.pop(int(p["port"]), None)
            if ls is None:
                ls = self._call("POST", "/listeners", {"listener": {"name": f"listener_{i}_{lb_name(svc)}", "protocol": "TCP",
                                                                     "protocol_port": int(p["port"]), "loadbalancer_id": lb["id"]}})["listener"]
                self._wait_active(lb["id"])
            pools = self._call("GET", "/pools", params={"listener_id": ls["id"]})["pools"]
            if pools:
                pool = pools[0]
            else:
                pool = self._call("POST", "/pools", {"pool": {"name": f"pool_{i}_{lb_name(svc)}", "protocol": "TCP",
                                                               "lb_algorithm": method, "listener_id": ls["id"]}})["pool"]
                self._wait_active(lb["id"])
            self._sync_pool(lb["id"], pool["id"], self._members(nodes, p))
            if str(self.cfg.get("create-monitor", "false")).lower() == "true" and not pool.get("healthmonitor_id"):
                self._call("POST", "/healthmonitors", {"healthmonitor": {
                    "pool_id": pool["id"], "type": "TCP", "delay": _secs(self.cfg.get("monitor-delay", "5s")),
                    "timeout": _secs(self.cfg.get("monitor-timeout", "3s")),
                    "max_retries": int(self.cfg.get("monitor-max-retries", 1))}})
                self._wait_active(lb["id"])
        for ls in listeners.values():                  # ports the service no longer has
            self._delete_listener(lb["id"], ls)
        fnet = self.cfg.get("floating-network-id")
        if fnet and self._floating(lb) is None:
            body = {"floating_network_id": fnet, "port_id": lb["vip_port_id"]}
            if spec.get("loadBalancerIP"):
                body["floating_ip_address"] = spec["loadBalancerIP"]
            self.os.client.call(NETWORK, "POST", "/v2.0/floatingips", {"floatingip": body})
        return self._status(lb)

    def _delete_listener(self, lb_id, ls):
        for pool in self._call("GET", "/pools", params={"listener_id": ls["id"]})["pools"]:
            if pool.get("healthmonitor_id"):
                self._call("DELETE", f"/healthmonitors/{pool['healthmonitor_id']}")
                self._wait_active(lb_id)
            for mb in self._call("GET", f"/pools/{pool['id']}/members")["members"]:
                self._call("DELETE", f"/pools/{pool['id']}/members/{mb['id']}")
                self._wait_active(lb_id)
            self._call("DELETE", f"/pools/{pool['id']}")
            self._wait_active(lb_id)
        self._call("DELETE", f"/listeners/{ls['id']}")
        self._wait_active(lb_id)

    def update(self, cluster: str, svc: dict, nodes: list[dict]):
        lb = self._find(svc)
        if lb is None:
            raise LookupError(f"load balancer for {m.key_of(svc)} not found")
        listeners = {ls["protocol_port"]: ls for ls in self._call("GET", "/listeners", params={"loadbalancer_id": lb["id"]})["listeners"]}
        for p in (svc.get("spec") or {}).get("ports") or []:
            ls = listeners.get(int(p["port"]))
            if ls is None:
                continue
            for pool in self._call("GET", "/pools", params={"listener_id": ls["id"]})["pools"]:
                self._sync_pool(lb["id"], pool["id"], self._members(nodes, p))

    def ensure_deleted(self, cluster: str, svc: dict):
        lb = self._find(svc)
        if lb is None:
            return
        fip = self._floating(lb) if self.cfg.get("floating-network-id") else None
        if fip is not None:
            self.os.client.call(NETWORK, "DELETE", f"/v2.0/floatingips/{fip['id']}")
        for ls in self._call("GET", "/listeners", params={"loadbalancer_id": lb["id"]})["listeners"]:
            self._delete_listener(lb["id"], ls)
        self._call("DELETE", f"/loadbalancers/{lb['id']}")


def _secs(v) -> int:
    s = str(v).strip()
    mt = re.fullmatch(r"(\d+)(ms|s|m)?", s)
    if not mt:
        return 5
    n, unit = int(mt.group(1)), mt.group(2) or "s"
    return max(1, n // 1000 if unit == "ms" else n * 60 if unit == "m" else n)


class Volumes:
    """Cinder block storage attached to servers through Nova (openstack_volumes.go)."""
    provisioner = "kubernetes.io/cinder"
    source_key = "cinder"

    def __init__(self, os_, cfg: dict):
        self.os, self.cfg = os_, cfg
        self.poll = 1.0

    def create(self, name: str, size_gib: int, vtype: str = "", zone: str = "", tags: dict | None = None) -> dict:
        body = {"name": name, "size": size_gib}
        if vtype:
            body["volume_type"] = vtype
        if zone:
            body["availability_zone"] = zone
        if tags:
            body["metadata"] = tags
        return self.os.client.call(VOLUME, "POST", "/volumes", {"volume": body})["volume"]

    def get(self, vid: str) -> dict:
        return self.os.client.call(VOLUME, "GET", f"/volumes/{vid}")["volume"]

    def delete(self, vid: str):
        v = self.get(vid)
        if v.get("attachments"):
            raise OpenStackError(409, f"volume {vid} is attached; detach it before deleting")
        self.os.client.call(VOLUME, "DELETE", f"/volumes/{vid}")

    def _wait(self, vid: str, status: str, timeout: float = 120):
        deadline = time.monotonic() + timeout
        while True:
            v = self.get(vid)
            if v.get("status") == status:
                return v
            if v.get("status") in ("error", "error_attaching", "error_detaching") or time.monotonic() > deadline:
                raise OpenStackError(500, f"volume {vid} is {v.get('status')}, wanted {status}")
            time.sleep(self.poll)

    def attach(self, node: str, vid: str) -> str:
        """Attach to the node's server; returns the device path Nova reports (may be a guess)."""
        srv = self.os.instances_.server(node)
        v = self.get(vid)
        for a in v.get("attachments") or []:
            if a.get("server_id") == srv["id"]:
                return a.get("device", "")
            raise OpenStackError(409, f"volume {vid} is attached to another server {a.get('server_id')}")
        att = self.os.client.call(COMPUTE, "POST", f"/servers/{srv['id']}/os-volume_attachments",
                                  {"volumeAttachment": {"volumeId": vid}})["volumeAttachment"]
        self._wait(vid, "in-use")
        return att.get("device", "")

    def detach(self, node: str, vid: str):
        srv = self.os.instances_.server(node)
        v = self.get(vid)
        if not any(a.get("server_id") == srv["id"] for a in v.get("attachments") or []):
            return
        self.os.client.call(COMPUTE, "DELETE", f"/servers/{srv['id']}/os-volume_attachments/{vid}")
        self._wait(vid, "available")

    def zone(self, vid: str) -> str:
        return self.get(vid).get("availability_zone", "")

    def device_candidates(self, vid: str, device_path: str = "") -> list[str]:
        """By serial first; Nova's reported device only with [BlockStorage] trust-device-path."""
        pats = device_candidates(vid)
        if device_path and str(self.cfg.get("trust-device-path", "false")).lower() == "true":
            pats = [device_path] + pats
        return pats

    # ---- the provisioner interface (controllers/volumes.py)
    def provision(self, name: str, gib: int, params: dict, tags: dict, pvc_name: str) -> tuple[dict, dict]:
        """cinder_util.go CreateVolume: the class's availability zone and type."""
        vol = self.create(f"kubernetes-dynamic-{name}", gib, params.get("type", ""), params.get("availability", ""), tags)
        labels = {}
        if vol.get("availability_zone"):
            labels["failure-domain.beta.kubernetes.io/zone"] = vol["availability_zone"]
        if self.os.client.region:
            labels["failure-domain.beta.kubernetes.io/region"] = self.os.client.region
        return {"volumeID": vol["id"], "fsType": params.get("fsType", "ext4")}, labels

    def delete_source(self, src: dict):
        self.delete(src["volumeID"])


def device_candidates(vid: str) -> list[str]:
    """Where a virtio/SCSI Cinder disk shows up (GetDevicePathBySerialId)."""
    s = vid[:20]
    return [f"/dev/disk/by-id/virtio-{s}", f"/dev/disk/by-id/scsi-0QEMU_QEMU_HARDDISK_{s}", f"/dev/disk/by-id/*{s}*"]


class OpenStack(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        cfg = parse_config(config)
        self.cfg = cfg
        self.client = Client(cfg.get("global") or {}, session=session)
        self.servers: dict[str, dict] = {}
        self.instances_ = Instances(self)
        lbc = cfg.get("loadbalancer") or {}
        self._lb = LoadBalancer(self, lbc) if lbc.get("subnet-id") and str(lbc.get("enabled", "true")).lower() != "false" else None
        rid = (cfg.get("route") or {}).get("router-id")
        self._routes = Routes(self, rid) if rid else None
        self.volumes_ = Volumes(self, cfg.get("blockstorage") or {})
        self._zone: Zone | None = None

    def load_balancer(self):
        return self._lb

    def instances(self):
        return self.instances_

    def routes(self):
        return self._routes

    def volumes(self):
        return self.volumes_

    def zones(self):
        """This host's zone from the metadata service (or [Global] zone)."""
        if self._zone is None:
            g = self.cfg.get("global") or {}
            az = g.get("zone", "")
            if not az:
                try:
                    r = self.client.http.get(METADATA_URL, timeout=2)
                    az = r.json().get("availability_zone", "") if r.ok else ""
                except Exception:
                    az = ""
            self._zone = Zone(az, self.client.region)
        return self._zone

    def zone_for_node(self, node_name: str) -> Zone:
        srv = self.servers.get(node_name)
        if srv is None:
            try:
                srv = self.instances_.server(node_name)
            except Exception:
                return self.zones()
        return Zone(srv.get("OS-EXT-AZ:availability_zone", ""), self.client.region)

    def labels_for_volume(self, pv: dict) -> dict:
        """PVLabeler: Cinder volumes get their availability zone and the region."""
        src = (pv.get("spec") or {}).get("cinder")
        if not src:
            return {}
        az = self.volumes_.zone(src["volumeID"])
        out = {"failure-domain.beta.kubernetes.io/region": self.client.region} if self.client.region else {}
        if az:
            out["failure-domain.beta.kubernetes.io/zone"] = az
        return out
