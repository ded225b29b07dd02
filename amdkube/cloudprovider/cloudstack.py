"""Apache CloudStack cloud provider (reference: pkg/cloudprovider/providers/cloudstack —
cloudstack.go config/zones, cloudstack_instances.go, cloudstack_loadbalancer.go, metadata.go).

The CloudStack API is one signed query endpoint: every call is `command=<Name>` plus
parameters, `apiKey` and `response=json`, signed with HMAC-SHA1 over the lower-cased, sorted,
URL-encoded query (`signature=`). Mutating calls answer `{jobid}` and are polled with
`queryAsyncJobResult` until `jobstatus` leaves 0.

  * Instances/Zones: `listVirtualMachines` by name (or id for provider IDs) within the
    configured project: the first NIC's address is the InternalIP, a static NAT public IP the
    ExternalIP, the service offering the instance type and the VM's zone both failure domain and
    region, as the reference reports it.
  * LoadBalancer: one public IP per Service (`associateIpAddress` on the nodes' network, or the
    address named by spec.loadBalancerIP found with `listPublicIpAddresses`) and one load
    balancer rule per service port named `<lb name>-<protocol>-<port>` (publicport = port,
    privateport = nodePort, roundrobin or `source` for ClientIP affinity). Rules whose ports
    changed are replaced, rules for ports the Service dropped are deleted, and the rules'
    instances track the node set (assignToLoadBalancerRule / removeFromLoadBalancerRule by
    symmetric difference). Deleting the Service deletes its rules and releases the address if
    the provider associated it.
  * Without API keys, a node answers Instances/Zones from the virtual router's metadata service
    (`http://<dhcp server>/latest/meta-data/…`, metadata.go) — `metadata-url` in the config.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import logging
import time
from urllib.parse import quote

from . import Interface, Zone, off_loop
from ..api import meta as m
from .openstack import parse_config

log = logging.getLogger("amdkube.cloudprovider.cloudstack")
PROVIDER = "cloudstack"


class CloudStackError(RuntimeError):
    def __init__(self, code: int, text: str):
        super().__init__(f"CloudStack API error {code}: {text}")
        self.code = code


def _enc(v: str) -> str:
    return quote(str(v), safe="*").replace("+", "%20")


def sign(params: dict, secret: str) -> str:
    """The API signature: HMAC-SHA1 over the lower-cased, key-sorted, encoded query, base64."""
    q = "&".join(f"{k}={_enc(v)}" for k, v in sorted(params.items(), key=lambda kv: kv[0].lower()))
    return base64.b64encode(hmac.new(secret.encode(), q.lower().encode(), hashlib.sha1).digest()).decode()


def lb_name(svc: dict) -> str:
    """cloudprovider.GetLoadBalancerName: 'a' + the Service UID without dashes, 32 chars."""
    return ("a" + m.uid_of(svc).replace("-", ""))[:32]


class Client:
    def __init__(self, url: str, api_key: str, secret: str, http, project_id: str = ""):
        self.url, self.key, self.secret, self.http, self.project = url, api_key, secret, http, project_id

    def call(self, command: str, **params) -> dict:
        p = {k: str(v) for k, v in params.items() if v not in (None, "")}
        p.update(command=command, apiKey=self.key, response="json")
        p["signature"] = sign(p, self.secret)
        r = self.http.get(self.url, params=p, timeout=30)
        try:
            body = r.json()
        except ValueError:
            raise CloudStackError(r.status_code, r.text[:200]) from None
        resp = body.get(command.lower() + "response") or next(iter(body.values()), {})
        if r.status_code >= 400 or "errorcode" in resp:
            raise CloudStackError(int(resp.get("errorcode", r.status_code)), resp.get("errortext", r.text[:200]))
        return resp

    def run(self, command: str, timeout: float = 300, **params) -> dict:
        """An async command: poll its job; the job result is returned."""
        job = self.call(command, **params).get("jobid")
        if not job:
            raise CloudStackError(530, f"{command} returned no job id")
        end = time.monotonic() + timeout
        delay = 0.05
        while True:
            st = self.call("queryAsyncJobResult", jobid=job)
            if int(st.get("jobstatus", 0)) == 1:
                return st.get("jobresult") or {}
            if int(st.get("jobstatus", 0)) == 2:
                res = st.get("jobresult") or {}
                raise CloudStackError(int(res.get("errorcode", 530)), res.get("errortext", f"{command} failed"))
            if time.monotonic() > end:
                raise TimeoutError(f"CloudStack job {job} ({command}) did not finish in {timeout}s")
            time.sleep(delay)
            delay = min(delay * 2, 2.0)

    def vms(self, **filt) -> list[dict]:
        return self.call("listVirtualMachines", projectid=self.project, listall="true", **filt).get("virtualmachine") or []


def _addresses(vm: dict) -> list[dict]:
    nics = vm.get("nic") or []
    if not nics or not nics[0].get("ipaddress"):
        raise LookupError(f"instance {vm.get('name')} has no NIC address")
    out = [{"type": "InternalIP", "address": nics[0]["ipaddress"]}]
    if vm.get("publicip"):
        out.append({"type": "ExternalIP", "address": vm["publicip"]})
    return out


class Instances:
    def __init__(self, cs: "CloudStack"):
        self.cs = cs

    def _by_name(self, name: str) -> dict:
        vms = [v for v in self.cs.client.vms(name=name) if v.get("name") == name]
        if not vms:
            raise LookupError(f"instance not found: {name}")
        if len(vms) > 1:
            raise LookupError(f"{len(vms)} instances are named {name}")
        return vms[0]

    def _by_id(self, pid: str) -> dict | None:
        vid = pid.split("://", 1)[-1].lstrip("/")
        vms = self.cs.client.vms(id=vid)
        return vms[0] if vms else None

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        return _addresses(self._by_name(name))

    @off_loop
    def node_addresses_by_provider_id(self, pid: str) -> list[dict]:
        vm = self._by_id(pid)
        if vm is None:
            raise LookupError(f"instance not found: {pid}")
        return _addresses(vm)

    @off_loop
    def instance_exists(self, name: str) -> bool:
        try:
            self._by_name(name)
            return True
        except LookupError:
            return False

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        return self._by_id(pid) is not None

    @off_loop
    def instance_id(self, name: str) -> str:
        return self._by_name(name)["id"]

    @off_loop
    def instance_type(self, name: str) -> str:
        return self._by_name(name).get("serviceofferingname", "")


class MetadataInstances:
    """metadata.go: a node without API credentials asks the virtual router about itself."""

    def __init__(self, cs: "CloudStack"):
        self.cs = cs

    def get(self, key: str) -> str:
        r = self.cs.http.get(self.cs.metadata_url.rstrip("/") + "/" + key, timeout=5)
        if r.status_code != 200:
            raise LookupError(f"metadata {key}: HTTP {r.status_code}")
        return r.text.strip()

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        out = [{"type": "InternalIP", "address": self.get("local-ipv4")}]
        try:
            pub = self.get("public-ipv4")
            if pub:
                out.append({"type": "ExternalIP", "address": pub})
        except LookupError:
            pass
        return out

    @off_loop
    def instance_exists(self, name: str) -> bool:
        return True

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        raise NotImplementedError("the metadata service only knows this instance")

    @off_loop
    def instance_id(self, name: str) -> str:
        return self.get("instance-id")

    @off_loop
    def instance_type(self, name: str) -> str:
        return self.get("service-offering")


class LoadBalancer:
    def __init__(self, cs: "CloudStack"):
        self.cs = cs

    @property
    def c(self) -> Client:
        return self.cs.client

    def _rules(self, name: str) -> dict[str, dict]:
        rules = self.c.call("listLoadBalancerRules", keyword=name, projectid=self.c.project, listall="true").get("loadbalancerrule") or []
        return {r["name"]: r for r in rules if r["name"].startswith(name + "-")}

    def get(self, cluster: str, svc: dict):
        rules = self._rules(lb_name(svc))
        if not rules:
            return None, False
        return {"ingress": [{"ip": next(iter(rules.values()))["publicip"]}]}, True

    def _hosts(self, nodes: list[dict]) -> tuple[list[str], str]:
        """verifyHosts: the VM ids of the nodes and the one network they share."""
        names = {m.name_of(n) for n in nodes}
        ids, nets = [], set()
        for vm in self.c.vms():
            if vm.get("name") in names:
                ids.append(vm["id"])
                nets.add((vm.get("nic") or [{}])[0].get("networkid", ""))
        if not ids:
            raise LookupError("none of the nodes is a CloudStack instance")
        if len(nets) != 1:
            raise ValueError(f"the nodes are on {len(nets)} networks; a CloudStack load balancer needs one")
        return sorted(ids), nets.pop()

    def _address(self, svc: dict, network: str, rules: dict) -> tuple[str, str, bool]:
        """(ip, ip id, associated by us) — an existing rule's address, the requested one, or a new one."""
        want = (svc.get("spec") or {}).get("loadBalancerIP") or ""
        for r in rules.values():
            if not want or r["publicip"] == want:
                return r["publicip"], r["publicipid"], False
        if want:
            ips = self.c.call("listPublicIpAddresses", ipaddress=want, projectid=self.c.project, listall="true").get("publicipaddress") or []
            if not ips:
                raise LookupError(f"could not find IP address {want}")
            return ips[0]["ipaddress"], ips[0]["id"], False
        ip = self.c.run("associateIpAddress", networkid=network, projectid=self.c.project)["ipaddress"]
        return ip["ipaddress"], ip["id"], True

    def ensure(self, cluster: str, svc: dict, nodes: list[dict]) -> dict:
        spec = svc.get("spec") or {}
        name = lb_name(svc)
        hosts, network = self._hosts(nodes)
        rules = self._rules(name)
        ip, ip_id, _ = self._address(svc, network, rules)
        algo = "source" if spec.get("sessionAffinity") == "ClientIP" else "roundrobin"
        keep = set()
        for p in spec.get("ports") or []:
            proto = (p.get("protocol") or "TCP").lower()
            if proto != "tcp":
                raise ValueError(f"CloudStack load balancers support TCP only, not {proto.upper()}")
            rname = f"{name}-{proto}-{p['port']}"
            keep.add(rname)
            r = rules.get(rname)
            if r and (str(r["publicport"]) != str(p["port"]) or str(r["privateport"]) != str(p.get("nodePort"))
                      or r["publicipid"] != ip_id):
                self.c.run("deleteLoadBalancerRule", id=r["id"])
                r = None
            if r is None:
                r = self.c.run("createLoadBalancerRule", name=rname, algorithm=algo, publicipid=ip_id, networkid=network,
                               publicport=p["port"], privateport=p.get("nodePort"), protocol=proto,
                               openfirewall="false")["loadbalancer"]
                self.c.run("assignToLoadBalancerRule", id=r["id"], virtualmachineids=",".join(hosts))
            elif r.get("algorithm") != algo:
                self.c.run("updateLoadBalancerRule", id=r["id"], algorithm=algo)
        for rname, r in rules.items():
            if rname not in keep:
                self.c.run("deleteLoadBalancerRule", id=r["id"])
        self._sync_hosts(name, hosts)
        return {"ingress": [{"ip": ip}]}

    def _sync_hosts(self, name: str, hosts: list[str]):
        for r in self._rules(name).values():
            have = {v["id"] for v in self.c.call("listLoadBalancerRuleInstances", id=r["id"], projectid=self.c.project,
                                                 listall="true").get("loadbalancerruleinstance") or []}
            add, drop = sorted(set(hosts) - have), sorted(have - set(hosts))
            if add:
                self.c.run("assignToLoadBalancerRule", id=r["id"], virtualmachineids=",".join(add))
            if drop:
                self.c.run("removeFromLoadBalancerRule", id=r["id"], virtualmachineids=",".join(drop))

    def update(self, cluster: str, svc: dict, nodes: list[dict]):
        self._sync_hosts(lb_name(svc), self._hosts(nodes)[0])

    def ensure_deleted(self, cluster: str, svc: dict):
        rules = self._rules(lb_name(svc))
        ip_ids = {r["publicipid"] for r in rules.values()}
        for r in rules.values():
            self.c.run("deleteLoadBalancerRule", id=r["id"])
        if (svc.get("spec") or {}).get("loadBalancerIP"):
            return                       # the user's address: not ours to release
        for ip_id in ip_ids:
            self.c.run("disassociateIpAddress", id=ip_id)


class CloudStack(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        g = parse_config(config).get("global") or {}
        self.http = session or requests.Session()
        self.metadata_url = g.get("metadata-url", "")
        self.zone = g.get("zone", "")
        self.client = None
        if g.get("api-url") and g.get("api-key") and g.get("secret-key"):
            if str(g.get("ssl-no-verify", "")).lower() in ("1", "true", "yes"):
                self.http.verify = False
            self.client = Client(g["api-url"], g["api-key"], g["secret-key"], self.http, g.get("project-id", ""))
        elif not self.metadata_url:
            raise ValueError("cloudstack: api-url, api-key and secret-key, or metadata-url, are needed in the cloud config")
        self.instances_ = Instances(self) if self.client else MetadataInstances(self)
        self._lb = LoadBalancer(self) if self.client else None

    def instances(self):
        return self.instances_

    def load_balancer(self):
        return self._lb

    def zones(self):
        if not self.zone:
            if self.client is None:
                self.zone = MetadataInstances(self).get("availability-zone")
            else:
                import socket
                vms = self.client.vms(name=socket.gethostname())
                self.zone = vms[0].get("zonename", "") if vms else ""
        return Zone(self.zone, self.zone)

    def zone_for_node(self, node_name: str) -> Zone:
        if self.client is not None:
            vms = [v for v in self.client.vms(name=node_name) if v.get("name") == node_name]
            if vms:
                return Zone(vms[0].get("zonename", ""), vms[0].get("zonename", ""))
        return self.zones()
