"""The GCE cloud provider: Compute Engine instances/zones/routes, external TCP/UDP load balancers
(target pool + forwarding rule), persistent disks.

The fork's README lists GCP GPU VMs among its platforms. Reference:
pkg/cloudprovider/providers/gce —
  * gce.go config ([global] project-id, network-name, subnetwork-name, node-tags,
    node-instance-prefix, multizone, api-endpoint, token-url/local-zone), the metadata server
    (project/project-id, instance/zone, service-account tokens);
  * gce_instances.go: node name = instance name; NodeAddresses of this instance from the
    metadata server (network-interfaces/0/ip and its access-config's external-ip), others'
    from instances.get; InstanceID `<project>/<zone>/<name>` (providerID `gce://…`),
    InstanceType = the machine type's last segment; multizone lookups across the region's zones;
  * gce_routes.go: routes named `<cluster[:26]>-<hint>`, description `k8s-node-route`, next hop
    the instance, priority 1000, listed by name prefix + network + description;
  * gce_loadbalancer_external.go + gce_loadbalancer_naming.go: static address `a<uid>`, firewall
    `k8s-fw-<name>` (loadBalancerSourceRanges → node tags, the service ports), an HTTP health
    check (`k8s-<cluster-id>-node` on kube-proxy's 10256/healthz, or the service's own
    healthCheckNodePort for externalTrafficPolicy=Local), target pool of the node instances with
    the session affinity, and a forwarding rule over the ports' min-max range;
  * gce_disks.go: zonal PDs (pd-standard / pd-ssd), attach with deviceName = disk name (the node
    sees /dev/disk/by-id/google-<name>), detach by device name, labels zone/region, the JSON
    description tags; gce_op.go: every mutation waits for its zone/region/global Operation.

The Compute v1 REST API is spoken directly with `requests` and OAuth2 bearer tokens from the
metadata server's default service account (or a configured token URL / static token).
"""
from __future__ import annotations

import configparser
import json
import logging
import re
import threading
import time

from . import Interface, Route, Zone, off_loop
from ..api import meta as m

log = logging.getLogger("amdkube.cloudprovider.gce")
PROVIDER = "gce"
API_ENDPOINT = "https://www.googleapis.com/compute/v1/"
METADATA_URL = "http://metadata.google.internal/computeMetadata/v1/"
ROUTE_TAG = "k8s-node-route"
PD_PROVISIONER = "kubernetes.io/gce-pd"
NODES_HC_PORT, NODES_HC_PATH = 10256, "/healthz"


class GCEError(RuntimeError):
    def __init__(self, status: int, reason: str, msg: str):
        super().__init__(f"gce: {reason} (HTTP {status}): {msg}")
        self.status, self.reason = status, reason


def parse_config(cfg) -> dict:
    """gce.conf ([global] gcfg keys) or a dict → {key: value}; node-tags may repeat (a list)."""
    if isinstance(cfg, str):
        try:
            cfg = json.loads(cfg)
        except ValueError:
            cp = configparser.ConfigParser(interpolation=None, strict=False)
            cp.read_string(cfg)
            cfg = {s: dict(cp.items(s)) for s in cp.sections()}
    cfg = cfg or {}
    glob = next((v for k, v in cfg.items() if str(k).lower() == "global"), None)
    out = {str(k).lower(): v for k, v in (glob if isinstance(glob, dict) else cfg).items()}
    tags = out.get("node-tags", [])
    out["node-tags"] = [t.strip() for t in (tags.split(",") if isinstance(tags, str) else tags) if str(t).strip()]
    return out


def _last(url: str) -> str:
    return str(url).rstrip("/").rsplit("/", 1)[-1]


def region_of_zone(zone: str) -> str:
    """GetGCERegion: `us-central1-b` → `us-central1`."""
    ix = zone.rfind("-")
    if ix < 0:
        raise ValueError(f"unexpected zone: {zone}")
    return zone[:ix]


def split_provider_id(pid: str) -> tuple[str, str, str]:
    mt = re.fullmatch(r"gce://([^/]+)/([^/]+)/([^/]+)", pid)
    if not mt:
        raise ValueError(f"error splitting providerID {pid!r}")
    return mt.group(1), mt.group(2), mt.group(3)


def canonical_instance_name(name: str) -> str:
    """mapNodeNameToInstanceName + canonicalizeInstanceName: the hostname's first label."""
    return name.split(".", 1)[0]


class Metadata:
    def __init__(self, http, url: str = METADATA_URL):
        self.http, self.url = http, url.rstrip("/") + "/"

    def get(self, path: str) -> str:
        r = self.http.get(self.url + path.lstrip("/"), headers={"Metadata-Flavor": "Google"}, timeout=5)
        if r.status_code != 200:
            raise GCEError(r.status_code, "metadata", f"{path}: {r.text[:120]}")
        return r.text


class Client:
    """JSON calls against compute/v1 with a cached OAuth2 access token."""

    def __init__(self, cfg: dict, md: Metadata, http):
        self.cfg, self.md, self.http = cfg, md, http
        self.base = str(cfg.get("api-endpoint") or API_ENDPOINT).rstrip("/") + "/"
        self._tok, self._exp = "", 0.0
        self._lock = threading.Lock()
        self.poll = 1.0

    def token(self) -> str:
        with self._lock:
            if self.cfg.get("token"):
                return self.cfg["token"]
            if self._tok and time.time() < self._exp - 60:
                return self._tok
            if self.cfg.get("token-url"):
                r = self.http.post(self.cfg["token-url"], data=self.cfg.get("token-body", ""), timeout=10)
                doc = r.json()
            else:
                doc = json.loads(self.md.get("instance/service-accounts/default/token"))
            self._tok, self._exp = doc["access_token"], time.time() + float(doc.get("expires_in", 3600))
            return self._tok

    def call(self, method: str, path: str, body=None, params=None, ok=(200,)):
        url = path if path.startswith("http") else self.base + path.lstrip("/")
        for attempt in (0, 1):
            r = self.http.request(method, url, json=body, params=params, timeout=60,
                                  headers={"Authorization": f"Bearer {self.token()}"})
            if r.status_code == 401 and attempt == 0:
                with self._lock:
                    self._tok = ""
                continue
            break
        if r.status_code not in ok:
            reason, msg = "unknown", r.text[:300]
            try:
                err = r.json().get("error") or {}
                msg = err.get("message", msg)
                reason = ((err.get("errors") or [{}])[0]).get("reason", reason)
            except ValueError:
                pass
            raise GCEError(r.status_code, reason, f"{method} {path}: {msg}")
        return r.json() if r.content else {}

    def wait(self, op: dict, timeout: float = 300) -> dict:
        """gce_op.go waitForOp: poll the Operation (zonal, regional or global) until DONE."""
        deadline = time.monotonic() + timeout
        while op.get("status") != "DONE":
            if time.monotonic() > deadline:
                raise GCEError(504, "timeout", f"operation {op.get('name')} did not finish")
            time.sleep(self.poll)
            op = self.call("GET", op["selfLink"])
        errs = ((op.get("error") or {}).get("errors")) or []
        if errs:
            raise GCEError(int(op.get("httpErrorStatusCode", 400)), errs[0].get("code", "error"), errs[0].get("message", ""))
        return op

    def mutate(self, method: str, path: str, body=None, params=None, ok=(200,)):
        return self.wait(self.call(method, path, body, params, ok))


def addresses_of(inst: dict) -> list[dict]:
    out = []
    nics = inst.get("networkInterfaces") or []
    if nics:
        if nics[0].get("networkIP"):
            out.append({"type": "InternalIP", "address": nics[0]["networkIP"]})
        for ac in nics[0].get("accessConfigs") or []:
            if ac.get("natIP"):
                out.append({"type": "ExternalIP", "address": ac["natIP"]})
    return out


class Instances:
    def __init__(self, gce):
        self.gce = gce

    def get(self, name: str) -> dict:
        """getInstanceByName: the instance in any of the managed zones."""
        name = canonical_instance_name(name)
        for z in self.gce.managed_zones():
            try:
                inst = self.gce.client.call("GET", f"projects/{self.gce.project}/zones/{z}/instances/{name}")
                inst["zone"] = _last(inst.get("zone", z))
                return inst
            except GCEError as e:
                if e.status != 404:
                    raise
        raise LookupError(f"instance not found: {name}")

    def _is_self(self, name: str) -> bool:
        return self.gce.self_name and canonical_instance_name(name) == self.gce.self_name

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        if self._is_self(name):
            out = [{"type": "InternalIP", "address": self.gce.md.get("instance/network-interfaces/0/ip").strip()}]
            try:
                ext = self.gce.md.get("instance/network-interfaces/0/access-configs/0/external-ip").strip()
                if ext:
                    out.append({"type": "ExternalIP", "address": ext})
            except GCEError:
                pass
            return out
        return addresses_of(self.get(name))

    @off_loop
    def node_addresses_by_provider_id(self, pid: str) -> list[dict]:
        project, zone, name = split_provider_id(pid)
        return addresses_of(self.gce.client.call("GET", f"projects/{project}/zones/{zone}/instances/{name}"))

    @off_loop
    def instance_exists(self, name: str) -> bool:
        try:
            self.get(name)
            return True
        except LookupError:
            return False

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        project, zone, name = split_provider_id(pid)
        try:
            self.gce.client.call("GET", f"projects/{project}/zones/{zone}/instances/{name}")
            return True
        except GCEError as e:
            if e.status == 404:
                return False
            raise

    @off_loop
    def instance_id(self, name: str) -> str:
        inst = self.get(name)
        return f"{self.gce.project}/{inst['zone']}/{inst['name']}"

    @off_loop
    def instance_type(self, name: str) -> str:
        return _last(self.get(name).get("machineType", ""))


class Routes:
    def __init__(self, gce):
        self.gce = gce

    def list(self, cluster: str) -> list[Route]:
        prefix = cluster[:26]
        flt = f"(name eq {prefix}-.*) (network eq {self.gce.network_url()}) (description eq {ROUTE_TAG})"
        out, token = [], None
        while True:
            params = {"filter": flt, **({"pageToken": token} if token else {})}
            d = self.gce.client.call("GET", f"projects/{self.gce.network_project}/global/routes", params=params)
            for r in d.get("items") or []:
                out.append(Route(r["name"], _last(r.get("nextHopInstance", "")), r.get("destRange", "")))
            token = d.get("nextPageToken")
            if not token:
                return out

    def create(self, cluster: str, name_hint: str, route: Route):
        inst = self.gce.instances_.get(route.target_node)
        body = {"name": f"{cluster[:26]}-{name_hint}", "destRange": route.destination_cidr,
                "nextHopInstance": f"zones/{inst['zone']}/instances/{inst['name']}", "network": self.gce.network_url(),
                "priority": 1000, "description": ROUTE_TAG}
        try:
            self.gce.client.mutate("POST", f"projects/{self.gce.network_project}/global/routes", body)
        except GCEError as e:
            if e.status != 409:
                raise

    def delete(self, cluster: str, route: Route):
        try:
            self.gce.client.mutate("DELETE", f"projects/{self.gce.network_project}/global/routes/{route.name}")
        except GCEError as e:
            if e.status != 404:
                raise


def lb_name(svc: dict) -> str:
    return ("a" + m.uid_of(svc).replace("-", ""))[:32]


def port_range(ports: list[dict]) -> str:
    """loadBalancerPortRange: one forwarding rule covers min..max of the service ports."""
    if not ports:
        raise ValueError("no ports specified for GCE load balancer")
    ps = [int(p["port"]) for p in ports]
    return f"{min(ps)}-{max(ps)}"


class LoadBalancer:
    def __init__(self, gce):
        self.gce = gce

    def _r(self, kind: str, name: str = "") -> str:
        return f"projects/{self.gce.project}/regions/{self.gce.region}/{kind}" + (f"/{name}" if name else "")

    def _g(self, kind: str, name: str = "") -> str:
        return f"projects/{self.gce.project}/global/{kind}" + (f"/{name}" if name else "")

    def _get(self, path: str) -> dict | None:
        try:
            return self.gce.client.call("GET", path)
        except GCEError as e:
            if e.status == 404:
                return None
            raise

    def get(self, cluster: str, svc: dict):
        fr = self._get(self._r("forwardingRules", lb_name(svc)))
        return ({"ingress": [{"ip": fr.get("IPAddress", "")}]}, True) if fr else (None, False)

    def _hosts(self, nodes: list[dict]) -> list[dict]:
        return [self.gce.instances_.get(m.name_of(n)) for n in nodes]

    def _host_url(self, inst: dict) -> str:
        return f"{self.gce.client.base}projects/{self.gce.project}/zones/{inst['zone']}/instances/{inst['name']}"

    def _health_check(self, svc: dict, name: str, cluster_id: str) -> tuple[str, dict]:
        spec = svc.get("spec") or {}
        if spec.get("externalTrafficPolicy") == "Local" and spec.get("healthCheckNodePort"):
            hc = {"name": name, "port": int(spec["healthCheckNodePort"]), "requestPath": "/healthz"}
        else:
            hc = {"name": f"k8s-{cluster_id}-node", "port": NODES_HC_PORT, "requestPath": NODES_HC_PATH}
        hc.update(checkIntervalSec=8, timeoutSec=1, healthyThreshold=1, unhealthyThreshold=3,
                  description=json.dumps({"kubernetes.io/service-name": m.key_of(svc)}))
        have = self._get(self._g("httpHealthChecks", hc["name"]))
        if have is None:
            self.gce.client.mutate("POST", self._g("httpHealthChecks"), hc)
        elif (have.get("port"), have.get("requestPath")) != (hc["port"], hc["requestPath"]):
            self.gce.client.mutate("PUT", self._g("httpHealthChecks", hc["name"]), {**have, **hc})
        return hc["name"], hc

    def ensure(self, cluster: str, svc: dict, nodes: list[dict]) -> dict:
        spec = svc.get("spec") or {}
        if not nodes:
            raise ValueError("cannot EnsureLoadBalancer() with no hosts")
        ports = spec.get("ports") or []
        protos = {p.get("protocol", "TCP") for p in ports}
        if len(protos) > 1:
            raise ValueError("mixed protocols are not supported for GCE load balancers")
        proto = (protos or {"TCP"}).pop()
        name, c = lb_name(svc), self.gce.client
        hosts = self._hosts(nodes)
        desc = json.dumps({"kubernetes.io/service-name": m.key_of(svc)})
        # static IP (ensureStaticIP); a user-requested IP must be free or already ours
        fr = self._get(self._r("forwardingRules", name))
        want_ip = spec.get("loadBalancerIP", "")
        addr = self._get(self._r("addresses", name))
        if addr is None:
            body = {"name": name, "description": desc, **({"address": want_ip} if want_ip else {})}
            c.mutate("POST", self._r("addresses"), body)
            addr = self._get(self._r("addresses", name)) or {}
        elif want_ip and addr.get("address") != want_ip:
            raise ValueError(f"requested loadBalancerIP {want_ip} differs from the reserved address {addr.get('address')}")
        ip = addr.get("address", "")
        # firewall k8s-fw-<name>
        fw_name = f"k8s-fw-{name}"
        fw = {"name": fw_name, "description": json.dumps({"kubernetes.io/service-name": m.key_of(svc), "kubernetes.io/service-ip": ip}),
              "network": self.gce.network_url(), "sourceRanges": sorted(spec.get("loadBalancerSourceRanges") or ["0.0.0.0/0"]),
              "targetTags": self.gce.node_tags(hosts),
              "allowed": [{"IPProtocol": proto.lower(), "ports": sorted({str(p["port"]) for p in ports}, key=int)}]}
        have_fw = self._get(self._g("firewalls", fw_name))
        if have_fw is None:
            c.mutate("POST", self._g("firewalls"), fw)
        elif any(have_fw.get(k) != fw[k] for k in ("sourceRanges", "allowed", "targetTags")):
            c.mutate("PUT", self._g("firewalls", fw_name), fw)
        # health check + target pool (recreated when the affinity changes)
        hc_name, _ = self._health_check(svc, name, self.gce.cluster_id)
        affinity = "CLIENT_IP" if spec.get("sessionAffinity") == "ClientIP" else "NONE"
        tp = self._get(self._r("targetPools", name))
        recreate = tp is not None and tp.get("sessionAffinity", "NONE") != affinity
        if tp is not None and [_last(h) for h in tp.get("healthChecks") or []] != [hc_name]:
            recreate = True
        fr_update = fr is not None and (fr.get("portRange") != port_range(ports) or fr.get("IPAddress") != ip
                                        or fr.get("IPProtocol") != proto)
        if fr is not None and (recreate or fr_update):
            c.mutate("DELETE", self._r("forwardingRules", name))
            fr = None
        if recreate:
            c.mutate("DELETE", self._r("targetPools", name))
            tp = None
        if tp is None:
            c.mutate("POST", self._r("targetPools"), {
                "name": name, "description": desc, "sessionAffinity": affinity,
                "instances": [self._host_url(h) for h in hosts],
                "healthChecks": [f"{c.base}{self._g('httpHealthChecks', hc_name)}"]})
        else:
            self._sync_pool(name, tp, hosts)
        if fr is None:
            c.mutate("POST", self._r("forwardingRules"), {
                "name": name, "description": desc, "IPAddress": ip, "IPProtocol": proto, "portRange": port_range(ports),
                "target": f"{c.base}{self._r('targetPools', name)}"})
        return {"ingress": [{"ip": ip}]}

    def _sync_pool(self, name: str, tp: dict, hosts: list[dict]):
        c = self.gce.client
        have = {_last(u): u for u in tp.get("instances") or []}
        want = {h["name"]: self._host_url(h) for h in hosts}
        add = [want[n] for n in sorted(set(want) - set(have))]
        rm = [have[n] for n in sorted(set(have) - set(want))]
        if add:
            c.mutate("POST", self._r("targetPools", name) + "/addInstance", {"instances": [{"instance": u} for u in add]})
        if rm:
            c.mutate("POST", self._r("targetPools", name) + "/removeInstance", {"instances": [{"instance": u} for u in rm]})

    def update(self, cluster: str, svc: dict, nodes: list[dict]):
        name = lb_name(svc)
        tp = self._get(self._r("targetPools", name))
        if tp is None:
            raise LookupError(f"target pool {name} not found")
        hosts = self._hosts(nodes)
        self._sync_pool(name, tp, hosts)
        fw = self._get(self._g("firewalls", f"k8s-fw-{name}"))
        tags = self.gce.node_tags(hosts)
        if fw is not None and fw.get("targetTags") != tags:
            self.gce.client.mutate("PUT", self._g("firewalls", f"k8s-fw-{name}"), {**fw, "targetTags": tags})

    def ensure_deleted(self, cluster: str, svc: dict):
        name, c = lb_name(svc), self.gce.client
        tp = self._get(self._r("targetPools", name))
        for path in (self._r("forwardingRules", name), self._r("addresses", name), self._g("firewalls", f"k8s-fw-{name}"),
                     self._r("targetPools", name)):
            try:
                c.mutate("DELETE", path)
            except GCEError as e:
                if e.status != 404:
                    raise
        # the service's own health check goes; the shared nodes check stays while other pools use it
        for hc in [_last(h) for h in (tp or {}).get("healthChecks") or []]:
            if hc == name:
                c.mutate("DELETE", self._g("httpHealthChecks", hc))
            else:
                users = [p for p in (c.call("GET", self._r("targetPools")).get("items") or [])
                         if any(_last(h) == hc for h in p.get("healthChecks") or [])]
                if not users:
                    try:
                        c.mutate("DELETE", self._g("httpHealthChecks", hc))
                    except GCEError as e:
                        if e.status != 404:
                            raise


class Volumes:
    """Zonal persistent disks (gce_disks.go)."""
    provisioner = PD_PROVISIONER
    source_key = "gcePersistentDisk"

    def __init__(self, gce):
        self.gce = gce

    def _zones_of(self, name: str) -> dict | None:
        for z in self.gce.managed_zones():
            try:
                d = self.gce.client.call("GET", f"projects/{self.gce.project}/zones/{z}/disks/{name}")
                d["zone"] = _last(d.get("zone", z))
                return d
            except GCEError as e:
                if e.status != 404:
                    raise
        return None

    def get(self, name: str) -> dict:
        d = self._zones_of(name)
        if d is None:
            raise LookupError(f"GCE persistent disk {name} not found in zones {self.gce.managed_zones()}")
        return d

    def zones_with_instances(self) -> list[str]:
        out = set()
        for z in self.gce.managed_zones():
            items = self.gce.client.call("GET", f"projects/{self.gce.project}/zones/{z}/instances").get("items") or []
            if any(i.get("status", "RUNNING") == "RUNNING" for i in items):
                out.add(z)
        return sorted(out)

    def create(self, name: str, size_gib: int, params: dict, tags: dict, pvc_name: str = "") -> dict:
        from .aws import choose_zone
        zone = params.get("zone", "")
        if not zone:
            zones = [z.strip() for z in params.get("zones", "").split(",") if z.strip()] or self.zones_with_instances()
            if not zones:
                raise LookupError("no zones with instances to create the disk in")
            zone = choose_zone(zones, pvc_name or name)
        dtype = params.get("type", "pd-standard")
        if dtype not in ("pd-standard", "pd-ssd"):
            raise ValueError(f"invalid GCE disk type {dtype!r}: must be pd-standard or pd-ssd")
        body = {"name": name, "sizeGb": str(size_gib), "description": json.dumps(tags, sort_keys=True),
                "type": f"{self.gce.client.base}projects/{self.gce.project}/zones/{zone}/diskTypes/{dtype}"}
        try:
            self.gce.client.mutate("POST", f"projects/{self.gce.project}/zones/{zone}/disks", body)
        except GCEError as e:
            if e.status != 409:          # an earlier attempt created it
                raise
        return self.get(name)

    def delete(self, name: str) -> bool:
        d = self._zones_of(name)
        if d is None:
            return False
        if d.get("users"):
            raise GCEError(400, "resourceInUseByAnotherResource", f"disk {name} is attached to {d['users']}")
        self.gce.client.mutate("DELETE", f"projects/{self.gce.project}/zones/{d['zone']}/disks/{name}")
        return True

    def attach(self, node: str, name: str, read_only: bool = False) -> str:
        inst = self.gce.instances_.get(node)
        d = self.get(name)
        if d["zone"] != inst["zone"]:
            raise GCEError(400, "zoneMismatch", f"disk {name} is in {d['zone']}, node {node} in {inst['zone']}")
        if any(_last(att.get("source", "")) == name for att in inst.get("disks") or []):
            return f"/dev/disk/by-id/google-{name}"
        self.gce.client.mutate("POST", f"projects/{self.gce.project}/zones/{inst['zone']}/instances/{inst['name']}/attachDisk",
                               {"source": d.get("selfLink") or f"projects/{self.gce.project}/zones/{d['zone']}/disks/{name}",
                                "deviceName": name, "mode": "READ_ONLY" if read_only else "READ_WRITE", "type": "PERSISTENT"})
        return f"/dev/disk/by-id/google-{name}"

    def detach(self, node: str, name: str):
        try:
            inst = self.gce.instances_.get(node)
        except LookupError:
            return                      # the instance is gone: nothing is attached
        if not any(att.get("deviceName") == name for att in inst.get("disks") or []):
            return
        self.gce.client.mutate("POST", f"projects/{self.gce.project}/zones/{inst['zone']}/instances/{inst['name']}/detachDisk",
                               params={"deviceName": name})

    def zone(self, name: str) -> str:
        return self.get(name)["zone"]

    def device_candidates(self, name: str, device_path: str = "") -> list[str]:
        return [f"/dev/disk/by-id/google-{name}", f"/dev/disk/by-id/scsi-0Google_PersistentDisk_{name}"]

    def provision(self, name: str, gib: int, params: dict, tags: dict, pvc_name: str) -> tuple[dict, dict]:
        p = {str(k).lower(): v for k, v in params.items()}
        dname = f"kubernetes-dynamic-{name}"[:63]
        d = self.create(dname, gib, p, tags, pvc_name)
        return ({"pdName": dname, "fsType": p.get("fstype", "ext4")},
                {"failure-domain.beta.kubernetes.io/zone": d["zone"],
                 "failure-domain.beta.kubernetes.io/region": region_of_zone(d["zone"])})

    def delete_source(self, src: dict):
        self.delete(src["pdName"])


class GCE(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        self.cfg = parse_config(config)
        self.http = session or requests.Session()
        self.md = Metadata(self.http, self.cfg.get("metadata-url", METADATA_URL))
        self.client = Client(self.cfg, self.md, self.http)
        self.project = self.cfg.get("project-id") or self._md("project/project-id")
        zone = self.cfg.get("local-zone") or _last(self._md("instance/zone"))
        if not self.project or not zone:
            raise ValueError("gce: project-id and the local zone are needed (config or metadata server)")
        self.zone, self.region = zone, region_of_zone(zone)
        self.network_project = self.cfg.get("network-project-id") or self.project
        self.network = self.cfg.get("network-name", "default")
        self.multizone = str(self.cfg.get("multizone", "false")).lower() == "true"
        self.cluster_id = self.cfg.get("cluster-id") or "kubernetes"
        try:
            self.self_name = canonical_instance_name(self.md.get("instance/hostname").strip())
        except Exception:               # noqa: BLE001 — not on GCE (e.g. a controller host)
            self.self_name = ""
        self._zones: list[str] | None = None
        self.instances_ = Instances(self)
        self._routes = Routes(self)
        self._lb = LoadBalancer(self)
        self.volumes_ = Volumes(self)

    def _md(self, path: str) -> str:
        try:
            return self.md.get(path).strip()
        except Exception:               # noqa: BLE001
            return ""

    def network_url(self) -> str:
        return f"{self.client.base}projects/{self.network_project}/global/networks/{self.network}"

    def managed_zones(self) -> list[str]:
        """The local zone, or with multizone every zone of the region."""
        if not self.multizone:
            return [self.zone]
        if self._zones is None:
            r = self.client.call("GET", f"projects/{self.project}/regions/{self.region}")
            self._zones = sorted(_last(z) for z in r.get("zones") or []) or [self.zone]
        return self._zones

    def node_tags(self, hosts: list[dict]) -> list[str]:
        """GetNodeTags: the configured node-tags, else the tags the hosts carry (the
        node-instance-prefix one when several)."""
        if self.cfg["node-tags"]:
            return sorted(self.cfg["node-tags"])
        tags = set()
        prefix = self.cfg.get("node-instance-prefix", "")
        for h in hosts:
            ts = (h.get("tags") or {}).get("items") or []
            pick = [t for t in ts if prefix and t.startswith(prefix)] or ts
            tags.update(pick)
        return sorted(tags)

    def load_balancer(self):
        return self._lb

    def instances(self):
        return self.instances_

    def routes(self):
        return self._routes

    def volumes(self):
        return self.volumes_

    def zones(self):
        return Zone(self.zone, self.region)

    def zone_for_node(self, node_name: str) -> Zone:
        try:
            z = self.instances_.get(node_name)["zone"]
            return Zone(z, region_of_zone(z))
        except Exception:               # noqa: BLE001
            return self.zones()

    def labels_for_volume(self, pv: dict) -> dict:
        src = (pv.get("spec") or {}).get("gcePersistentDisk")
        if not src:
            return {}
        z = self.volumes_.zone(src["pdName"])
        return {"failure-domain.beta.kubernetes.io/zone": z, "failure-domain.beta.kubernetes.io/region": region_of_zone(z)}
