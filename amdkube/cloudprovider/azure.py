"""The Azure cloud provider: VM instances/zones, route table routes, the shared per-cluster load
balancer with its network security group, managed disks.

Azure is the public cloud that rents AMD Instinct GPU VMs, so an MI355X cluster there needs
this provider. Reference: pkg/cloudprovider/providers/azure —
  * azure.go Config (azure.json: tenantId, subscriptionId, aadClientId/aadClientSecret or
    useManagedIdentityExtension, resourceGroup, location, vnetName/vnetResourceGroup,
    subnetName, securityGroupName, routeTableName, primaryAvailabilitySetName, useInstanceMetadata);
  * azure_instances.go / azure_util.go getIPForMachine: the VM's primary NIC → its primary IP
    configuration's private IP (InternalIP) and public IP (ExternalIP), the node name as
    Hostname; InstanceID = the VM resource ID (providerID `azure://<id>`), InstanceType =
    hardwareProfile.vmSize; azure_zones.go: failure domain = the VM's platformFaultDomain,
    region = location;
  * azure_routes.go: one route table (created on first use), a route per node named after the
    node, nextHopType VirtualAppliance to the node's IP;
  * azure_loadbalancer.go + azure_util.go naming: one load balancer per cluster (`<cluster>`,
    `<cluster>-internal` for service.beta.kubernetes.io/azure-load-balancer-internal), a
    frontend IP configuration per service (`a<uid>`), public IP `<cluster>-a<uid>` (static,
    DNS label from azure-dns-label-name), backend pool `<cluster>` holding the nodes' primary
    IP configurations, one rule + probe per port (`a<uid>-<Proto>-<port>`, floating IP, TCP
    probe on the nodePort or HTTP on healthCheckNodePort), NSG rules
    `a<uid>-<Proto>-<port>-<source>` allowing the sources to the service IP, priorities from 500;
  * azure_managedDiskController.go / azure_controllerCommon.go: managed disks (Standard_LRS /
    Premium_LRS) attached to the VM's dataDisks at the lowest free LUN; the kubelet finds the
    disk by LUN (/dev/disk/azure/scsi1/lun<N>, the udev names of the Azure Linux agent).

Azure Resource Manager is spoken directly (JSON over HTTPS, `api-version` per provider,
long-running operations followed through Azure-AsyncOperation); tokens come from Azure AD
client credentials or the instance's managed identity through the metadata service.
"""
from __future__ import annotations

import json
import logging
import re
import threading
import time

from . import Interface, Route, Zone, off_loop
from ..api import meta as m

log = logging.getLogger("amdkube.cloudprovider.azure")
PROVIDER = "azure"
ARM = "https://management.azure.com/"
AAD = "https://login.microsoftonline.com/"
IMDS = "http://169.254.169.254/metadata/"
API = {"Microsoft.Compute": "2017-12-01", "Microsoft.Network": "2017-09-01", "disks": "2017-03-30"}
ANN_INTERNAL = "service.beta.kubernetes.io/azure-load-balancer-internal"
ANN_INTERNAL_SUBNET = "service.beta.kubernetes.io/azure-load-balancer-internal-subnet"
ANN_DNS_LABEL = "service.beta.kubernetes.io/azure-dns-label-name"
DISK_PROVISIONER = "kubernetes.io/azure-disk"


class AzureError(RuntimeError):
    def __init__(self, status: int, code: str, msg: str):
        super().__init__(f"azure: {code} (HTTP {status}): {msg}")
        self.status, self.code = status, code


def parse_config(cfg) -> dict:
    if isinstance(cfg, str):
        cfg = json.loads(cfg)
    cfg = dict(cfg or {})
    for k in ("subscriptionId", "resourceGroup", "location"):
        if not cfg.get(k):
            raise ValueError(f"azure: {k} is required in the cloud config")
    cfg.setdefault("vnetResourceGroup", cfg["resourceGroup"])
    return cfg


class Client:
    """ARM calls with an Azure AD bearer token (client credentials or managed identity)."""

    def __init__(self, cfg: dict, http):
        self.cfg, self.http = cfg, http
        self.arm = str(cfg.get("resourceManagerEndpoint") or ARM).rstrip("/") + "/"
        self.aad = str(cfg.get("activeDirectoryEndpoint") or AAD).rstrip("/") + "/"
        self.imds = str(cfg.get("instanceMetadataEndpoint") or IMDS).rstrip("/") + "/"
        self.sub, self.rg = cfg["subscriptionId"], cfg["resourceGroup"]
        self._tok, self._exp = "", 0.0
        self._lock = threading.Lock()
        self.poll = 1.0

    def token(self) -> str:
        with self._lock:
            if self._tok and time.time() < self._exp - 60:
                return self._tok
            resource = self.cfg.get("resource", "https://management.azure.com/")
            if self.cfg.get("useManagedIdentityExtension"):
                r = self.http.get(self.imds + "identity/oauth2/token", params={"api-version": "2018-02-01", "resource": resource},
                                  headers={"Metadata": "true"}, timeout=10)
            else:
                r = self.http.post(f"{self.aad}{self.cfg.get('tenantId', '')}/oauth2/token", timeout=10, data={
                    "grant_type": "client_credentials", "client_id": self.cfg.get("aadClientId", ""),
                    "client_secret": self.cfg.get("aadClientSecret", ""), "resource": resource})
            if r.status_code != 200:
                raise AzureError(r.status_code, "AuthenticationFailed", r.text[:200])
            doc = r.json()
            self._tok, self._exp = doc["access_token"], time.time() + float(doc.get("expires_in", 3600))
            return self._tok

    def rid(self, provider: str, kind: str, name: str = "", rg: str | None = None) -> str:
        return f"/subscriptions/{self.sub}/resourceGroups/{rg or self.rg}/providers/{provider}/{kind}" + (f"/{name}" if name else "")

    def call(self, method: str, rid: str, body=None, api: str | None = None, params=None, ok=(200, 201, 202, 204)):
        if api is None:
            api = API["disks"] if "/Microsoft.Compute/disks" in rid else API[rid.split("/providers/", 1)[1].split("/", 1)[0]]
        url = rid if rid.startswith("http") else self.arm + rid.lstrip("/")
        for attempt in (0, 1):
            r = self.http.request(method, url, json=body, params={"api-version": api, **(params or {})}, timeout=60,
                                  headers={"Authorization": f"Bearer {self.token()}"})
            if r.status_code == 401 and attempt == 0:
                with self._lock:
                    self._tok = ""
                continue
            break
        if r.status_code not in ok:
            code, msg = "Unknown", r.text[:300]
            try:
                err = r.json().get("error") or {}
                code, msg = err.get("code", code), err.get("message", msg)
            except ValueError:
                pass
            raise AzureError(r.status_code, code, f"{method} {rid}: {msg}")
        out = r.json() if r.content else {}
        poll = r.headers.get("Azure-AsyncOperation")
        if poll and method in ("PUT", "DELETE", "POST"):
            self._wait(poll)
            if method == "PUT":
                out = self.call("GET", rid, api=api)
        return out

    def _wait(self, url: str, timeout: float = 600):
        deadline = time.monotonic() + timeout
        while True:
            st = self.http.get(url, headers={"Authorization": f"Bearer {self.token()}"}, timeout=30).json()
            if st.get("status") == "Succeeded":
                return
            if st.get("status") in ("Failed", "Canceled"):
                err = st.get("error") or {}
                raise AzureError(409, err.get("code", st["status"]), err.get("message", ""))
            if time.monotonic() > deadline:
                raise AzureError(504, "Timeout", url)
            time.sleep(self.poll)

    def get(self, rid: str) -> dict | None:
        try:
            return self.call("GET", rid)
        except AzureError as e:
            if e.status == 404:
                return None
            raise


def _last(rid: str) -> str:
    return str(rid).rstrip("/").rsplit("/", 1)[-1]


def _primary(items: list[dict]) -> dict:
    if not items:
        raise LookupError("no network interface / IP configuration")
    return next((x for x in items if (x.get("properties") or {}).get("primary")), items[0])


class Instances:
    def __init__(self, az):
        self.az = az

    def vm(self, name: str, view: bool = False) -> dict:
        c = self.az.client
        try:
            return c.call("GET", c.rid("Microsoft.Compute", "virtualMachines", name), params={"$expand": "instanceView"} if view else None)
        except AzureError as e:
            if e.status == 404:
                raise LookupError(f"instance not found: {name}") from None
            raise

    def nic(self, vm: dict) -> dict:
        ref = _primary(((vm.get("properties") or {}).get("networkProfile") or {}).get("networkInterfaces") or [])
        return self.az.client.call("GET", ref["id"])

    def ip_config(self, nic: dict) -> dict:
        return _primary((nic.get("properties") or {}).get("ipConfigurations") or [])

    def ips(self, name: str) -> tuple[str, str]:
        """getIPForMachine: the primary IP configuration's private and public address."""
        ipc = self.ip_config(self.nic(self.vm(name)))
        props = ipc.get("properties") or {}
        pub = ""
        if props.get("publicIPAddress"):
            pip = self.az.client.call("GET", props["publicIPAddress"]["id"])
            pub = (pip.get("properties") or {}).get("ipAddress", "")
        return props.get("privateIPAddress", ""), pub

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        return self._addresses(name)

    def _addresses(self, name: str) -> list[dict]:
        priv, pub = self.ips(name)
        out = [{"type": "InternalIP", "address": priv}, {"type": "Hostname", "address": name}]
        if pub:
            out.append({"type": "ExternalIP", "address": pub})
        return out

    @off_loop
    def node_addresses_by_provider_id(self, pid: str) -> list[dict]:
        return self._addresses(node_name_from_provider_id(pid))

    @off_loop
    def instance_exists(self, name: str) -> bool:
        return self._exists(name)

    def _exists(self, name: str) -> bool:
        try:
            self.vm(name)
            return True
        except LookupError:
            return False

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        return self._exists(node_name_from_provider_id(pid))

    @off_loop
    def instance_id(self, name: str) -> str:
        return self.vm(name)["id"]

    @off_loop
    def instance_type(self, name: str) -> str:
        return ((self.vm(name).get("properties") or {}).get("hardwareProfile") or {}).get("vmSize", "")


def node_name_from_provider_id(pid: str) -> str:
    """splitProviderID: `azure:///subscriptions/…/virtualMachines/<name>` → name."""
    mt = re.fullmatch(r"azure://(/subscriptions/.+/virtualMachines/([^/]+))", pid)
    if not mt:
        raise ValueError(f"error splitting providerID {pid!r}")
    return mt.group(2)


class Routes:
    def __init__(self, az):
        self.az = az

    def _rid(self, name: str = "") -> str:
        c = self.az.client
        base = c.rid("Microsoft.Network", "routeTables", self.az.cfg["routeTableName"])
        return base + (f"/routes/{name}" if name else "")

    def list(self, cluster: str) -> list[Route]:
        t = self.az.client.get(self._rid())
        return [Route(r["name"], r["name"], (r.get("properties") or {}).get("addressPrefix", ""))
                for r in ((t or {}).get("properties") or {}).get("routes") or []]

    def create(self, cluster: str, name_hint: str, route: Route):
        c = self.az.client
        if c.get(self._rid()) is None:
            c.call("PUT", self._rid(), {"location": self.az.location, "properties": {}})
        ip, _ = self.az.instances_.ips(route.target_node)
        c.call("PUT", self._rid(route.target_node), {"name": route.target_node, "properties": {
            "addressPrefix": route.destination_cidr, "nextHopType": "VirtualAppliance", "nextHopIpAddress": ip}})

    def delete(self, cluster: str, route: Route):
        try:
            self.az.client.call("DELETE", self._rid(route.target_node or route.name))
        except AzureError as e:
            if e.status != 404:
                raise


def rule_prefix(svc: dict) -> str:
    """getRulePrefix = cloudprovider.GetLoadBalancerName: "a" + uid without dashes (32 chars)."""
    return ("a" + m.uid_of(svc).replace("-", ""))[:32]


def _internal(svc: dict) -> bool:
    return m.annotations_of(svc).get(ANN_INTERNAL) == "true"


def _safe(prefix: str) -> str:
    return prefix.replace("/", "_").replace(":", ".")


class LoadBalancer:
    def __init__(self, az):
        self.az = az

    def _lb_name(self, cluster: str, svc: dict) -> str:
        return cluster + ("-internal" if _internal(svc) else "")

    def _pip_name(self, cluster: str, svc: dict) -> str:
        return f"{cluster}-{rule_prefix(svc)}"

    def _subnet_id(self, svc: dict) -> str:
        cfg, c = self.az.cfg, self.az.client
        sub = m.annotations_of(svc).get(ANN_INTERNAL_SUBNET) or cfg.get("subnetName", "")
        return c.rid("Microsoft.Network", "virtualNetworks", f"{cfg.get('vnetName', '')}/subnets/{sub}", rg=cfg["vnetResourceGroup"])

    def _frontend_ip(self, lb: dict, fname: str) -> str:
        for f in (lb.get("properties") or {}).get("frontendIPConfigurations") or []:
            if f["name"] != fname:
                continue
            p = f.get("properties") or {}
            if p.get("privateIPAddress"):
                return p["privateIPAddress"]
            if p.get("publicIPAddress"):
                pip = self.az.client.call("GET", p["publicIPAddress"]["id"])
                return (pip.get("properties") or {}).get("ipAddress", "")
        return ""

    def get(self, cluster: str, svc: dict):
        lb = self.az.client.get(self.az.client.rid("Microsoft.Network", "loadBalancers", self._lb_name(cluster, svc)))
        if lb is None:
            return None, False
        ip = self._frontend_ip(lb, rule_prefix(svc))
        return ({"ingress": [{"ip": ip}]}, True) if ip else (None, False)

    def _ensure_pip(self, cluster: str, svc: dict) -> dict:
        c, spec = self.az.client, svc.get("spec") or {}
        want = spec.get("loadBalancerIP", "")
        if want:
            for pip in c.call("GET", c.rid("Microsoft.Network", "publicIPAddresses")).get("value") or []:
                if (pip.get("properties") or {}).get("ipAddress") == want:
                    return pip
            raise LookupError(f"user supplied IP address {want} was not found in resource group {c.rg}")
        name = self._pip_name(cluster, svc)
        props = {"publicIPAllocationMethod": "Static"}
        label = m.annotations_of(svc).get(ANN_DNS_LABEL)
        if label:
            props["dnsSettings"] = {"domainNameLabel": label}
        rid = c.rid("Microsoft.Network", "publicIPAddresses", name)
        have = c.get(rid)
        if have is None or (have.get("properties") or {}).get("dnsSettings", {}).get("domainNameLabel") != label:
            have = c.call("PUT", rid, {"location": self.az.location, "tags": {"service": m.key_of(svc)}, "properties": props})
        return have

    def ensure(self, cluster: str, svc: dict, nodes: list[dict]) -> dict:
        spec, c = svc.get("spec") or {}, self.az.client
        ports = spec.get("ports") or []
        if not ports:
            raise ValueError("requested load balancer with no ports")
        prefix, internal = rule_prefix(svc), _internal(svc)
        lb_rid = c.rid("Microsoft.Network", "loadBalancers", self._lb_name(cluster, svc))
        lb = c.get(lb_rid) or {"location": self.az.location, "properties": {}}
        props = lb.setdefault("properties", {})
        # frontend
        if internal:
            fprops = {"subnet": {"id": self._subnet_id(svc)}, "privateIPAllocationMethod": "Dynamic"}
            if spec.get("loadBalancerIP"):
                fprops.update(privateIPAllocationMethod="Static", privateIPAddress=spec["loadBalancerIP"])
        else:
            fprops = {"publicIPAddress": {"id": self._ensure_pip(cluster, svc)["id"]}}
        fronts = [f for f in props.get("frontendIPConfigurations") or [] if f["name"] != prefix]
        old = next((f for f in props.get("frontendIPConfigurations") or [] if f["name"] == prefix), None)
        if old is not None and internal and not spec.get("loadBalancerIP") and (old.get("properties") or {}).get("privateIPAddress"):
            fprops.setdefault("privateIPAddress", old["properties"]["privateIPAddress"])
        fronts.append({"name": prefix, "properties": fprops})
        props["frontendIPConfigurations"] = fronts
        # backend pool
        pool = cluster
        pools = props.get("backendAddressPools") or []
        if not any(p["name"] == pool for p in pools):
            pools.append({"name": pool})
        props["backendAddressPools"] = pools
        # rules + probes
        front_id, pool_id = f"{lb_rid}/frontendIPConfigurations/{prefix}", f"{lb_rid}/backendAddressPools/{pool}"
        local_hc = spec.get("externalTrafficPolicy") == "Local" and spec.get("healthCheckNodePort")
        rules = [r for r in props.get("loadBalancingRules") or [] if not r["name"].startswith(prefix + "-")]
        probes = [p for p in props.get("probes") or [] if not p["name"].startswith(prefix + "-")]
        for p in ports:
            proto = p.get("protocol", "TCP")
            name = f"{prefix}-{proto}-{p['port']}"
            if local_hc:
                probe = {"protocol": "Http", "port": int(spec["healthCheckNodePort"]), "requestPath": "/healthz"}
            else:
                probe = {"protocol": "Tcp", "port": int(p.get("nodePort") or p["port"])}
            probes.append({"name": name, "properties": {**probe, "intervalInSeconds": 5, "numberOfProbes": 2}})
            rules.append({"name": name, "properties": {
                "protocol": "Udp" if proto == "UDP" else "Tcp", "frontendPort": int(p["port"]), "backendPort": int(p["port"]),
                "enableFloatingIP": True, "idleTimeoutInMinutes": 4,
                "loadDistribution": "SourceIP" if spec.get("sessionAffinity") == "ClientIP" else "Default",
                "frontendIPConfiguration": {"id": front_id}, "backendAddressPool": {"id": pool_id},
                "probe": {"id": f"{lb_rid}/probes/{name}"}}})
        props["loadBalancingRules"], props["probes"] = rules, probes
        lb = c.call("PUT", lb_rid, lb)
        ip = self._frontend_ip(lb, prefix)
        self._pool_members(pool_id, nodes)
        self._nsg(svc, ip, ports, spec.get("loadBalancerSourceRanges") or (["*"] if internal else ["Internet"]), want=True)
        return {"ingress": [{"ip": ip}]}

    def _pool_members(self, pool_id: str, nodes: list[dict], remove_others: bool = False):
        """ensureHostInPool: each node's primary IP configuration joins the backend pool."""
        c, inst = self.az.client, self.az.instances_
        for n in nodes:
            try:
                nic = inst.nic(inst.vm(m.name_of(n)))
            except LookupError:
                continue
            ipc = inst.ip_config(nic)
            pools = (ipc.setdefault("properties", {})).setdefault("loadBalancerBackendAddressPools", [])
            if not any(p.get("id", "").lower() == pool_id.lower() for p in pools):
                pools.append({"id": pool_id})
                c.call("PUT", nic["id"], nic)

    def _nsg(self, svc: dict, ip: str, ports: list[dict], sources: list[str], want: bool):
        cfg, c = self.az.cfg, self.az.client
        if not cfg.get("securityGroupName"):
            return
        rid = c.rid("Microsoft.Network", "networkSecurityGroups", cfg["securityGroupName"])
        nsg = c.get(rid)
        if nsg is None:
            return
        prefix = rule_prefix(svc)
        rules = (nsg.setdefault("properties", {})).get("securityRules") or []
        mine = [r for r in rules if r["name"].startswith(prefix + "-")]
        keep = [r for r in rules if not r["name"].startswith(prefix + "-")]
        wanted = []
        if want:
            used = {int((r.get("properties") or {}).get("priority", 0)) for r in keep}
            have = {r["name"]: r for r in mine}
            for p in ports:
                proto = p.get("protocol", "TCP")
                for src in sources:
                    name = f"{prefix}-{proto}-{p['port']}-{_safe(src)}"
                    pri = int(((have.get(name) or {}).get("properties") or {}).get("priority", 0))
                    if not pri or pri in used:
                        pri = next(x for x in range(500, 4097) if x not in used)
                    used.add(pri)
                    wanted.append({"name": name, "properties": {
                        "protocol": "Udp" if proto == "UDP" else "Tcp", "sourcePortRange": "*",
                        "destinationPortRange": str(p["port"]), "sourceAddressPrefix": src,
                        "destinationAddressPrefix": ip or "*", "access": "Allow", "direction": "Inbound", "priority": pri}})
        if sorted(json.dumps(r, sort_keys=True) for r in mine) == sorted(json.dumps(r, sort_keys=True) for r in wanted):
            return
        nsg["properties"]["securityRules"] = keep + wanted
        c.call("PUT", rid, nsg)

    def update(self, cluster: str, svc: dict, nodes: list[dict]):
        c = self.az.client
        lb_rid = c.rid("Microsoft.Network", "loadBalancers", self._lb_name(cluster, svc))
        self._pool_members(f"{lb_rid}/backendAddressPools/{cluster}", nodes)

    def ensure_deleted(self, cluster: str, svc: dict):
        c, prefix = self.az.client, rule_prefix(svc)
        lb_rid = c.rid("Microsoft.Network", "loadBalancers", self._lb_name(cluster, svc))
        lb = c.get(lb_rid)
        if lb is not None:
            props = lb.get("properties") or {}
            props["frontendIPConfigurations"] = [f for f in props.get("frontendIPConfigurations") or [] if f["name"] != prefix]
            props["loadBalancingRules"] = [r for r in props.get("loadBalancingRules") or [] if not r["name"].startswith(prefix + "-")]
            props["probes"] = [p for p in props.get("probes") or [] if not p["name"].startswith(prefix + "-")]
            if props["frontendIPConfigurations"]:
                c.call("PUT", lb_rid, lb)
            else:
                # the last service on the LB: members leave the pool, then the LB goes
                pool_id = f"{lb_rid}/backendAddressPools/{cluster}".lower()
                for ipc_ref in [ip for p in props.get("backendAddressPools") or []
                                for ip in ((p.get("properties") or {}).get("backendIPConfigurations") or [])]:
                    nic_id = ipc_ref["id"].split("/ipConfigurations/", 1)[0]
                    nic = c.get(nic_id)
                    if nic is None:
                        continue
                    for ipc in (nic.get("properties") or {}).get("ipConfigurations") or []:
                        ps = ipc.get("properties") or {}
                        ps["loadBalancerBackendAddressPools"] = [x for x in ps.get("loadBalancerBackendAddressPools") or []
                                                                 if x.get("id", "").lower() != pool_id]
                    c.call("PUT", nic_id, nic)
                c.call("DELETE", lb_rid)
        self._nsg(svc, "", [], [], want=False)
        if not _internal(svc) and not (svc.get("spec") or {}).get("loadBalancerIP"):
            try:
                c.call("DELETE", c.rid("Microsoft.Network", "publicIPAddresses", self._pip_name(cluster, svc)))
            except AzureError as e:
                if e.status != 404:
                    raise


class Volumes:
    """Managed disks (azure_managedDiskController.go, azure_controllerCommon.go)."""
    provisioner = DISK_PROVISIONER
    source_key = "azureDisk"
    max_luns = 64

    def __init__(self, az):
        self.az = az
        self.lock = threading.Lock()

    def _rid(self, name: str) -> str:
        return self.az.client.rid("Microsoft.Compute", "disks", name)

    def create(self, name: str, size_gib: int, sku: str = "Standard_LRS", tags: dict | None = None) -> dict:
        if sku not in ("Standard_LRS", "Premium_LRS"):
            raise ValueError(f"azureDisk - {sku} is not a supported storage account type")
        return self.az.client.call("PUT", self._rid(name), {
            "location": self.az.location, "tags": {k.replace("/", "-"): v for k, v in (tags or {}).items()},
            "sku": {"name": sku}, "properties": {"creationData": {"createOption": "Empty"}, "diskSizeGB": size_gib}})

    def delete(self, uri: str) -> bool:
        d = self.az.client.get(uri)
        if d is None:
            return False
        if d.get("managedBy") or (d.get("properties") or {}).get("diskState") == "Attached":
            raise AzureError(409, "OperationNotAllowed", f"disk {_last(uri)} is attached to {d.get('managedBy')}")
        self.az.client.call("DELETE", uri)
        return True

    def attach(self, node: str, uri: str, caching: str = "ReadOnly") -> str:
        """AttachDisk: the lowest free LUN of the VM's dataDisks; returns the LUN."""
        c = self.az.client
        with self.lock:
            vm = self.az.instances_.vm(node)
            disks = ((vm.setdefault("properties", {})).setdefault("storageProfile", {})).setdefault("dataDisks", [])
            for d in disks:
                if ((d.get("managedDisk") or {}).get("id", "")).lower() == uri.lower():
                    return str(d["lun"])
            used = {int(d["lun"]) for d in disks}
            lun = next((x for x in range(self.max_luns) if x not in used), None)
            if lun is None:
                raise AzureError(409, "NoFreeLun", f"all {self.max_luns} LUNs of {node} are in use")
            disks.append({"lun": lun, "name": _last(uri), "createOption": "Attach", "caching": caching,
                          "managedDisk": {"id": uri}})
            vm.get("properties", {}).pop("instanceView", None)
            c.call("PUT", vm["id"], {"location": vm.get("location"), "properties": {"storageProfile": vm["properties"]["storageProfile"]}})
            return str(lun)

    def detach(self, node: str, uri: str):
        c = self.az.client
        with self.lock:
            try:
                vm = self.az.instances_.vm(node)
            except LookupError:
                return
            sp = (vm.get("properties") or {}).get("storageProfile") or {}
            disks = sp.get("dataDisks") or []
            keep = [d for d in disks if ((d.get("managedDisk") or {}).get("id", "")).lower() != uri.lower()
                    and d.get("name") != _last(uri)]
            if len(keep) == len(disks):
                return
            sp["dataDisks"] = keep
            c.call("PUT", vm["id"], {"location": vm.get("location"), "properties": {"storageProfile": sp}})

    def device_candidates(self, uri: str, lun: str = "") -> list[str]:
        """findDiskByLun: the agent's udev links for data disks, by LUN."""
        return [f"/dev/disk/azure/scsi1/lun{lun}"] if lun != "" else []

    def provision(self, name: str, gib: int, params: dict, tags: dict, pvc_name: str) -> tuple[dict, dict]:
        p = {str(k).lower(): v for k, v in params.items()}
        kind = p.get("kind", "Managed")
        if kind.lower() != "managed":
            raise ValueError(f"azureDisk kind {kind!r} needs blob storage accounts; only kind: Managed is supported")
        sku = p.get("skuname") or p.get("storageaccounttype") or "Standard_LRS"
        dname = f"kubernetes-dynamic-{name}"
        d = self.create(dname, gib, sku, tags)
        return ({"diskName": dname, "diskURI": d["id"], "kind": "Managed", "cachingMode": p.get("cachingmode", "ReadOnly"),
                 "fsType": p.get("fstype", "ext4")}, {"failure-domain.beta.kubernetes.io/region": self.az.location})

    def delete_source(self, src: dict):
        self.delete(src["diskURI"])


class Azure(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        self.cfg = parse_config(config)
        self.http = session or requests.Session()
        self.client = Client(self.cfg, self.http)
        self.location = self.cfg["location"]
        self.instances_ = Instances(self)
        self._routes = Routes(self) if self.cfg.get("routeTableName") else None
        self._lb = LoadBalancer(self)
        self.volumes_ = Volumes(self)

    def load_balancer(self):
        return self._lb

    def instances(self):
        return self.instances_

    def routes(self):
        return self._routes

    def volumes(self):
        return self.volumes_

    def zones(self):
        """GetZone: this VM's fault domain from the instance metadata service."""
        try:
            r = self.http.get(self.client.imds + "instance/compute", params={"api-version": "2017-08-01"},
                              headers={"Metadata": "true"}, timeout=5)
            fd = str(r.json().get("platformFaultDomain", "")) if r.status_code == 200 else ""
        except Exception:               # noqa: BLE001
            fd = ""
        return Zone(fd, self.location)

    def zone_for_node(self, node_name: str) -> Zone:
        try:
            vm = self.instances_.vm(node_name, view=True)
        except Exception:               # noqa: BLE001
            return self.zones()
        fd = ((vm.get("properties") or {}).get("instanceView") or {}).get("platformFaultDomain")
        return Zone("" if fd is None else str(fd), vm.get("location", self.location))

    def labels_for_volume(self, pv: dict) -> dict:
        return {}
