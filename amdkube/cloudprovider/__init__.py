"""Cloud-provider interface and the providers amdkube ships.

Reference: pkg/cloudprovider/cloud.go (Interface: Instances, LoadBalancer, Routes, Zones,
ProviderName, HasClusterID), plugins.go (RegisterCloudProvider / GetCloudProvider by
--cloud-provider name) and providers/fake (the recording fake used by controller tests).

The reference ships AWS / GCE / Azure / vSphere / OpenStack / … drivers; the
fork's README names EC2 and GCP GPU VMs next to on-prem DGX hosts. An MI355X node runs on-prem
(bare metal or an OpenStack cloud) or on a public GPU cloud, so the providers here are:
  * `aws` (cloudprovider/aws.py): EC2 instances/zones/routes, classic ELB, EBS volumes — the
    query APIs spoken directly with Signature V4;
  * `gce` (cloudprovider/gce.py): Compute Engine instances/zones/routes, external load
    balancers (address, firewall, health check, target pool, forwarding rule), persistent disks;
  * `azure` (cloudprovider/azure.py): ARM VMs/NICs, route table, the per-cluster load balancer
    with its NSG rules, managed disks — the cloud that rents AMD Instinct VMs;
  * `openstack` (cloudprovider/openstack.py): Keystone + Nova instances/zones, Neutron router
    routes, Octavia/LBaaS v2 load balancers with floating IPs, Cinder volumes;
  * `cloudstack` (cloudprovider/cloudstack.py): signed query API — VMs, zones, public-IP load
    balancer rules; the virtual router's metadata service without API keys;
  * `ovirt` (cloudprovider/ovirt.py): the engine's VM list (XML) for node addresses and IDs;
  * `photon` (cloudprovider/photon.py): Photon controller VMs, flavors and persistent disks;
  * `vsphere` (cloudprovider/vsphere.py): vCenter over the vim25 SOAP API — VMs by inventory
    path, guest addresses, VMDK create/attach/detach/delete;
  * `baremetal`: load balancers get addresses from a configured pool (the MetalLB model),
    routes are kept in a table and programmed with `ip route` when privileged, and instance
    data comes from the Node objects;
  * `fake`: the reference's recording fake, for tests.
"""
from __future__ import annotations

import asyncio
import functools
import ipaddress
import logging
import os
import shutil
import subprocess
from dataclasses import dataclass

from ..api import meta as m

log = logging.getLogger("amdkube.cloudprovider")


def off_loop(fn):
    """The public-cloud providers speak blocking HTTP (`requests`): their Instances methods are
    awaited by the kubelet and the cloud controllers, so each call runs in a worker thread
    instead of stalling the event loop for a slow cloud API."""
    @functools.wraps(fn)
    async def wrapper(*a, **kw):
        return await asyncio.to_thread(fn, *a, **kw)
    return wrapper


@dataclass(frozen=True)
class Route:
    name: str
    target_node: str
    destination_cidr: str


@dataclass(frozen=True)
class Zone:
    failure_domain: str = ""
    region: str = ""


class Interface:
    """cloud.go Interface. Sub-interfaces return None when unsupported, like the reference's (x, false)."""
    name = "none"

    def initialize(self, client=None):
        pass

    def load_balancer(self):
        return None

    def instances(self):
        return None

    def zones(self):
        return None

    def routes(self):
        return None

    def has_cluster_id(self) -> bool:
        return True


class BareMetalLoadBalancer:
    def __init__(self, pool: str):
        self.pool = [str(ip) for ip in ipaddress.ip_network(pool, strict=False).hosts()] if pool else []
        self.assigned: dict[str, str] = {}   # service key -> ip

    def get(self, cluster: str, svc: dict):
        ip = self.assigned.get(m.key_of(svc))
        return ({"ingress": [{"ip": ip}]}, True) if ip else (None, False)

    def ensure(self, cluster: str, svc: dict, nodes: list[dict]) -> dict:
        key = m.key_of(svc)
        want = (svc.get("spec") or {}).get("loadBalancerIP")
        ip = self.assigned.get(key)
        if want and ip != want:
            if want in self.assigned.values() or (self.pool and want not in self.pool):
                raise ValueError(f"requested loadBalancerIP {want} is unavailable")
            ip = want
        if ip is None:
            used = set(self.assigned.values())
            ip = next((a for a in self.pool if a not in used), None)
            if ip is None:
                raise RuntimeError("load-balancer address pool exhausted")
        self.assigned[key] = ip
        return {"ingress": [{"ip": ip}]}

    def update(self, cluster: str, svc: dict, nodes: list[dict]):
        pass   # addresses are announced by every node's proxy; nothing per-node to program

    def ensure_deleted(self, cluster: str, svc: dict):
        self.assigned.pop(m.key_of(svc), None)


class BareMetalRoutes:
    def __init__(self, program: bool | None = None):
        self.table: dict[str, Route] = {}
        can = shutil.which("ip") is not None and os.geteuid() == 0
        self.program = can if program is None else program
        self.node_ips: dict[str, str] = {}

    def list(self, cluster: str) -> list[Route]:
        return list(self.table.values())

    def create(self, cluster: str, name_hint: str, route: Route):
        if self.program and route.target_node in self.node_ips:
            r = subprocess.run(["ip", "route", "replace", route.destination_cidr, "via", self.node_ips[route.target_node]],
                               capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(r.stderr.strip())
        self.table[route.name] = route

    def delete(self, cluster: str, route: Route):
        if self.program:
            subprocess.run(["ip", "route", "del", route.destination_cidr], capture_output=True)
        self.table.pop(route.name, None)


class BareMetalInstances:
    """cloud.go Instances for on-prem MI355X hosts. With an `instances` inventory in the cloud
    config ({node: {addresses, providerID, instanceType, zone, region}} — what a bare-metal
    provisioner such as an Ironic/Metal3 inventory knows) every answer comes from it and a node
    missing from it does not exist; without one the Node objects are the inventory."""

    def __init__(self, client=None, inventory: dict | None = None):
        self.client = client
        self.inventory = dict(inventory or {})

    async def _node(self, name):
        return await self.client.get_or_none("nodes", name) if self.client else None

    async def node_addresses(self, node_name: str) -> list[dict]:
        if self.inventory:
            inv = self.inventory.get(node_name)
            if inv is None:
                raise LookupError(f"instance {node_name} not found")
            return [dict(a) for a in inv.get("addresses") or []]
        return list((((await self._node(node_name)) or {}).get("status") or {}).get("addresses") or [])

    async def instance_exists(self, node_name: str) -> bool:
        if self.inventory:
            return node_name in self.inventory
        return (await self._node(node_name)) is not None

    async def instance_exists_by_provider_id(self, provider_id: str) -> bool:
        if self.inventory:
            return any(self.provider_id_of(n) == provider_id for n in self.inventory)
        return True

    def provider_id_of(self, node_name: str) -> str:
        inv = self.inventory.get(node_name) or {}
        return inv.get("providerID") or f"baremetal://{node_name}"

    async def instance_id(self, node_name: str) -> str:
        if self.inventory and node_name not in self.inventory:
            raise LookupError(f"instance {node_name} not found")
        return self.provider_id_of(node_name)

    async def instance_type(self, node_name: str) -> str:
        if self.inventory:
            return (self.inventory.get(node_name) or {}).get("instanceType", "amd-mi355x-8gpu")
        n = await self._node(node_name)
        return m.labels_of(n or {}).get("beta.kubernetes.io/instance-type", "amd-mi355x-8gpu")

    def zone_of(self, node_name: str, default: "Zone") -> "Zone":
        inv = self.inventory.get(node_name) or {}
        return Zone(inv.get("zone", default.failure_domain), inv.get("region", default.region))


class BareMetal(Interface):
    name = "baremetal"

    def __init__(self, config: dict | None = None):
        config = config or {}
        self._lb = BareMetalLoadBalancer(config.get("loadBalancerIPRange", ""))
        self._routes = BareMetalRoutes(config.get("programRoutes"))
        self._zone = Zone(config.get("zone", ""), config.get("region", ""))
        self._instances = BareMetalInstances(inventory=config.get("instances"))

    def initialize(self, client=None):
        self._instances.client = client

    def load_balancer(self):
        return self._lb if self._lb.pool else None

    def routes(self):
        return self._routes

    def zones(self):
        return self._zone

    def instances(self):
        return self._instances

    def zone_for_node(self, node_name: str) -> Zone:
        return self._instances.zone_of(node_name, self._zone)

    def labels_for_volume(self, pv: dict) -> dict:
        """PVLabeler: node-local volumes (local, hostPath) carry the cluster's zone/region so the
        scheduler's NoVolumeZoneConflict keeps their pods in the zone."""
        spec = pv.get("spec") or {}
        if not (spec.get("local") or spec.get("hostPath")):
            return {}
        out = {}
        if self._zone.failure_domain:
            out["failure-domain.beta.kubernetes.io/zone"] = self._zone.failure_domain
        if self._zone.region:
            out["failure-domain.beta.kubernetes.io/region"] = self._zone.region
        return out


class Fake(Interface):
    """providers/fake/fake.go: records every call; load balancers get 1.2.3.<n>."""
    name = "fake"

    def __init__(self, config: dict | None = None):
        self.calls: list[str] = []
        self.balancers: dict[str, dict] = {}
        self.route_table: dict[str, Route] = {}
        self.err: Exception | None = None
        outer = self

        class LB:
            def get(self, cluster, svc):
                outer.calls.append("get")
                st = outer.balancers.get(m.key_of(svc))
                return (st, st is not None)

            def ensure(self, cluster, svc, nodes):
                outer.calls.append("create")
                if outer.err:
                    raise outer.err
                st = outer.balancers.get(m.key_of(svc)) or {"ingress": [{"ip": f"1.2.3.{len(outer.balancers) + 1}"}]}
                outer.balancers[m.key_of(svc)] = st
                return st

            def update(self, cluster, svc, nodes):
                outer.calls.append("update")

            def ensure_deleted(self, cluster, svc):
                outer.calls.append("delete")
                outer.balancers.pop(m.key_of(svc), None)

        class Routes:
            def list(self, cluster):
                outer.calls.append("list-routes")
                return list(outer.route_table.values())

            def create(self, cluster, hint, route):
                outer.calls.append("create-route")
                outer.route_table[route.name] = route

            def delete(self, cluster, route):
                outer.calls.append("delete-route")
                outer.route_table.pop(route.name, None)
        self._lb, self._routes = LB(), Routes()
        self._instances = BareMetalInstances(inventory=(config or {}).get("instances") or {})
        self.volume_labels: dict[str, dict] = {}

    def load_balancer(self):
        return self._lb

    def routes(self):
        return self._routes

    def zones(self):
        return Zone("fake-zone", "fake-region")

    def instances(self):
        return self._instances

    def zone_for_node(self, node_name: str) -> Zone:
        return self._instances.zone_of(node_name, Zone("fake-zone", "fake-region"))

    def labels_for_volume(self, pv: dict) -> dict:
        self.calls.append("labels-for-volume")
        return dict(self.volume_labels.get(m.name_of(pv), {}))


def _openstack(config):
    from .openstack import OpenStack
    return OpenStack(config)


def _aws(config):
    from .aws import AWS
    return AWS(config)


def _gce(config):
    from .gce import GCE
    return GCE(config)


def _azure(config):
    from .azure import Azure
    return Azure(config)


def _cloudstack(config):
    from .cloudstack import CloudStack
    return CloudStack(config)


def _ovirt(config):
    from .ovirt import OVirt
    return OVirt(config)


def _photon(config):
    from .photon import Photon
    return Photon(config)


def _vsphere(config):
    from .vsphere import VSphere
    return VSphere(config)


_PROVIDERS = {"baremetal": BareMetal, "fake": Fake, "openstack": _openstack, "aws": _aws, "gce": _gce, "azure": _azure,
              "cloudstack": _cloudstack, "ovirt": _ovirt, "photon": _photon,
              "vsphere": _vsphere}


def load_config(path: str | None):
    """--cloud-config: YAML/JSON, or the reference's INI cloud.conf (returned as text for the
    provider to parse)."""
    if not path:
        return None
    import yaml
    text = open(path).read()
    try:
        data = yaml.safe_load(text)
    except yaml.YAMLError:
        return text
    return data if isinstance(data, dict) else text


def register_cloud_provider(name: str, factory):
    if name in _PROVIDERS:
        raise ValueError(f"cloud provider {name!r} was registered twice")
    _PROVIDERS[name] = factory


def get_cloud_provider(name: str, config: dict | None = None) -> Interface | None:
    if not name:
        return None
    if name not in _PROVIDERS:
        raise ValueError(f"unknown cloud provider {name!r} (have: {', '.join(sorted(_PROVIDERS))})")
    return _PROVIDERS[name](config)
