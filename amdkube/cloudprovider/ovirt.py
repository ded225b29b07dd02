"""oVirt / Red Hat Virtualization cloud provider (reference:
pkg/cloudprovider/providers/ovirt/ovirt.go).

The oVirt engine's REST API lists VMs as XML (`GET <uri>/vms?search=<filter>` with basic auth):
a VM is a node when it is up and its guest agent reports an FQDN, which is the node name; its
first guest IP is both InternalIP and ExternalIP (the engine does not tell them apart), falling
back to a DNS lookup of the name. The instance ID is `/<vm id>` (so providerIDs read
`ovirt:///<vm id>`) and existence by provider ID looks the VM up by id. oVirt has no zones,
load balancers or routes, as in the reference. Config (INI): `[connection] uri, username
(default admin@internal), password`, `[filters] vms` (the engine search query).
"""
from __future__ import annotations

import socket
import xml.etree.ElementTree as ET

from . import Interface, off_loop
from .openstack import parse_config

PROVIDER = "ovirt"


def instances_from_xml(text: str) -> dict[str, dict]:
    """{fqdn: {id, name, ip}} for the VMs that are up and report an FQDN."""
    out = {}
    for vm in ET.fromstring(text).findall("vm"):
        fqdn = (vm.findtext("guest_info/fqdn") or "").strip()
        state = (vm.findtext("status/state") or vm.findtext("status") or "").strip().lower()
        if not fqdn or state != "up":
            continue
        ips = [ip.get("address") for ip in vm.findall("guest_info/ips/ip") if ip.get("address")]
        out[fqdn] = {"id": vm.get("id", ""), "name": vm.findtext("name") or "", "ip": ips[0] if ips else ""}
    return out


class Instances:
    def __init__(self, ov: "OVirt"):
        self.ov = ov

    def all(self, search: str | None = None) -> dict[str, dict]:
        r = self.ov.http.get(self.ov.uri.rstrip("/") + "/vms", params={"search": self.ov.search if search is None else search},
                             auth=(self.ov.username, self.ov.password), headers={"Accept": "application/xml"}, timeout=30)
        if r.status_code != 200:
            raise RuntimeError(f"ovirt: GET vms: HTTP {r.status_code}")
        return instances_from_xml(r.text)

    def get(self, name: str) -> dict:
        inst = self.all().get(name)
        if inst is None:
            raise LookupError(f"cannot find instance: {name}")
        return inst

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        ip = self.get(name)["ip"]
        if not ip:
            try:
                ip = socket.gethostbyname(name)
            except OSError as e:
                raise LookupError(f"couldn't lookup address: {name}") from e
        return [{"type": "InternalIP", "address": ip}, {"type": "ExternalIP", "address": ip}]

    @off_loop
    def instance_exists(self, name: str) -> bool:
        return name in self.all()

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        vid = pid.split("://", 1)[-1].lstrip("/")
        return any(i["id"] == vid for i in self.all().values())

    @off_loop
    def instance_id(self, name: str) -> str:
        return "/" + self.get(name)["id"]

    @off_loop
    def instance_type(self, name: str) -> str:
        return ""


class OVirt(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        if config is None:
            raise ValueError("missing configuration file for ovirt cloud provider")
        cfg = parse_config(config)
        conn, filt = cfg.get("connection") or {}, cfg.get("filters") or {}
        self.uri = conn.get("uri", "")
        if not self.uri:
            raise ValueError("missing ovirt uri in cloud provider configuration")
        self.username, self.password = conn.get("username", "admin@internal"), conn.get("password", "")
        self.search = filt.get("vms", "")
        self.http = session or requests.Session()
        self.instances_ = Instances(self)

    def instances(self):
        return self.instances_
