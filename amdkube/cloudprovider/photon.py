"""VMware Photon Platform cloud provider (reference: pkg/cloudprovider/providers/photon/photon.go)
and the volumes behind the photonPersistentDisk plugin (pkg/volume/photon_pd).

The Photon controller's REST API (`<target>/…`, optional bearer token from
`POST /auth/tokens`-style password login, done here with the configured token endpoint):
  * VMs of the one configured project: `GET /projects/{p}/vms`; a VM's addresses come from
    `GET /vms/{id}/subnets`, a task whose result lists network connections — the address on
    a NIC whose MAC has a vCenter/ESX OUI (00:50:56 / 00:0c:29) is the ExternalIP, the others
    InternalIPs (photon.go's MAC filter). With `overrideIP`, node names are IP addresses and
    VMs are found by address.
  * Instance ID = VM id; instance type = the VM's flavor. Zones are the configured ones.
  * Persistent disks: `POST /projects/{p}/disks` (kind persistent-disk, flavor, capacityGb),
    `POST /vms/{id}/attach_disk` / `detach_disk` with {diskId}, `DELETE /disks/{id}`; every
    mutation is a task polled at `GET /tasks/{id}` until COMPLETED or ERROR. An attached disk
    appears as `/dev/disk/by-id/wwn-0x<disk id without dashes>` (photon_util.go).
"""
from __future__ import annotations

import time

from . import Interface, Zone, off_loop
from .openstack import parse_config

PROVIDER = "photon"
PD_PROVISIONER = "kubernetes.io/photon-pd"
MAC_OUI_VC, MAC_OUI_ESX = "00:50:56", "00:0c:29"


class PhotonError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"photon: HTTP {status}: {msg}")
        self.status = status


class Client:
    def __init__(self, target: str, http, token: str = ""):
        self.base, self.http, self.token = target.rstrip("/"), http, token

    def call(self, method: str, path: str, body=None) -> dict:
        h = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        r = self.http.request(method, self.base + path, json=body, headers=h, timeout=30)
        if r.status_code >= 400:
            raise PhotonError(r.status_code, r.text[:200])
        return r.json() if r.content else {}

    def wait(self, task: dict, timeout: float = 300) -> dict:
        end, delay = time.monotonic() + timeout, 0.05
        while True:
            if task.get("state") == "COMPLETED":
                return task
            if task.get("state") == "ERROR":
                errs = "; ".join(e.get("message", "") for e in task.get("errors") or []) or "task failed"
                raise PhotonError(500, f"task {task.get('id')} ({task.get('operation')}): {errs}")
            if time.monotonic() > end:
                raise TimeoutError(f"photon task {task.get('id')} did not finish in {timeout}s")
            time.sleep(delay)
            delay = min(delay * 2, 2.0)
            task = self.call("GET", f"/tasks/{task['id']}")

    def mutate(self, method: str, path: str, body=None) -> dict:
        return self.wait(self.call(method, path, body))


def _addresses_of(conns: list[dict]) -> list[dict]:
    out = []
    for c in conns:
        ip, mac = c.get("ipAddress") or "", (c.get("macAddress") or "").lower()
        if not ip or ip.startswith("127.") or ":" in ip:
            continue
        ext = mac.startswith(MAC_OUI_VC) or mac.startswith(MAC_OUI_ESX)
        out.append({"type": "ExternalIP" if ext else "InternalIP", "address": ip})
    return out


class Instances:
    def __init__(self, pc: "Photon"):
        self.pc = pc

    def vms(self) -> list[dict]:
        return self.pc.client.call("GET", f"/projects/{self.pc.project}/vms").get("items") or []

    def networks(self, vm_id: str) -> list[dict]:
        task = self.pc.client.wait(self.pc.client.call("GET", f"/vms/{vm_id}/subnets"))
        return ((task.get("resourceProperties") or {}).get("networkConnections")) or []

    def vm_id(self, name: str) -> str:
        if self.pc.override_ip:
            for vm in self.vms():
                if any(a["address"] == name for a in _addresses_of(self.networks(vm["id"]))):
                    return vm["id"]
        else:
            for vm in self.vms():
                if vm.get("name") == name:
                    return vm["id"]
        raise LookupError(f"no Photon VM for node {name}")

    def vm(self, vm_id: str) -> dict | None:
        try:
            return self.pc.client.call("GET", f"/vms/{vm_id}")
        except PhotonError as e:
            if e.status == 404:
                return None
            raise

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        return _addresses_of(self.networks(self.vm_id(name)))

    @off_loop
    def node_addresses_by_provider_id(self, pid: str) -> list[dict]:
        return _addresses_of(self.networks(pid.split("://", 1)[-1].lstrip("/")))

    @off_loop
    def instance_exists(self, name: str) -> bool:
        try:
            self.vm_id(name)
            return True
        except LookupError:
            return False

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        return self.vm(pid.split("://", 1)[-1].lstrip("/")) is not None

    @off_loop
    def instance_id(self, name: str) -> str:
        return self.vm_id(name)

    @off_loop
    def instance_type(self, name: str) -> str:
        return (self.vm(self.vm_id(name)) or {}).get("flavor", "")


class Volumes:
    provisioner = PD_PROVISIONER
    source_key = "photonPersistentDisk"

    def __init__(self, pc: "Photon"):
        self.pc = pc

    def disk(self, pd_id: str) -> dict | None:
        try:
            return self.pc.client.call("GET", f"/disks/{pd_id}")
        except PhotonError as e:
            if e.status == 404:
                return None
            raise

    def attach(self, node: str, pd_id: str) -> str:
        vm = self.pc.instances_.vm_id(node)
        d = self.disk(pd_id)
        if d is None:
            raise LookupError(f"photon disk {pd_id} not found")
        if vm not in (d.get("vms") or []):
            self.pc.client.mutate("POST", f"/vms/{vm}/attach_disk", {"diskId": pd_id})
        return self.device_candidates(pd_id)[0]

    def detach(self, node: str, pd_id: str):
        try:
            vm = self.pc.instances_.vm_id(node)
        except LookupError:
            return
        d = self.disk(pd_id)
        if d is not None and vm in (d.get("vms") or []):
            self.pc.client.mutate("POST", f"/vms/{vm}/detach_disk", {"diskId": pd_id})

    def device_candidates(self, pd_id: str, device_path: str = "") -> list[str]:
        return [f"/dev/disk/by-id/wwn-0x{pd_id.replace('-', '')}"]

    def create(self, name: str, gib: int, flavor: str) -> str:
        task = self.pc.client.mutate("POST", f"/projects/{self.pc.project}/disks",
                                     {"name": name, "kind": "persistent-disk", "flavor": flavor, "capacityGb": gib})
        return (task.get("entity") or {}).get("id", "")

    def delete(self, pd_id: str):
        d = self.disk(pd_id)
        if d is None:
            return
        if d.get("vms"):
            raise PhotonError(409, f"disk {pd_id} is attached to {d['vms']}")
        self.pc.client.mutate("DELETE", f"/disks/{pd_id}")

    def provision(self, name: str, gib: int, params: dict, tags: dict, pvc_name: str) -> tuple[dict, dict]:
        p = {str(k).lower(): v for k, v in params.items()}
        pd_id = self.create(f"kubernetes-dynamic-{name}", gib, p.get("flavor", "default"))
        z = self.pc.zones()
        labels = {}
        if z.failure_domain:
            labels["failure-domain.beta.kubernetes.io/zone"] = z.failure_domain
        return {"pdID": pd_id, "fsType": p.get("fstype", "ext4")}, labels

    def delete_source(self, src: dict):
        self.delete(src["pdID"])


class Photon(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        g = parse_config(config).get("global") or {}
        if not g.get("target") or not g.get("project"):
            raise ValueError("photon: target and project are required in the cloud config")
        self.http = session or requests.Session()
        if str(g.get("ignorecertificate", "")).lower() == "true":
            self.http.verify = False
        token = g.get("token", "")
        if not token and g.get("username"):
            r = self.http.post(g["target"].rstrip("/") + "/auth/tokens", timeout=30,
                               json={"username": g["username"], "password": g.get("password", "")})
            if r.status_code >= 400:
                raise PhotonError(r.status_code, "authentication failed")
            token = r.json().get("access_token", "")
        self.client = Client(g["target"], self.http, token)
        self.project = g["project"]
        self.override_ip = str(g.get("overrideip", "")).lower() == "true"
        self.zone = Zone(g.get("zone", ""), g.get("region", ""))
        self.instances_ = Instances(self)
        self.volumes_ = Volumes(self)

    def instances(self):
        return self.instances_

    def volumes(self):
        return self.volumes_

    def zones(self):
        return self.zone

    def zone_for_node(self, node_name: str) -> Zone:
        return self.zone
