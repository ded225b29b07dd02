"""OpenStack cloud provider and Cinder volumes (reference: pkg/cloudprovider/providers/openstack
openstack_test.go, openstack_routes_test.go, openstack_loadbalancer.go, openstack_volumes.go;
pkg/volume/cinder attacher_test.go), against the in-repo fake OpenStack (tests/fake_openstack.py):
no OpenStack exists offline, so parity with a real cloud is unpinned; the REST shapes follow the
public Nova / Neutron / Octavia / Cinder / Keystone v3 APIs."""
import asyncio

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.cloudprovider import Route, get_cloud_provider
from amdkube.cloudprovider.openstack import instance_id_from_provider_id, lb_name, node_addresses
from amdkube.controllers import ControllerManager, Options
from amdkube.localcluster import LocalCluster
from tests.fake_openstack import FakeOpenStack


@pytest.fixture()
def cloud():
    f = FakeOpenStack().start()
    f.add_router()
    try:
        yield f
    finally:
        f.stop()


def test_instances_addresses_zones_and_reauth(cloud):
    sid = cloud.add_server("gpu-node-1", "10.0.0.11", floating_ip="203.0.113.50", az="az-2")
    os_ = get_cloud_provider("openstack", cloud.config())
    inst = os_.instances()

    async def go():
        addrs = await inst.node_addresses("gpu-node-1")
        assert addrs == [{"type": "InternalIP", "address": "10.0.0.11"}, {"type": "ExternalIP", "address": "203.0.113.50"}]
        pid = await inst.instance_id("gpu-node-1")
        assert pid == f"openstack:///{sid}" and instance_id_from_provider_id(pid) == sid
        assert await inst.instance_type("gpu-node-1") == "gpu.mi355x.8x"
        assert await inst.instance_exists("gpu-node-1") and not await inst.instance_exists("nope")
        assert not await inst.instance_exists_by_provider_id("openstack:///gone")
        z = os_.zone_for_node("gpu-node-1")
        assert (z.failure_domain, z.region) == ("az-2", "RegionOne")
        # an expired token is renewed once, transparently
        cloud.tokens.clear()
        assert await inst.instance_exists("gpu-node-1") and cloud.auth_calls == 2
    asyncio.run(go())
    with pytest.raises(ValueError):
        instance_id_from_provider_id("aws:///i-1")
    # "public" network and accessIPv4 count as external
    assert node_addresses({"addresses": {"public": [{"addr": "198.51.100.1"}]}, "accessIPv4": "198.51.100.2"}) == [
        {"type": "ExternalIP", "address": "198.51.100.1"}, {"type": "ExternalIP", "address": "198.51.100.2"}]


def test_ini_cloud_conf_and_routes_with_unwind(cloud, tmp_path):
    sid = cloud.add_server("gpu-node-1", "10.0.0.11")
    conf = tmp_path / "cloud.conf"
    conf.write_text(f"[Global]\nauth-url = {cloud.url}/identity/v3\nusername = admin\npassword = secret\n"
                    f"tenant-id = {cloud.project}\nregion = RegionOne\n\n[Route]\nrouter-id = router-1\n")
    from amdkube.cloudprovider import load_config
    os_ = get_cloud_provider("openstack", load_config(str(conf)))
    assert os_.load_balancer() is None                 # no [LoadBalancer] subnet-id: no LB support
    rt = os_.routes()
    r = Route("k-1", "gpu-node-1", "10.244.1.0/24")
    rt.create("kubernetes", "k-1", r)
    assert cloud.routers["router-1"]["routes"] == [{"destination": "10.244.1.0/24", "nexthop": "10.0.0.11"}]
    port = next(p for p in cloud.ports.values() if p["device_id"] == sid)
    assert port["allowed_address_pairs"] == [{"ip_address": "10.244.1.0/24"}]
    assert [(x.target_node, x.destination_cidr) for x in rt.list("kubernetes")] == [("gpu-node-1", "10.244.1.0/24")]
    rt.delete("kubernetes", r)
    assert cloud.routers["router-1"]["routes"] == [] and port["allowed_address_pairs"] == []
    # the port update fails: the router change is unwound (openstack_routes.go onFailure)
    cloud.fail_next["PUT /network/v2.0/ports/"] = 500
    with pytest.raises(Exception):
        rt.create("kubernetes", "k-2", Route("k-2", "gpu-node-1", "10.244.2.0/24"))
    assert cloud.routers["router-1"]["routes"] == []


def _svc(ports, uid="0f9a2c3e-1111-2222-3333-444455556666"):
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "inference", "namespace": "ml", "uid": uid},
            "spec": {"type": "LoadBalancer", "ports": [{"port": p, "nodePort": np, "protocol": "TCP"} for p, np in ports]}}


def _node(name, ip):
    return {"metadata": {"name": name}, "status": {"addresses": [{"type": "InternalIP", "address": ip}],
                                                   "conditions": [{"type": "Ready", "status": "True"}]}}


def test_load_balancer_lifecycle(cloud):
    os_ = get_cloud_provider("openstack", cloud.config(**{"create-monitor": "true"}))
    lb = os_.load_balancer()
    svc = _svc([(80, 30080), (443, 30443)])
    st = lb.ensure("kubernetes", svc, [_node("n1", "10.0.0.11"), _node("n2", "10.0.0.12")])
    [obj] = cloud.lbs.values()
    assert obj["name"] == lb_name(svc) == "a0f9a2c3e111122223333444455556666"[:32]
    assert obj["vip_subnet_id"] == "subnet-1"
    assert sorted(x["protocol_port"] for x in cloud.listeners.values()) == [80, 443]
    assert sorted((x["address"], x["protocol_port"]) for x in cloud.members.values()) == [
        ("10.0.0.11", 30080), ("10.0.0.11", 30443), ("10.0.0.12", 30080), ("10.0.0.12", 30443)]
    assert len(cloud.monitors) == 2
    [fip] = cloud.fips.values()
    assert st == {"ingress": [{"ip": fip["floating_ip_address"]}]} and fip["port_id"] == obj["vip_port_id"]
    assert lb.get("kubernetes", svc) == (st, True)
    # node churn: members follow the ready nodes
    lb.update("kubernetes", svc, [_node("n2", "10.0.0.12"), _node("n3", "10.0.0.13")])
    assert sorted({x["address"] for x in cloud.members.values()}) == ["10.0.0.12", "10.0.0.13"]
    # a port leaves the service: its listener, pool, monitor and members go
    lb.ensure("kubernetes", _svc([(80, 30080)]), [_node("n2", "10.0.0.12")])
    assert [x["protocol_port"] for x in cloud.listeners.values()] == [80] and len(cloud.pools) == 1
    assert [(x["address"], x["protocol_port"]) for x in cloud.members.values()] == [("10.0.0.12", 30080)]
    with pytest.raises(ValueError):
        lb.ensure("kubernetes", {**_svc([(53, 30053)]), "spec": {"type": "LoadBalancer", "ports": [
            {"port": 53, "nodePort": 30053, "protocol": "UDP"}]}}, [])
    lb.ensure_deleted("kubernetes", svc)
    assert not (cloud.lbs or cloud.listeners or cloud.pools or cloud.members or cloud.monitors or cloud.fips)
    assert lb.get("kubernetes", svc) == (None, False)


def test_cinder_provision_attach_mount_detach(cloud, tmp_path):
    """The Cinder plugin's attach half over the provider, device discovery by serial, and the
    provisioner creating / deleting the volume with zone labels."""
    from amdkube.volume import NoopMounter, PluginMgr, Spec, VolumeHost, default_plugins
    sid = cloud.add_server("gpu-node-1", "10.0.0.11")
    dev_root = tmp_path / "root"

    def on_attach(srv, v):          # the guest sees the disk under its serial
        d = dev_root / "dev" / "disk" / "by-id"
        d.mkdir(parents=True, exist_ok=True)
        (d / f"virtio-{v['id'][:20]}").write_text("")
    cloud.on_attach = on_attach
    os_ = get_cloud_provider("openstack", cloud.config())
    os_.volumes().poll = 0.01
    vol = os_.volumes().create("kubernetes-dynamic-pvc-1", 100, zone="az-gpu")
    host = VolumeHost(str(tmp_path / "kubelet"), node_name="gpu-node-1", mounter=NoopMounter())
    host.cloud, host.dev_root, host.attach_poll = os_, str(dev_root), 0.01
    mgr = PluginMgr(default_plugins(), host)
    pv = {"metadata": {"name": "pv-1"}, "spec": {"cinder": {"volumeID": vol["id"], "fsType": "ext4"}}}
    spec = Spec(pv=pv)
    plugin = mgr.find_by_spec(spec)
    assert plugin.name == "kubernetes.io/cinder" and plugin.unique_name(spec, "u") == f"kubernetes.io/cinder/{vol['id']}"

    async def go():
        dev = await plugin.attach(spec, "gpu-node-1")
        assert dev == "/dev/vdb" and cloud.volumes[vol["id"]]["attachments"][0]["server_id"] == sid
        found = await plugin.wait_for_attach(spec, dev, None, 5)
        assert found == str(dev_root / "dev" / "disk" / "by-id" / f"virtio-{vol['id'][:20]}")
        await plugin.detach(vol["id"], "gpu-node-1")
        assert cloud.volumes[vol["id"]]["status"] == "available"
    asyncio.run(go())
    assert os_.labels_for_volume(pv) == {"failure-domain.beta.kubernetes.io/region": "RegionOne",
                                         "failure-domain.beta.kubernetes.io/zone": "az-gpu"}
    os_.volumes().delete(vol["id"])
    assert vol["id"] not in cloud.volumes


def test_controllers_drive_openstack(cloud):
    """service-LB, route and PV-binder controllers against the provider: a LoadBalancer service
    gets the floating IP, each node's podCIDR becomes a router route, a Cinder StorageClass
    claim is provisioned as a labelled Cinder PV and its volume deleted with the claim."""
    from tests.conftest import run

    async def go():
        async with LocalCluster(gpus="none", with_controllers=False, with_kubelet=False) as lc:
            c = lc.client
            os_ = get_cloud_provider("openstack", cloud.config())
            os_.volumes().poll = 0.01
            cloud.add_server("gpu-node-1", "10.0.0.11")
            await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "gpu-node-1"},
                            "spec": {"podCIDR": "10.244.7.0/24"},
                            "status": {"addresses": [{"type": "InternalIP", "address": "10.0.0.11"}],
                                       "conditions": [{"type": "Ready", "status": "True"}]}})
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default"},
                            "spec": {"type": "LoadBalancer", "ports": [{"port": 80, "protocol": "TCP"}]}}, "default")
            await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": "cinder"},
                            "provisioner": "kubernetes.io/cinder", "parameters": {"availability": "az-gpu"}})
            await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data", "namespace": "default"},
                            "spec": {"storageClassName": "cinder", "accessModes": ["ReadWriteOnce"],
                                     "resources": {"requests": {"storage": "1536Mi"}}}}, "default")
            cmc = Client(lc.api.url, token=lc.api.loopback_token)
            cm = await ControllerManager(cmc,
                                         ["service", "route", "persistentvolume-binder", "pvc-protection", "pv-protection"],
                                         options=Options(cloud=os_, cluster_name="kubernetes")).start()
            try:
                async def until(fn, t=20):
                    end = asyncio.get_running_loop().time() + t
                    while asyncio.get_running_loop().time() < end:
                        v = await fn()
                        if v:
                            return v
                        await asyncio.sleep(0.05)
                    raise AssertionError("condition not met")

                async def lb_ip():
                    s = await c.get("services", "web", "default")
                    return ((s.get("status") or {}).get("loadBalancer") or {}).get("ingress")
                ing = await until(lb_ip)
                assert ing[0]["ip"] == next(iter(cloud.fips.values()))["floating_ip_address"]

                async def routed():
                    return cloud.routers["router-1"]["routes"]
                assert await until(routed) == [{"destination": "10.244.7.0/24", "nexthop": "10.0.0.11"}]

                async def bound():
                    p = await c.get("persistentvolumeclaims", "data", "default")
                    return p if (p.get("status") or {}).get("phase") == "Bound" else None
                pvc = await until(bound)
                pv = await c.get("persistentvolumes", pvc["spec"]["volumeName"])
                vid = pv["spec"]["cinder"]["volumeID"]
                assert cloud.volumes[vid]["size"] == 2 and cloud.volumes[vid]["availability_zone"] == "az-gpu"
                assert m.labels_of(pv)["failure-domain.beta.kubernetes.io/zone"] == "az-gpu"
                assert pv["spec"]["capacity"]["storage"] == "2Gi"
                await c.delete("persistentvolumeclaims", "data", "default")

                async def gone():
                    return vid not in cloud.volumes
                await until(gone)
            finally:
                await cm.stop()
                await cmc.close()
    run(go(), 90)


def test_kubelet_with_the_in_tree_openstack_provider(cloud, tmp_path):
    """kubelet --cloud-provider=openstack --cloud-config cloud.conf: the node registers with
    the server's providerID, the cloud's addresses (--node-ip first), instance type and zone."""
    from tests.conftest import run
    sid = cloud.add_server("mi355x-node-0", "10.0.0.21", floating_ip="203.0.113.77", az="az-gpu")
    conf = tmp_path / "cloud.conf"
    conf.write_text(f"[Global]\nauth-url = {cloud.url}/identity/v3\nusername = admin\npassword = secret\n"
                    f"tenant-id = {cloud.project}\nregion = RegionOne\n")

    async def go():
        async with LocalCluster(gpus="fake", n_gpus=1, with_controllers=False, relist_period=0.2,
                                kubelet_kw={"cloud_provider": "openstack", "cloud_config": str(conf),
                                            "node_ip": "10.0.0.21"}) as lc:
            n = await lc.client.get("nodes", lc.node_name)
            assert n["spec"]["providerID"] == f"openstack:///{sid}"
            lab = m.labels_of(n)
            assert lab["beta.kubernetes.io/instance-type"] == "gpu.mi355x.8x"
            assert lab["failure-domain.beta.kubernetes.io/zone"] == "az-gpu"
            assert lab["failure-domain.beta.kubernetes.io/region"] == "RegionOne"
            assert n["status"]["addresses"] == [{"type": "InternalIP", "address": "10.0.0.21"},
                                                {"type": "ExternalIP", "address": "203.0.113.77"},
                                                {"type": "Hostname", "address": "mi355x-node-0"}]
    run(go(), 60)
