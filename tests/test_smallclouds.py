"""CloudStack, oVirt and Photon cloud providers (reference: pkg/cloudprovider/providers/cloudstack
— cloudstack_test.go, cloudstack_loadbalancer.go; providers/ovirt — ovirt_test.go
TestOVirtCloudXmlParsing; providers/photon — photon_test.go TestInstances / TestVolumes;
pkg/volume/photon_pd), against the in-repo fakes in tests/fake_smallclouds.py. None of these
services exists offline, so parity with them is unpinned; request shapes follow their public APIs."""
import asyncio

import pytest

from amdkube.cloudprovider import get_cloud_provider
from amdkube.cloudprovider.cloudstack import CloudStackError, lb_name, sign
from amdkube.cloudprovider.ovirt import instances_from_xml
from amdkube.volume import cinder
from tests.fake_smallclouds import FakeCloudStack, FakeOVirt, FakePhoton


@pytest.fixture()
def cs():
    f = FakeCloudStack().start()
    yield f
    f.stop()


def _svc(ports, uid="0f6c2a4e-1111-2222-3333-444455556666", **spec):
    return {"metadata": {"name": "web", "namespace": "default", "uid": uid},
            "spec": {"type": "LoadBalancer", "ports": ports, **spec}}


def _node(name):
    return {"metadata": {"name": name}}


def test_cloudstack_signature_instances_and_zones(cs):
    a = cs.add_vm("gpu-a", "10.1.0.5", public="198.51.100.7")
    cs.add_vm("gpu-b", "10.1.0.6", offering="mi355x.4gpu")
    cloud = get_cloud_provider("cloudstack", cs.config())
    ins = cloud.instances()

    async def go():
        assert await ins.node_addresses("gpu-a") == [{"type": "InternalIP", "address": "10.1.0.5"},
                                                     {"type": "ExternalIP", "address": "198.51.100.7"}]
        assert await ins.instance_id("gpu-a") == a
        assert await ins.instance_type("gpu-b") == "mi355x.4gpu"
        assert await ins.instance_exists("gpu-b") and not await ins.instance_exists("nope")
        assert await ins.instance_exists_by_provider_id(f"cloudstack://{a}")
        assert not await ins.instance_exists_by_provider_id("cloudstack://gone")
        assert await ins.node_addresses_by_provider_id(f"cloudstack://{a}") == await ins.node_addresses("gpu-a")
    asyncio.run(go())
    z = cloud.zone_for_node("gpu-b")
    assert (z.failure_domain, z.region) == ("zone-mi355x", "zone-mi355x")
    # the signature is over the lower-cased sorted query; a wrong secret is refused by the API
    assert sign({"command": "listZones", "apiKey": "K", "response": "json"}, "s") != sign({"command": "listZones", "apiKey": "K", "response": "json"}, "t")
    bad = get_cloud_provider("cloudstack", cs.config().replace(cs.SECRET, "wrong"))
    with pytest.raises(CloudStackError) as e:
        asyncio.run(bad.instances().instance_exists("gpu-a"))
    assert e.value.code == 401


def test_cloudstack_load_balancer_lifecycle(cs):
    a, b = cs.add_vm("gpu-a", "10.1.0.5"), cs.add_vm("gpu-b", "10.1.0.6")
    c = cs.add_vm("gpu-c", "10.1.0.7")
    lb = get_cloud_provider("cloudstack", cs.config()).load_balancer()
    svc = _svc([{"port": 80, "nodePort": 30080, "protocol": "TCP"}, {"port": 443, "nodePort": 30443}])
    name = lb_name(svc)
    assert name == "a0f6c2a4e111122223333444455556666"[:32]
    st = lb.ensure("k", svc, [_node("gpu-a"), _node("gpu-b")])
    ip = st["ingress"][0]["ip"]
    assert ip.startswith("203.0.113.") and len(cs.ips) == 1
    rules = {r["name"]: r for r in cs.rules.values()}
    assert set(rules) == {f"{name}-tcp-80", f"{name}-tcp-443"}
    assert rules[f"{name}-tcp-80"]["privateport"] == "30080" and rules[f"{name}-tcp-80"]["algorithm"] == "roundrobin"
    assert all(cs.members[r["id"]] == {a, b} for r in rules.values())
    assert lb.get("k", svc) == ({"ingress": [{"ip": ip}]}, True)
    # node set changes: instances follow by symmetric difference
    lb.update("k", svc, [_node("gpu-b"), _node("gpu-c")])
    assert all(cs.members[r["id"]] == {b, c} for r in cs.rules.values())
    # port 443 dropped, 80 moves to another node port, ClientIP affinity: rules replaced/updated, same address
    svc2 = _svc([{"port": 80, "nodePort": 31080}], sessionAffinity="ClientIP")
    assert lb.ensure("k", svc2, [_node("gpu-b"), _node("gpu-c")])["ingress"][0]["ip"] == ip
    (r,) = cs.rules.values()
    assert (r["name"], r["privateport"], r["algorithm"]) == (f"{name}-tcp-80", "31080", "source")
    assert cs.members[r["id"]] == {b, c}
    with pytest.raises(ValueError):
        lb.ensure("k", _svc([{"port": 53, "nodePort": 30053, "protocol": "UDP"}]), [_node("gpu-a")])
    lb.ensure_deleted("k", svc2)
    assert not cs.rules and not cs.ips and lb.get("k", svc2) == (None, False)


def test_cloudstack_requested_ip_is_not_released(cs):
    cs.add_vm("gpu-a", "10.1.0.5")
    lb = get_cloud_provider("cloudstack", cs.config()).load_balancer()
    own = cs._cmd("associateIpAddress", {"networkid": "net-1"})
    ip = cs.jobs.popitem()[1]["ipaddress"]
    svc = _svc([{"port": 80, "nodePort": 30080}], loadBalancerIP=ip["ipaddress"])
    assert lb.ensure("k", svc, [_node("gpu-a")])["ingress"][0]["ip"] == ip["ipaddress"]
    lb.ensure_deleted("k", svc)
    assert not cs.rules and ip["id"] in cs.ips and own["jobid"]
    with pytest.raises(LookupError):
        lb.ensure("k", _svc([{"port": 80, "nodePort": 30080}], loadBalancerIP="192.0.2.99"), [_node("gpu-a")])


def test_ovirt_instances():
    f = FakeOVirt().start()
    try:
        a = f.add_vm("vm-a", "gpu-a.lab", ips=["10.2.0.5", "10.2.0.6"])
        f.add_vm("vm-b", "gpu-b.lab", ips=["10.2.0.7"], state="down")
        f.add_vm("vm-c", "", ips=["10.2.0.8"])
        cloud = get_cloud_provider("ovirt", f.config())
        ins = cloud.instances()
        assert cloud.zones() is None and cloud.load_balancer() is None and cloud.routes() is None

        async def go():
            assert await ins.node_addresses("gpu-a.lab") == [{"type": "InternalIP", "address": "10.2.0.5"},
                                                             {"type": "ExternalIP", "address": "10.2.0.5"}]
            assert await ins.instance_id("gpu-a.lab") == "/" + a
            assert await ins.instance_exists("gpu-a.lab")
            assert not await ins.instance_exists("gpu-b.lab")      # down VMs are not nodes
            assert await ins.instance_exists_by_provider_id(f"ovirt:///{a}")
            with pytest.raises(LookupError):
                await ins.node_addresses("gpu-b.lab")
        asyncio.run(go())
        assert f.searches and set(f.searches) == {"cluster=gpu"}
        with pytest.raises(ValueError):
            get_cloud_provider("ovirt", "[connection]\nusername = x\n")
        xml = ('<vms><vm id="u1"><name>n</name><guest_info><fqdn>h1</fqdn><ips><ip address="1.2.3.4"/></ips>'
               '</guest_info><status><state>up</state></status></vm><vm id="u2"><name>m</name><status><state>up</state>'
               '</status></vm></vms>')
        assert instances_from_xml(xml) == {"h1": {"id": "u1", "name": "n", "ip": "1.2.3.4"}}
    finally:
        f.stop()


def test_photon_instances_and_disks():
    f = FakePhoton().start()
    try:
        a = f.add_vm("gpu-a", [{"ipAddress": "10.3.0.5", "macAddress": "02:00:00:00:00:01"},
                               {"ipAddress": "192.0.2.5", "macAddress": "00:50:56:aa:bb:cc"}])
        b = f.add_vm("gpu-b", [{"ipAddress": "10.3.0.6", "macAddress": "02:00:00:00:00:02"}], flavor="big")
        cloud = get_cloud_provider("photon", f.config(zone="rack-1"))
        ins = cloud.instances()

        async def go():
            assert await ins.node_addresses("gpu-a") == [{"type": "InternalIP", "address": "10.3.0.5"},
                                                         {"type": "ExternalIP", "address": "192.0.2.5"}]
            assert await ins.instance_id("gpu-b") == b and await ins.instance_type("gpu-b") == "big"
            assert await ins.instance_exists_by_provider_id(f"photon://{a}")
            assert not await ins.instance_exists_by_provider_id("photon://gone")
            assert not await ins.instance_exists("nope")
        asyncio.run(go())
        # overrideIP: node names are addresses
        by_ip = get_cloud_provider("photon", f.config(overrideIP="true")).instances()
        assert asyncio.run(by_ip.instance_id("10.3.0.6")) == b
        vols = cloud.volumes()
        src, labels = vols.provision("pvc-1", 20, {"flavor": "ssd", "fsType": "xfs"}, {}, "claim")
        pd = src["pdID"]
        assert f.disks[pd]["capacityGb"] == 20 and f.disks[pd]["flavor"] == "ssd" and src["fsType"] == "xfs"
        assert labels == {"failure-domain.beta.kubernetes.io/zone": "rack-1"}
        dev = vols.attach("gpu-a", pd)
        assert dev == "/dev/disk/by-id/wwn-0x" + pd.replace("-", "") and f.disks[pd]["vms"] == [a]
        assert vols.attach("gpu-a", pd) == dev                # idempotent
        with pytest.raises(Exception):
            vols.delete_source(src)                           # attached
        vols.detach("gpu-a", pd)
        assert f.disks[pd]["vms"] == []
        vols.detach("gpu-a", pd)
        vols.delete_source(src)
        assert pd not in f.disks
        vols.delete_source(src)                               # already gone
    finally:
        f.stop()


def test_photon_pd_plugin_is_a_cloud_disk():
    names = {p.source_key: p for p in cinder.plugins()}
    p = names["photonPersistentDisk"]
    assert p.name == "kubernetes.io/photon-pd" and p.id_field == "pdID" and p.provider == "photon"
    from amdkube.volume import default_plugins
    [q] = [q for q in default_plugins() if getattr(q, "source_key", None) == "photonPersistentDisk"]
    assert type(q) is type(p) and q.name == p.name
