"""GCE cloud provider and persistent disks (reference: pkg/cloudprovider/providers/gce
gce_test.go — TestGetRegion, TestSplitProviderID, gce_loadbalancer_external_test.go —
TestEnsureExternalLoadBalancer / TestUpdateExternalLoadBalancer / TestEnsureExternalLoadBalancerDeleted,
gce_disks_test.go — TestCreateDisk_Basic / TestAttachDisk / TestDeleteDisk_NotFound,
gce_routes.go; pkg/volume/gce_pd attacher_test.go), against the in-repo fake Compute Engine
and metadata server (tests/fake_gce.py). No GCP exists offline: parity with the real service is
unpinned; request and resource shapes follow the public compute/v1 API."""
import asyncio

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.cloudprovider import Route, get_cloud_provider
from amdkube.cloudprovider.gce import GCEError, lb_name, port_range, region_of_zone, split_provider_id
from amdkube.controllers import ControllerManager, Options
from amdkube.localcluster import LocalCluster
from tests.conftest import run
from tests.fake_gce import FakeGCE


@pytest.fixture()
def gce():
    f = FakeGCE().start()
    try:
        yield f
    finally:
        f.stop()


def test_instances_zones_tokens_and_provider_ids(gce):
    gce.add_instance("gpu-node-1", "10.128.0.11", external="34.1.2.3")
    gce.add_instance("gpu-node-2", "10.128.0.12", zone="us-central1-b", mtype="a3-highgpu-8g")
    cloud = get_cloud_provider("gce", gce.config())
    assert (cloud.project, cloud.zone, cloud.region) == ("mi355x-proj", "us-central1-a", "us-central1")
    assert cloud.managed_zones() == ["us-central1-a", "us-central1-b"]
    ins = cloud.instances()

    async def go():
        # this instance: the metadata server; another one: instances.get across the region's zones
        assert await ins.node_addresses("gpu-node-1") == [{"type": "InternalIP", "address": "10.128.0.11"},
                                                         {"type": "ExternalIP", "address": "34.1.2.3"}]
        assert await ins.node_addresses("gpu-node-2.c.mi355x-proj.internal") == [{"type": "InternalIP", "address": "10.128.0.12"}]
        assert await ins.instance_id("gpu-node-2") == "mi355x-proj/us-central1-b/gpu-node-2"
        assert await ins.instance_type("gpu-node-2") == "a3-highgpu-8g"
        assert await ins.instance_exists("gpu-node-2") and not await ins.instance_exists("nope")
        assert await ins.instance_exists_by_provider_id("gce://mi355x-proj/us-central1-b/gpu-node-2")
        assert not await ins.instance_exists_by_provider_id("gce://mi355x-proj/us-central1-b/gone")
        assert await ins.node_addresses_by_provider_id("gce://mi355x-proj/us-central1-a/gpu-node-1") == [
            {"type": "InternalIP", "address": "10.128.0.11"}, {"type": "ExternalIP", "address": "34.1.2.3"}]
    asyncio.run(go())
    z = cloud.zone_for_node("gpu-node-2")
    assert (z.failure_domain, z.region) == ("us-central1-b", "us-central1")
    # an expired token is replaced once on a 401
    calls = gce.token_calls
    gce.tokens.clear()
    assert asyncio.run(ins.instance_exists("gpu-node-2")) and gce.token_calls == calls + 1
    assert split_provider_id("gce://p/z-a/n") == ("p", "z-a", "n") and region_of_zone("europe-west4-c") == "europe-west4"
    with pytest.raises(ValueError):
        split_provider_id("aws:///us-east-1a/i-1")


def test_routes(gce):
    gce.add_instance("gpu-node-1", "10.128.0.11")
    cloud = get_cloud_provider("gce", gce.config())
    rt = cloud.routes()
    rt.create("kubernetes", "uid-1", Route("", "gpu-node-1", "10.244.1.0/24"))
    r = gce.routes["kubernetes-uid-1"]
    assert (r["destRange"], r["nextHopInstance"], r["priority"], r["description"]) == (
        "10.244.1.0/24", "zones/us-central1-a/instances/gpu-node-1", 1000, "k8s-node-route")
    rt.create("kubernetes", "uid-1", Route("", "gpu-node-1", "10.244.1.0/24"))          # 409: already there
    gce.routes["other-cluster-x"] = dict(r, name="other-cluster-x")                     # not ours
    got = rt.list("kubernetes")
    assert got == [Route("kubernetes-uid-1", "gpu-node-1", "10.244.1.0/24")]
    rt.delete("kubernetes", got[0])
    assert "kubernetes-uid-1" not in gce.routes
    rt.delete("kubernetes", got[0])


def _svc(ports, uid="0f9a2c3e-1111-2222-3333-444455556666", proto="TCP", **spec):
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "inference", "namespace": "ml", "uid": uid},
            "spec": {"type": "LoadBalancer", "ports": [{"port": p, "nodePort": np, "protocol": proto} for p, np in ports], **spec}}


def _node(name):
    return {"metadata": {"name": name}}


def test_external_load_balancer_lifecycle(gce):
    gce.add_instance("gpu-node-1", "10.128.0.11")
    gce.add_instance("gpu-node-2", "10.128.0.12", zone="us-central1-b")
    gce.add_instance("gpu-node-3", "10.128.0.13")
    cloud = get_cloud_provider("gce", gce.config(**{"cluster-id": "c1"}))
    cloud.client.poll = 0.01
    lb = cloud.load_balancer()
    svc = _svc([(80, 30080), (443, 30443)], loadBalancerSourceRanges=["10.1.0.0/16"])
    st = lb.ensure("kubernetes", svc, [_node("gpu-node-1"), _node("gpu-node-2")])
    name = lb_name(svc)
    ip = gce.addresses[name]["address"]
    assert st == {"ingress": [{"ip": ip}]}
    fw = gce.firewalls[f"k8s-fw-{name}"]
    assert fw["sourceRanges"] == ["10.1.0.0/16"] and fw["targetTags"] == ["gke-node"]
    assert fw["allowed"] == [{"IPProtocol": "tcp", "ports": ["80", "443"]}]
    tp = gce.pools[name]
    assert sorted(u.rsplit("/", 1)[-1] for u in tp["instances"]) == ["gpu-node-1", "gpu-node-2"]
    assert tp["sessionAffinity"] == "NONE" and tp["healthChecks"][0].endswith("/httpHealthChecks/k8s-c1-node")
    assert (gce.hcs["k8s-c1-node"]["port"], gce.hcs["k8s-c1-node"]["requestPath"]) == (10256, "/healthz")
    fr = gce.rules[name]
    assert (fr["IPAddress"], fr["portRange"], fr["IPProtocol"]) == (ip, "80-443", "TCP") and fr["target"].endswith(f"/targetPools/{name}")
    assert lb.get("kubernetes", svc) == (st, True)
    # node churn only touches the pool; ports / affinity changes rebuild rule and pool on the same IP
    lb.update("kubernetes", svc, [_node("gpu-node-2"), _node("gpu-node-3")])
    assert sorted(u.rsplit("/", 1)[-1] for u in gce.pools[name]["instances"]) == ["gpu-node-2", "gpu-node-3"]
    svc2 = _svc([(8080, 31080)], sessionAffinity="ClientIP", externalTrafficPolicy="Local", healthCheckNodePort=32000)
    st2 = lb.ensure("kubernetes", svc2, [_node("gpu-node-3")])
    assert st2 == st and gce.rules[name]["portRange"] == "8080-8080" and gce.pools[name]["sessionAffinity"] == "CLIENT_IP"
    assert gce.pools[name]["healthChecks"][0].endswith(f"/httpHealthChecks/{name}") and gce.hcs[name]["port"] == 32000
    assert gce.firewalls[f"k8s-fw-{name}"]["allowed"] == [{"IPProtocol": "tcp", "ports": ["8080"]}]
    with pytest.raises(ValueError):
        lb.ensure("kubernetes", _svc([(80, 30080)]), [])
    lb.ensure_deleted("kubernetes", svc2)
    assert not (gce.rules or gce.pools or gce.addresses or gce.firewalls)
    assert name not in gce.hcs                    # the service's own health check went with it
    assert lb.get("kubernetes", svc) == (None, False)
    lb.ensure_deleted("kubernetes", svc)          # idempotent
    assert port_range([{"port": 53}, {"port": 5353}]) == "53-5353"
    st3 = lb.ensure("kubernetes", _svc([(53, 30053)], uid="u-udp", proto="UDP", loadBalancerIP="35.0.0.99"), [_node("gpu-node-1")])
    assert st3 == {"ingress": [{"ip": "35.0.0.99"}]} and gce.rules[lb_name(_svc([], uid="u-udp"))]["IPProtocol"] == "UDP"


def test_persistent_disks_and_plugin(gce, tmp_path):
    from amdkube.volume import NoopMounter, PluginMgr, Spec, VolumeHost, default_plugins
    gce.add_instance("gpu-node-1", "10.128.0.11")
    gce.add_instance("gpu-node-2", "10.128.0.12", zone="us-central1-b")
    cloud = get_cloud_provider("gce", gce.config())
    cloud.client.poll = 0.01
    vols = cloud.volumes()
    src, labels = vols.provision("pvc-1", 200, {"type": "pd-ssd", "zone": "us-central1-a"}, {"kubernetes.io/created-for/pvc/name": "data"}, "data")
    d = gce.disks[("us-central1-a", "kubernetes-dynamic-pvc-1")]
    assert src == {"pdName": "kubernetes-dynamic-pvc-1", "fsType": "ext4"} and d["sizeGb"] == "200"
    assert d["type"].endswith("/zones/us-central1-a/diskTypes/pd-ssd") and '"kubernetes.io/created-for/pvc/name": "data"' in d["description"]
    assert labels == {"failure-domain.beta.kubernetes.io/zone": "us-central1-a", "failure-domain.beta.kubernetes.io/region": "us-central1"}
    with pytest.raises(ValueError):
        vols.provision("pvc-x", 1, {"type": "pd-fast"}, {}, "x")
    dev_root = tmp_path / "root"
    host = VolumeHost(str(tmp_path / "kubelet"), node_name="gpu-node-1", mounter=NoopMounter())
    host.cloud, host.dev_root, host.attach_poll = cloud, str(dev_root), 0.01
    pv = {"metadata": {"name": "pv-1"}, "spec": {"gcePersistentDisk": src}}
    spec = Spec(pv=pv)
    plugin = PluginMgr(default_plugins(), host).find_by_spec(spec)
    assert plugin.name == "kubernetes.io/gce-pd"

    async def go():
        dev = await plugin.attach(spec, "gpu-node-1")
        assert dev == "/dev/disk/by-id/google-kubernetes-dynamic-pvc-1"
        inst = gce.instances[("us-central1-a", "gpu-node-1")]
        assert [x["deviceName"] for x in inst["disks"]] == ["boot", "kubernetes-dynamic-pvc-1"] and inst["disks"][1]["mode"] == "READ_WRITE"
        assert await plugin.attach(spec, "gpu-node-1") == dev             # idempotent
        with pytest.raises(GCEError):
            await plugin.attach(spec, "gpu-node-2")                        # other zone
        byid = dev_root / "dev" / "disk" / "by-id"
        byid.mkdir(parents=True)
        (byid / "google-kubernetes-dynamic-pvc-1").write_text("")
        assert (await plugin.wait_for_attach(spec, dev, None, 5)).endswith("google-kubernetes-dynamic-pvc-1")
        with pytest.raises(GCEError):
            vols.delete("kubernetes-dynamic-pvc-1")                        # in use
        await plugin.detach("kubernetes-dynamic-pvc-1", "gpu-node-1")
        assert [x["deviceName"] for x in inst["disks"]] == ["boot"]
    asyncio.run(go())
    assert cloud.labels_for_volume(pv) == labels
    assert vols.delete("kubernetes-dynamic-pvc-1") and not vols.delete("kubernetes-dynamic-pvc-1")


def test_controllers_and_kubelet_drive_gce(gce):
    gce.add_instance("mi355x-node-0", "10.128.0.21", external="34.9.9.9", mtype="a3-mi355x-8g")

    async def go():
        import json
        import tempfile
        cfgf = tempfile.NamedTemporaryFile("w", suffix=".json", delete=False)
        json.dump(gce.config(), cfgf)
        cfgf.close()
        async with LocalCluster(gpus="fake", n_gpus=1, with_controllers=False, relist_period=0.2,
                                kubelet_kw={"cloud_provider": "gce", "cloud_config": cfgf.name}) as lc:
            c = lc.client
            n = await c.get("nodes", lc.node_name)
            assert n["spec"]["providerID"] == "gce://mi355x-proj/us-central1-a/mi355x-node-0"
            lab = m.labels_of(n)
            assert lab["beta.kubernetes.io/instance-type"] == "a3-mi355x-8g"
            assert lab["failure-domain.beta.kubernetes.io/zone"] == "us-central1-a"
            assert {"type": "ExternalIP", "address": "34.9.9.9"} in n["status"]["addresses"]
            await c.patch("nodes", lc.node_name, {"spec": {"podCIDR": "10.244.3.0/24"}})
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default"},
                            "spec": {"type": "LoadBalancer", "ports": [{"port": 80, "protocol": "TCP"}]}}, "default")
            await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": "pd"},
                            "provisioner": "kubernetes.io/gce-pd", "parameters": {"type": "pd-ssd"}})
            await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data", "namespace": "default"},
                            "spec": {"storageClassName": "pd", "accessModes": ["ReadWriteOnce"],
                                     "resources": {"requests": {"storage": "10Gi"}}}}, "default")
            cloud = get_cloud_provider("gce", gce.config())
            cloud.client.poll = 0.01
            cmc = Client(lc.api.url, token=lc.api.loopback_token)
            cm = await ControllerManager(cmc, ["service", "route", "persistentvolume-binder", "pvc-protection", "pv-protection"],
                                         options=Options(cloud=cloud, cluster_name="kubernetes")).start()
            try:
                async def until(fn, t=30):
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
                assert ing[0]["ip"].startswith("35.0.0.")

                async def routed():
                    return [r for r in gce.routes.values() if r["destRange"] == "10.244.3.0/24"]
                assert (await until(routed))[0]["nextHopInstance"].endswith("/instances/mi355x-node-0")

                async def bound():
                    p = await c.get("persistentvolumeclaims", "data", "default")
                    return p if (p.get("status") or {}).get("phase") == "Bound" else None
                pvc = await until(bound)
                pv = await c.get("persistentvolumes", pvc["spec"]["volumeName"])
                pd = pv["spec"]["gcePersistentDisk"]["pdName"]
                assert gce.disks[("us-central1-a", pd)]["sizeGb"] == "10"       # the only zone running instances
                assert m.labels_of(pv)["failure-domain.beta.kubernetes.io/zone"] == "us-central1-a"
                await c.delete("persistentvolumeclaims", "data", "default")

                async def gone():
                    return ("us-central1-a", pd) not in gce.disks
                await until(gone)
            finally:
                await cm.stop()
                await cmc.close()
    run(go(), 90)
