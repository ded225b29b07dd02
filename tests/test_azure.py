"""Azure cloud provider and managed disks (reference: pkg/cloudprovider/providers/azure
azure_test.go — TestReconcileLoadBalancer*, TestReconcileSecurityGroup*, TestNewCloudFromJSON,
TestSplitProviderID, TestGetZone; azure_loadbalancer_test.go; azure_routes.go;
azure_managedDiskController.go; pkg/volume/azure_dd azure_common_test.go findDiskByLun),
against the in-repo fake Azure AD + Resource Manager + instance metadata service
(tests/fake_azure.py). No Azure exists offline: parity with the real service is unpinned; the
resource shapes and api-versions follow the public ARM REST API."""
import asyncio

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.cloudprovider import Route, get_cloud_provider
from amdkube.cloudprovider.azure import AzureError, node_name_from_provider_id, rule_prefix
from amdkube.controllers import ControllerManager, Options
from amdkube.localcluster import LocalCluster
from tests.conftest import run
from tests.fake_azure import FakeAzure


@pytest.fixture()
def az():
    f = FakeAzure().start()
    try:
        yield f
    finally:
        f.stop()


def test_instances_zones_and_tokens(az):
    vm = az.add_vm("mi355x-0", "10.240.0.4", public="52.1.1.1", fault_domain=2)
    az.add_vm("mi355x-1", "10.240.0.5")
    cloud = get_cloud_provider("azure", az.config())
    ins = cloud.instances()

    async def go():
        assert await ins.node_addresses("mi355x-0") == [{"type": "InternalIP", "address": "10.240.0.4"},
                                                       {"type": "Hostname", "address": "mi355x-0"},
                                                       {"type": "ExternalIP", "address": "52.1.1.1"}]
        assert await ins.instance_id("mi355x-0") == vm["id"]
        assert await ins.instance_type("mi355x-1") == "Standard_ND96isr_MI355X_v6"
        assert await ins.instance_exists("mi355x-1") and not await ins.instance_exists("nope")
        assert await ins.instance_exists_by_provider_id("azure://" + vm["id"])
        assert await ins.node_addresses_by_provider_id("azure://" + vm["id"]) == await ins.node_addresses("mi355x-0")
    asyncio.run(go())
    z = cloud.zone_for_node("mi355x-0")
    assert (z.failure_domain, z.region) == ("2", "eastus")
    assert cloud.zones().failure_domain == "2"                 # this VM, from the instance metadata service
    assert node_name_from_provider_id("azure://" + vm["id"]) == "mi355x-0"
    with pytest.raises(ValueError):
        node_name_from_provider_id("gce://p/z/n")
    # client credentials: one token, renewed once after a 401; a managed identity works too
    calls = az.token_calls
    az.tokens.clear()
    assert asyncio.run(ins.instance_exists("mi355x-1")) and az.token_calls == calls + 1
    msi = get_cloud_provider("azure", az.config(useManagedIdentityExtension=True, aadClientSecret=""))
    assert asyncio.run(msi.instances().instance_type("mi355x-0")) == "Standard_ND96isr_MI355X_v6"
    bad = get_cloud_provider("azure", az.config(aadClientSecret="wrong"))
    with pytest.raises(AzureError):
        asyncio.run(bad.instances().instance_type("mi355x-0"))
    with pytest.raises(ValueError):
        get_cloud_provider("azure", {"subscriptionId": "s"})


def test_route_table(az):
    az.add_vm("mi355x-0", "10.240.0.4")
    cloud = get_cloud_provider("azure", az.config())
    rt = cloud.routes()
    rt.create("kubernetes", "hint", Route("", "mi355x-0", "10.244.0.0/24"))      # creates the table too
    t = az.get(az.rid("Microsoft.Network", "routeTables", "k8s-routes"))
    assert [(r["name"], r["properties"]["addressPrefix"], r["properties"]["nextHopType"], r["properties"]["nextHopIpAddress"])
            for r in t["properties"]["routes"]] == [("mi355x-0", "10.244.0.0/24", "VirtualAppliance", "10.240.0.4")]
    assert rt.list("kubernetes") == [Route("mi355x-0", "mi355x-0", "10.244.0.0/24")]
    rt.delete("kubernetes", Route("mi355x-0", "mi355x-0", "10.244.0.0/24"))
    assert rt.list("kubernetes") == []
    rt.delete("kubernetes", Route("mi355x-0", "mi355x-0", "10.244.0.0/24"))
    assert get_cloud_provider("azure", az.config(routeTableName="")).routes() is None


def _svc(ports, uid="0f9a2c3e-1111-2222-3333-444455556666", ann=None, **spec):
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "inference", "namespace": "ml", "uid": uid,
                                                                 "annotations": ann or {}},
            "spec": {"type": "LoadBalancer", "ports": [{"port": p, "nodePort": np, "protocol": "TCP"} for p, np in ports], **spec}}


def test_shared_load_balancer_and_nsg(az):
    az.add_vm("mi355x-0", "10.240.0.4")
    az.add_vm("mi355x-1", "10.240.0.5")
    az.add_nsg()
    cloud = get_cloud_provider("azure", az.config())
    lb = cloud.load_balancer()
    a = _svc([(80, 30080), (443, 30443)], ann={"service.beta.kubernetes.io/azure-dns-label-name": "mi355x-infer"},
             loadBalancerSourceRanges=["10.1.0.0/16"])
    b = _svc([(8080, 31080)], uid="bbbbbbbb-0000-0000-0000-000000000000")
    nodes = [{"metadata": {"name": "mi355x-0"}}, {"metadata": {"name": "mi355x-1"}}]
    st_a = lb.ensure("kubernetes", a, nodes)
    st_b = lb.ensure("kubernetes", b, nodes[:1])
    obj = az.get(az.rid("Microsoft.Network", "loadBalancers", "kubernetes"))
    props = obj["properties"]
    pa, pb = rule_prefix(a), rule_prefix(b)
    assert sorted(f["name"] for f in props["frontendIPConfigurations"]) == sorted([pa, pb])
    assert sorted(r["name"] for r in props["loadBalancingRules"]) == sorted([f"{pa}-TCP-80", f"{pa}-TCP-443", f"{pb}-TCP-8080"])
    r80 = next(r for r in props["loadBalancingRules"] if r["name"] == f"{pa}-TCP-80")["properties"]
    assert r80["enableFloatingIP"] and r80["backendPort"] == 80 and r80["probe"]["id"].endswith(f"/probes/{pa}-TCP-80")
    assert next(p for p in props["probes"] if p["name"] == f"{pa}-TCP-80")["properties"]["port"] == 30080
    pip = az.get(az.rid("Microsoft.Network", "publicIPAddresses", f"kubernetes-{pa}"))
    assert st_a == {"ingress": [{"ip": pip["properties"]["ipAddress"]}]} and pip["properties"]["dnsSettings"]["domainNameLabel"] == "mi355x-infer"
    assert st_b["ingress"][0]["ip"] != st_a["ingress"][0]["ip"]
    members = [x["id"] for x in props["backendAddressPools"][0]["properties"]["backendIPConfigurations"]]
    assert len(members) == 2                                      # both nodes' primary IP configs joined the pool
    nsg = az.get(az.rid("Microsoft.Network", "networkSecurityGroups", "k8s-nsg"))
    rules = {r["name"]: r["properties"] for r in nsg["properties"]["securityRules"]}
    assert rules[f"{pa}-TCP-80-10.1.0.0_16"]["destinationAddressPrefix"] == st_a["ingress"][0]["ip"]
    assert rules[f"{pb}-TCP-8080-Internet"]["sourceAddressPrefix"] == "Internet"
    assert len({r["priority"] for r in rules.values()}) == len(rules) and rules["allow-ssh"]["priority"] == 500
    assert lb.get("kubernetes", a) == (st_a, True)
    # a port change rewrites only this service's rules; deleting one service keeps the other's
    lb.ensure("kubernetes", _svc([(80, 30080)], ann=a["metadata"]["annotations"]), nodes)
    props = az.get(az.rid("Microsoft.Network", "loadBalancers", "kubernetes"))["properties"]
    assert sorted(r["name"] for r in props["loadBalancingRules"]) == sorted([f"{pa}-TCP-80", f"{pb}-TCP-8080"])
    lb.ensure_deleted("kubernetes", a)
    props = az.get(az.rid("Microsoft.Network", "loadBalancers", "kubernetes"))["properties"]
    assert [f["name"] for f in props["frontendIPConfigurations"]] == [pb]
    assert az.get(az.rid("Microsoft.Network", "publicIPAddresses", f"kubernetes-{pa}")) is None
    assert not any(n.startswith(pa) for n in (r["name"] for r in az.get(
        az.rid("Microsoft.Network", "networkSecurityGroups", "k8s-nsg"))["properties"]["securityRules"]))
    lb.ensure_deleted("kubernetes", b)                            # the last one: the LB goes, the pool empties
    assert az.get(az.rid("Microsoft.Network", "loadBalancers", "kubernetes")) is None
    nic = az.get(az.rid("Microsoft.Network", "networkInterfaces", "mi355x-0-nic"))
    assert nic["properties"]["ipConfigurations"][0]["properties"]["loadBalancerBackendAddressPools"] == []
    # an internal service gets a private frontend on the <cluster>-internal LB
    intl = _svc([(80, 30080)], uid="cccc", ann={"service.beta.kubernetes.io/azure-load-balancer-internal": "true"})
    st = lb.ensure("kubernetes", intl, nodes)
    assert st["ingress"][0]["ip"].startswith("10.240.0.")
    ilb = az.get(az.rid("Microsoft.Network", "loadBalancers", "kubernetes-internal"))
    assert ilb["properties"]["frontendIPConfigurations"][0]["properties"]["subnet"]["id"].endswith(
        "/virtualNetworks/k8s-vnet/subnets/k8s-subnet")


def test_managed_disks_and_plugin(az, tmp_path):
    from amdkube.volume import NoopMounter, PluginMgr, Spec, VolumeHost, default_plugins
    az.add_vm("mi355x-0", "10.240.0.4")
    cloud = get_cloud_provider("azure", az.config())
    cloud.client.poll = 0.01
    vols = cloud.volumes()
    src, labels = vols.provision("pvc-1", 1024, {"skuName": "Premium_LRS"}, {"kubernetes.io/created-for/pvc/name": "data"}, "data")
    disk = az.get(src["diskURI"])
    assert disk["sku"]["name"] == "Premium_LRS" and disk["properties"]["diskSizeGB"] == 1024
    assert src["kind"] == "Managed" and labels == {"failure-domain.beta.kubernetes.io/region": "eastus"}
    with pytest.raises(ValueError):
        vols.provision("pvc-2", 1, {"kind": "Shared"}, {}, "x")
    with pytest.raises(ValueError):
        vols.provision("pvc-2", 1, {"skuName": "Ultra_XYZ"}, {}, "x")
    dev_root = tmp_path / "root"
    host = VolumeHost(str(tmp_path / "kubelet"), node_name="mi355x-0", mounter=NoopMounter())
    host.cloud, host.dev_root, host.attach_poll = cloud, str(dev_root), 0.01
    spec = Spec(pv={"metadata": {"name": "pv-1"}, "spec": {"azureDisk": src}})
    plugin = PluginMgr(default_plugins(), host).find_by_spec(spec)
    assert plugin.name == "kubernetes.io/azure-disk"
    # a second disk already sits at LUN 0: the new one lands on LUN 1
    other, _ = vols.provision("pvc-0", 8, {}, {}, "y")
    vols.attach("mi355x-0", other["diskURI"])

    async def go():
        lun = await plugin.attach(spec, "mi355x-0")
        assert lun == "1" and az.get(src["diskURI"])["properties"]["diskState"] == "Attached"
        assert await plugin.attach(spec, "mi355x-0") == "1"
        d = dev_root / "dev" / "disk" / "azure" / "scsi1"
        d.mkdir(parents=True)
        (d / "lun1").write_text("")
        assert (await plugin.wait_for_attach(spec, lun, None, 5)).endswith("scsi1/lun1")
        with pytest.raises(AzureError):
            vols.delete(src["diskURI"])
        await plugin.detach(src["diskURI"], "mi355x-0")
        vm = az.get(az.rid("Microsoft.Compute", "virtualMachines", "mi355x-0"))
        assert [x["lun"] for x in vm["properties"]["storageProfile"]["dataDisks"]] == [0]
        blob = Spec(volume={"name": "b", "azureDisk": {"diskName": "x", "diskURI": "https://acct.blob/x.vhd"}})
        with pytest.raises(Exception):
            await plugin.attach(blob, "mi355x-0")
    asyncio.run(go())
    assert vols.delete(src["diskURI"]) and not vols.delete(src["diskURI"])


def test_controllers_and_kubelet_drive_azure(az):
    az.add_vm("mi355x-node-0", "10.240.0.21", public="52.9.9.9")
    az.add_nsg()

    async def go():
        import json
        import tempfile
        cfgf = tempfile.NamedTemporaryFile("w", suffix=".json", delete=False)
        json.dump(az.config(), cfgf)
        cfgf.close()
        async with LocalCluster(gpus="fake", n_gpus=1, with_controllers=False, relist_period=0.2,
                                kubelet_kw={"cloud_provider": "azure", "cloud_config": cfgf.name}) as lc:
            c = lc.client
            n = await c.get("nodes", lc.node_name)
            assert n["spec"]["providerID"] == "azure://" + az.rid("Microsoft.Compute", "virtualMachines", "mi355x-node-0")
            lab = m.labels_of(n)
            assert lab["beta.kubernetes.io/instance-type"] == "Standard_ND96isr_MI355X_v6"
            assert (lab["failure-domain.beta.kubernetes.io/zone"], lab["failure-domain.beta.kubernetes.io/region"]) == ("1", "eastus")
            await c.patch("nodes", lc.node_name, {"spec": {"podCIDR": "10.244.5.0/24"}})
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default"},
                            "spec": {"type": "LoadBalancer", "ports": [{"port": 80, "protocol": "TCP"}]}}, "default")
            await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": "managed-premium"},
                            "provisioner": "kubernetes.io/azure-disk", "parameters": {"skuName": "Premium_LRS", "kind": "Managed"}})
            await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data", "namespace": "default"},
                            "spec": {"storageClassName": "managed-premium", "accessModes": ["ReadWriteOnce"],
                                     "resources": {"requests": {"storage": "64Gi"}}}}, "default")
            cloud = get_cloud_provider("azure", az.config())
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
                assert (await until(lb_ip))[0]["ip"].startswith("52.0.0.")

                async def routed():
                    t = az.get(az.rid("Microsoft.Network", "routeTables", "k8s-routes"))
                    return (t or {}).get("properties", {}).get("routes")
                assert (await until(routed))[0]["properties"]["addressPrefix"] == "10.244.5.0/24"

                async def bound():
                    p = await c.get("persistentvolumeclaims", "data", "default")
                    return p if (p.get("status") or {}).get("phase") == "Bound" else None
                pvc = await until(bound)
                pv = await c.get("persistentvolumes", pvc["spec"]["volumeName"])
                uri = pv["spec"]["azureDisk"]["diskURI"]
                assert az.get(uri)["properties"]["diskSizeGB"] == 64 and pv["spec"]["azureDisk"]["kind"] == "Managed"
                await c.delete("persistentvolumeclaims", "data", "default")

                async def gone():
                    return az.get(uri) is None
                await until(gone)
            finally:
                await cm.stop()
                await cmc.close()
    run(go(), 90)
