"""AWS cloud provider and EBS volumes (reference: pkg/cloudprovider/providers/aws aws_test.go —
TestNodeAddresses, TestGetRegion, TestFindVPCID-style metadata, TestBuildListener,
TestDescribeLoadBalancerOnDelete/OnGet/OnUpdate, TestGetVolumeLabels; device_allocator_test.go;
aws_routes.go; pkg/volume/aws_ebs attacher_test.go), against the in-repo fake EC2/ELB/metadata
service (tests/fake_aws.py). No AWS exists offline, so parity with the real services is
unpinned; Signature V4 itself is pinned to the two published AWS test-suite vectors."""
import asyncio

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.cloudprovider import Route, get_cloud_provider, load_config
from amdkube.cloudprovider.aws import (AWSError, DeviceAllocator, choose_zone, instance_id_from_provider_id, lb_name,
                                       listeners_for, sign_v4, volume_id, xml_to_obj)
from amdkube.controllers import ControllerManager, Options
from amdkube.localcluster import LocalCluster
from tests.conftest import run
from tests.fake_aws import FakeAWS


@pytest.fixture()
def aws():
    f = FakeAWS().start()
    try:
        yield f
    finally:
        f.stop()


def test_signature_v4_matches_the_published_vectors():
    key = "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY"
    h = sign_v4("GET", "https://example.amazonaws.com/", {"Host": "example.amazonaws.com"}, b"", "us-east-1", "service",
                "AKIDEXAMPLE", key, "20150830T123600Z")
    assert h["Authorization"].endswith("Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")
    h = sign_v4("GET", "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08",
                {"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"}, b"", "us-east-1", "iam",
                "AKIDEXAMPLE", key, "20150830T123600Z")
    assert "SignedHeaders=content-type;host;x-amz-date," in h["Authorization"]
    assert h["Authorization"].endswith("Signature=5d672d79c15b13162d9279b0855cfba6789a8edb4c82c400e06b5924a6f2b5d7")
    import xml.etree.ElementTree as ET
    doc = ET.fromstring('<R xmlns="x"><a><item><b>1</b></item><item><b>2</b></item></a><c/></R>')
    assert xml_to_obj(doc) == {"a": [{"b": "1"}, {"b": "2"}], "c": ""}


def test_instances_zones_iam_credentials_and_provider_ids(aws):
    inst = aws.add_instance("10.0.0.11", az="us-east-1b", public="198.51.100.7", itype="gpu.mi355x.48xlarge")
    cloud = get_cloud_provider("aws", aws.config())
    assert (cloud.zone, cloud.region) == ("us-east-1a", "us-east-1")
    ins = cloud.instances()
    name = inst["privateDnsName"]

    async def go():
        addrs = await ins.node_addresses(name)
        assert addrs == [{"type": "InternalIP", "address": "10.0.0.11"}, {"type": "ExternalIP", "address": "198.51.100.7"},
                         {"type": "InternalDNS", "address": name},
                         {"type": "ExternalDNS", "address": "ec2-198-51-100-7.compute-1.amazonaws.com"}]
        iid = await ins.instance_id(name)
        assert iid == f"/us-east-1b/{inst['instanceId']}"
        assert await ins.instance_type(name) == "gpu.mi355x.48xlarge"
        assert await ins.instance_exists(name) and not await ins.instance_exists("ip-1-2-3-4.ec2.internal")
        assert await ins.instance_exists_by_provider_id(f"aws:///us-east-1b/{inst['instanceId']}")
        assert not await ins.instance_exists_by_provider_id("aws:///us-east-1b/i-0000dead")
        assert await ins.node_addresses_by_provider_id(f"aws:///us-east-1b/{inst['instanceId']}") == addrs
    asyncio.run(go())
    z = cloud.zone_for_node(name)
    assert (z.failure_domain, z.region) == ("us-east-1b", "us-east-1")
    assert aws.bad_signatures == 0 and "DescribeInstances" in aws.calls
    assert instance_id_from_provider_id("aws:///us-east-1a/i-0abc") == "i-0abc" and instance_id_from_provider_id("i-9") == "i-9"
    with pytest.raises(ValueError):
        instance_id_from_provider_id("openstack:///1234")
    # a wrong secret is refused by the service (the signature is really checked)
    bad = get_cloud_provider("aws", aws.config(**{"access-key-id": "AKIDAMDKUBETEST", "secret-access-key": "nope"}))
    with pytest.raises(AWSError) as ei:
        asyncio.run(bad.instances().instance_type(name))
    assert ei.value.code == "SignatureDoesNotMatch"
    # the zone comes from the metadata service when the config has none; an INI aws.conf parses
    cfg = aws.config()
    del cfg["Global"]["Zone"]
    assert get_cloud_provider("aws", cfg).zone == "us-east-1b"      # the metadata's own instance


def test_ini_config_and_routes(aws, tmp_path):
    a = aws.add_instance("10.0.0.11")
    rtb = aws.add_route_table()
    aws.add_route_table(tagged=False)                   # another cluster's table is ignored
    conf = tmp_path / "aws.conf"
    conf.write_text(f"[Global]\nZone = us-east-1a\nKubernetesClusterID = {aws.cluster}\nec2-endpoint = {aws.url}/ec2/\n"
                    f"elb-endpoint = {aws.url}/elb/\nmetadata-url = {aws.url}/latest/meta-data/\n")
    cloud = get_cloud_provider("aws", load_config(str(conf)))
    rt = cloud.routes()
    r = Route("", a["privateDnsName"], "10.244.1.0/24")
    rt.create("kubernetes", "hint", r)
    assert aws.tables[rtb]["routeSet"] == [{"destinationCidrBlock": "10.244.1.0/24", "instanceId": a["instanceId"], "state": "active"}]
    assert aws.instances[a["instanceId"]]["sourceDestCheck"] is False
    assert rt.list("kubernetes") == [Route("kubernetes-10.244.1.0/24", a["privateDnsName"], "10.244.1.0/24")]
    # a blackhole route for the CIDR (its instance died) is replaced
    aws.tables[rtb]["routeSet"][0].update(state="blackhole", instanceId="i-gone")
    assert rt.list("kubernetes") == [Route("kubernetes-10.244.1.0/24", "", "10.244.1.0/24")]
    rt.create("kubernetes", "hint", r)
    assert aws.tables[rtb]["routeSet"][0]["state"] == "active"
    rt.delete("kubernetes", r)
    assert aws.tables[rtb]["routeSet"] == []
    rt.delete("kubernetes", r)                          # already gone: fine


def _svc(ports, ann=None, uid="0f9a2c3e-1111-2222-3333-444455556666", **spec):
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": "inference", "namespace": "ml", "uid": uid, "annotations": ann or {}},
            "spec": {"type": "LoadBalancer", "ports": [{"port": p, "nodePort": np, "protocol": "TCP"} for p, np in ports], **spec}}


def _node(inst):
    return {"metadata": {"name": inst["privateDnsName"]}, "spec": {"providerID": f"aws:///us-east-1a/{inst['instanceId']}"}}


def test_listeners_from_annotations():
    ann = {"service.beta.kubernetes.io/aws-load-balancer-ssl-cert": "arn:aws:acm:cert/1",
           "service.beta.kubernetes.io/aws-load-balancer-ssl-ports": "443",
           "service.beta.kubernetes.io/aws-load-balancer-backend-protocol": "http"}
    got = listeners_for(_svc([(80, 30080), (443, 30443)], ann))
    assert got == [{"Protocol": "HTTP", "LoadBalancerPort": 80, "InstanceProtocol": "HTTP", "InstancePort": 30080},
                   {"Protocol": "HTTPS", "LoadBalancerPort": 443, "InstanceProtocol": "HTTP", "InstancePort": 30443,
                    "SSLCertificateId": "arn:aws:acm:cert/1"}]
    assert listeners_for(_svc([(80, 30080)])) == [{"Protocol": "TCP", "LoadBalancerPort": 80, "InstanceProtocol": "TCP", "InstancePort": 30080}]
    with pytest.raises(ValueError):
        listeners_for({"metadata": {}, "spec": {"ports": [{"port": 53, "nodePort": 30053, "protocol": "UDP"}]}})


def test_classic_elb_lifecycle(aws):
    node_sg = aws.add_group("k8s-nodes")
    a = aws.add_instance("10.0.0.11", groups=[node_sg])
    b = aws.add_instance("10.0.0.12", az="us-east-1b", groups=[node_sg])
    c3 = aws.add_instance("10.0.0.13", groups=[node_sg])
    s1 = aws.add_subnet("us-east-1a")
    s1elb = aws.add_subnet("us-east-1a", role="kubernetes.io/role/elb")
    s2 = aws.add_subnet("us-east-1b")
    aws.add_subnet("us-east-1c", tagged=False)         # not the cluster's
    cloud = get_cloud_provider("aws", aws.config())
    lb = cloud.load_balancer()
    ann = {"service.beta.kubernetes.io/aws-load-balancer-connection-idle-timeout": "300",
           "service.beta.kubernetes.io/aws-load-balancer-cross-zone-load-balancing-enabled": "true",
           "service.beta.kubernetes.io/aws-load-balancer-healthcheck-interval": "7"}
    svc = _svc([(80, 30080), (443, 30443)], ann, loadBalancerSourceRanges=["10.1.0.0/16"])
    st = lb.ensure("kubernetes", svc, [_node(a), _node(b)])
    name = lb_name(svc)
    assert name == "a0f9a2c3e111122223333444455556666"[:32] and list(aws.lbs) == [name]
    obj = aws.lbs[name]
    assert st == {"ingress": [{"hostname": obj["DNSName"]}]} and obj["Scheme"] == "internet-facing"
    assert sorted(obj["Subnets"]) == sorted([s1elb, s2]) and s1 not in obj["Subnets"]       # role-tagged subnet wins in 1a
    assert sorted((li["LoadBalancerPort"], li["InstancePort"]) for li in obj["Listeners"]) == [("443", "30443"), ("80", "30080")]
    assert sorted(obj["Instances"]) == sorted([a["instanceId"], b["instanceId"]])
    assert obj["HealthCheck"]["Target"] == "TCP:30080" and obj["HealthCheck"]["Interval"] == "7"
    assert obj["Attributes"]["ConnectionSettings.IdleTimeout"] == "300" and obj["Attributes"]["CrossZoneLoadBalancing.Enabled"] == "true"
    assert obj["Tags"]["kubernetes.io/service-name"] == "ml/inference"
    elb_sg = obj["SecurityGroups_"][0]["groupId"]
    g = aws.groups[elb_sg]
    assert g["groupName"] == f"k8s-elb-{name}"
    assert sorted((p["ipProtocol"], p["fromPort"], p["ipRanges"][0]["cidrIp"]) for p in g["ipPermissions"]) == [
        ("icmp", 3, "0.0.0.0/0"), ("tcp", 80, "10.1.0.0/16"), ("tcp", 443, "10.1.0.0/16")]
    assert any(x["groupId"] == elb_sg for p in aws.groups[node_sg]["ipPermissions"] for x in p["groups"])
    assert lb.get("kubernetes", svc) == (st, True)
    # node churn re-registers; a port change rewrites the listeners and the SG rules
    lb.update("kubernetes", svc, [_node(b), _node(c3)])
    assert sorted(aws.lbs[name]["Instances"]) == sorted([b["instanceId"], c3["instanceId"]])
    svc2 = _svc([(8080, 31080)], ann)
    lb.ensure("kubernetes", svc2, [_node(b)])
    assert [(li["LoadBalancerPort"], li["InstancePort"]) for li in aws.lbs[name]["Listeners"]] == [("8080", "31080")]
    assert sorted((p["ipProtocol"], p["fromPort"]) for p in aws.groups[elb_sg]["ipPermissions"]) == [("icmp", 3), ("tcp", 8080)]
    # an internal ELB and validation errors
    with pytest.raises(ValueError):
        lb.ensure("kubernetes", _svc([(80, 30080)], loadBalancerIP="1.2.3.4"), [])
    with pytest.raises(ValueError):
        lb.ensure("kubernetes", _svc([(80, 30080)], sessionAffinity="ClientIP"), [])
    lb.ensure_deleted("kubernetes", svc)
    assert name not in aws.lbs and elb_sg not in aws.groups
    assert not any(x["groupId"] == elb_sg for p in aws.groups[node_sg]["ipPermissions"] for x in p["groups"])
    assert lb.get("kubernetes", svc) == (None, False)
    lb.ensure_deleted("kubernetes", svc)                # idempotent
    intl = _svc([(80, 30080)], {"service.beta.kubernetes.io/aws-load-balancer-internal": "0.0.0.0/0"}, uid="aaaa-bbbb")
    st = lb.ensure("kubernetes", intl, [_node(a)])
    assert aws.lbs[lb_name(intl)]["Scheme"] == "internal" and st["ingress"][0]["hostname"].startswith("internal-")
    assert aws.bad_signatures == 0


def test_ebs_volumes_allocator_and_plugin(aws, tmp_path):
    from amdkube.volume import NoopMounter, PluginMgr, Spec, VolumeHost, default_plugins
    a = aws.add_instance("10.0.0.11", az="us-east-1a")
    aws.add_instance("10.0.0.12", az="us-east-1b")
    cloud = get_cloud_provider("aws", aws.config())
    vols = cloud.volumes()
    vols.poll = 0.01
    src, labels = vols.provision("pvc-1", 100, {"type": "io1", "iopsPerGB": "50", "zone": "us-east-1a", "fsType": "xfs"},
                                 {"kubernetes.io/created-for/pvc/name": "data"}, "data")
    vid = volume_id(src["volumeID"])
    v = aws.volumes[vid]
    assert src == {"volumeID": f"aws://us-east-1a/{vid}", "fsType": "xfs"}
    assert (v["size"], v["volumeType"], v["iops"]) == ("100", "io1", "5000")
    assert {"key": "kubernetes.io/cluster/mi355x", "value": "owned"} in v["tagSet"]
    assert labels == {"failure-domain.beta.kubernetes.io/zone": "us-east-1a", "failure-domain.beta.kubernetes.io/region": "us-east-1"}
    dev_root = tmp_path / "root"
    host = VolumeHost(str(tmp_path / "kubelet"), node_name=a["privateDnsName"], mounter=NoopMounter())
    host.cloud, host.dev_root, host.attach_poll = cloud, str(dev_root), 0.01
    pv = {"metadata": {"name": "pv-1"}, "spec": {"awsElasticBlockStore": src}}
    spec = Spec(pv=pv)
    plugin = PluginMgr(default_plugins(), host).find_by_spec(spec)
    assert plugin.name == "kubernetes.io/aws-ebs"

    async def go():
        dev = await plugin.attach(spec, a["privateDnsName"])
        assert dev == "/dev/xvdba" and aws.volumes[vid]["attachmentSet"][0]["instanceId"] == a["instanceId"]
        assert await plugin.attach(spec, a["privateDnsName"]) == dev          # idempotent
        # a Nitro GPU instance shows the disk as NVMe by its volume id
        nv = dev_root / "dev" / "disk" / "by-id"
        nv.mkdir(parents=True)
        (nv / f"nvme-Amazon_Elastic_Block_Store_{vid.replace('-', '')}").write_text("")
        found = await plugin.wait_for_attach(spec, dev, None, 5)
        assert found.endswith(f"nvme-Amazon_Elastic_Block_Store_{vid.replace('-', '')}")
        with pytest.raises(AWSError):
            vols.delete(src["volumeID"])               # in use
        await plugin.detach(src["volumeID"], a["privateDnsName"])
        assert aws.volumes[vid]["status"] == "available"
    asyncio.run(go())
    assert cloud.labels_for_volume(pv) == labels
    assert vols.delete(src["volumeID"]) and not vols.delete(src["volumeID"])
    # dynamic zone choice follows the zones that run (non-master) instances
    kid = vols.create("z", 1, {}, {}, "claim")
    assert kid.split("/")[2] in ("us-east-1a", "us-east-1b")
    # the device allocator hands out the least recently used device
    al = DeviceAllocator()
    assert [al.next(set()) for _ in range(2)] == ["ba", "bb"] and al.next({"bc"}) == "bd"
    assert choose_zone(["b", "a"], "data-web-0") != choose_zone(["b", "a"], "data-web-1")
    with pytest.raises(ValueError):
        volume_id("aws://us-east-1a/not-a-volume")


def test_controllers_and_kubelet_drive_aws(aws):
    """service-LB, route and PV-binder controllers against the AWS provider, and a kubelet
    --cloud-provider=aws registering with the instance's providerID, type, zone and addresses."""
    inst = aws.add_instance("10.0.0.21", public="198.51.100.9", itype="gpu.mi355x.48xlarge")
    aws.add_subnet("us-east-1a")
    rtb = aws.add_route_table()
    node = inst["privateDnsName"]

    async def go():
        import json
        import tempfile
        cfgf = tempfile.NamedTemporaryFile("w", suffix=".json", delete=False)
        json.dump(aws.config(), cfgf)
        cfgf.close()
        async with LocalCluster(gpus="fake", n_gpus=1, with_controllers=False, relist_period=0.2, node_name=node,
                                kubelet_kw={"cloud_provider": "aws", "cloud_config": cfgf.name}) as lc:
            c = lc.client
            n = await c.get("nodes", node)
            assert n["spec"]["providerID"] == f"aws:///us-east-1a/{inst['instanceId']}"
            lab = m.labels_of(n)
            assert lab["beta.kubernetes.io/instance-type"] == "gpu.mi355x.48xlarge"
            assert (lab["failure-domain.beta.kubernetes.io/zone"], lab["failure-domain.beta.kubernetes.io/region"]) == \
                ("us-east-1a", "us-east-1")
            assert {"type": "ExternalIP", "address": "198.51.100.9"} in n["status"]["addresses"]
            await c.patch("nodes", node, {"spec": {"podCIDR": "10.244.9.0/24"}})
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default"},
                            "spec": {"type": "LoadBalancer", "ports": [{"port": 80, "protocol": "TCP"}]}}, "default")
            await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": "ebs"},
                            "provisioner": "kubernetes.io/aws-ebs", "parameters": {"type": "gp2", "zone": "us-east-1a"}})
            await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data", "namespace": "default"},
                            "spec": {"storageClassName": "ebs", "accessModes": ["ReadWriteOnce"],
                                     "resources": {"requests": {"storage": "1536Mi"}}}}, "default")
            cloud = get_cloud_provider("aws", aws.config())
            cloud.volumes().poll = 0.01
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

                async def lb_host():
                    s = await c.get("services", "web", "default")
                    return ((s.get("status") or {}).get("loadBalancer") or {}).get("ingress")
                ing = await until(lb_host)
                assert ing[0]["hostname"].endswith(".elb.amazonaws.com")

                async def routed():
                    return aws.tables[rtb]["routeSet"]
                assert (await until(routed))[0]["destinationCidrBlock"] == "10.244.9.0/24"

                async def bound():
                    p = await c.get("persistentvolumeclaims", "data", "default")
                    return p if (p.get("status") or {}).get("phase") == "Bound" else None
                pvc = await until(bound)
                pv = await c.get("persistentvolumes", pvc["spec"]["volumeName"])
                vid = volume_id(pv["spec"]["awsElasticBlockStore"]["volumeID"])
                assert aws.volumes[vid]["size"] == "2" and pv["spec"]["capacity"]["storage"] == "2Gi"
                assert m.labels_of(pv)["failure-domain.beta.kubernetes.io/zone"] == "us-east-1a"
                await c.delete("persistentvolumeclaims", "data", "default")

                async def gone():
                    return vid not in aws.volumes
                await until(gone)
            finally:
                await cm.stop()
                await cmc.close()
    run(go(), 90)
    assert aws.bad_signatures == 0
