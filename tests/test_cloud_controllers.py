"""cloud-controller-manager (pkg/controller/cloud/node_controller_test.go, pvlcontroller_test.go):
a kubelet started with --cloud-provider=external registers tainted and without addresses;
the cloud node controller initialises it from the provider's inventory (providerID,
addresses honouring the kubelet's provided IP, instance type and zone labels), drops the taint
so pods schedule, and deletes NotReady nodes the cloud no longer knows; the PV labeler labels
initializer-pending volumes and publishes them."""
import asyncio

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.cloudprovider import get_cloud_provider
from amdkube.controllers import ControllerManager, Options
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


async def _until(fn, timeout=20.0):
    end = asyncio.get_running_loop().time() + timeout
    while True:
        v = await fn()
        if v:
            return v
        if asyncio.get_running_loop().time() > end:
            raise AssertionError("condition not met")
        await asyncio.sleep(0.05)


def test_cloud_node_initialisation_monitoring_and_pv_labels():
    async def go():
        chain = ("NamespaceLifecycle", "Initializers", "ResourceV2")
        async with LocalCluster(gpus="none", with_controllers=False, relist_period=0.2, node_status_update_frequency=0.3,
                                kubelet_kw={"cloud_provider": "external", "node_ip": "127.0.0.1"},
                                api_kw={"admission_plugins": chain}) as lc:
            c = lc.client
            node = await c.get("nodes", lc.node_name)
            assert [t["key"] for t in node["spec"]["taints"]] == ["node.cloudprovider.kubernetes.io/uninitialized"]
            assert m.annotations_of(node)["alpha.kubernetes.io/provided-node-ip"] == "127.0.0.1"
            assert not node["status"].get("addresses")
            # tainted: a pod waits for the cloud
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "w"}, "spec": {
                "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"]}]}}, "default")
            await asyncio.sleep(0.5)
            assert not (await c.get("pods", "w", "default"))["spec"].get("nodeName")
            cloud = get_cloud_provider("baremetal", {"zone": "rack-7", "region": "dc-west", "instances": {
                lc.node_name: {"providerID": "baremetal://dc-west/rack-7/u12", "instanceType": "amd-mi355x-8gpu", "zone": "rack-7",
                               "region": "dc-west", "addresses": [{"type": "InternalIP", "address": "127.0.0.1"},
                                                                  {"type": "ExternalIP", "address": "203.0.113.9"}]}}})
            await c.create({"apiVersion": "admissionregistration.k8s.io/v1alpha1", "kind": "InitializerConfiguration",
                            "metadata": {"name": "pvl"}, "initializers": [{"name": "pvl.kubernetes.io", "rules": [
                                {"apiGroups": [""], "apiVersions": ["v1"], "resources": ["persistentvolumes"]}]}]})
            ccm = await ControllerManager(Client(lc.api.url, token=lc.api.loopback_token), ["cloud-node", "persistentvolume-labeler"],
                                          options=Options(cloud=cloud, extra={"node_status_update_frequency": 0.3,
                                                                              "node_monitor_period": 0.2})).start()
            try:
                async def initialised():
                    n = await c.get("nodes", lc.node_name)
                    return n if not n["spec"].get("taints") and n["status"].get("addresses") else None
                n = await _until(initialised)
                assert n["spec"]["providerID"] == "baremetal://dc-west/rack-7/u12"
                lab = m.labels_of(n)
                assert lab["beta.kubernetes.io/instance-type"] == "amd-mi355x-8gpu"
                assert lab["failure-domain.beta.kubernetes.io/zone"] == "rack-7"
                assert lab["failure-domain.beta.kubernetes.io/region"] == "dc-west"
                # the kubelet's --node-ip wins over the cloud's other addresses; the hostname is kept
                assert [a["address"] for a in n["status"]["addresses"]] == ["127.0.0.1"]
                await asyncio.sleep(0.8)      # kubelet status updates do not take the addresses back
                assert [a["address"] for a in (await c.get("nodes", lc.node_name))["status"]["addresses"]] == ["127.0.0.1"]
                pod = await wait_pod(c, "default", "w", timeout=20)
                assert pod["spec"]["nodeName"] == lc.node_name
                # a NotReady node the cloud does not know is deleted; a Ready one stays
                for name, ready in (("ghost", "False"), ("live", "True")):
                    await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": name},
                                    "status": {"conditions": [{"type": "Ready", "status": ready}]}})

                async def ghost_gone():
                    return await c.get_or_none("nodes", "ghost") is None
                await _until(ghost_gone)
                assert await c.get_or_none("nodes", "live") is not None
                # PV labeler: local volumes get the zone, then become visible
                aff = ('{"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [{"matchExpressions": '
                       '[{"key": "kubernetes.io/hostname", "operator": "In", "values": ["live"]}]}]}}')
                pv = {"apiVersion": "v1", "kind": "PersistentVolume", "metadata": {
                          "name": "scratch", "annotations": {"volume.alpha.kubernetes.io/node-affinity": aff}},
                      "spec": {"capacity": {"storage": "1Ti"}, "accessModes": ["ReadWriteOnce"], "local": {"path": "/mnt/nvme0"}}}
                created = await c.request("POST", "/api/v1/persistentvolumes", params={"includeUninitialized": "true"}, body=pv)
                assert created["metadata"]["initializers"]["pending"] == [{"name": "pvl.kubernetes.io"}]

                async def published():      # listed (ordinary lists hide uninitialized objects)
                    items = (await c.request("GET", "/api/v1/persistentvolumes"))["items"]
                    return next((x for x in items if m.name_of(x) == "scratch"), None)
                got = await _until(published)
                assert m.labels_of(got)["failure-domain.beta.kubernetes.io/zone"] == "rack-7"
                assert "initializers" not in got["metadata"] or not got["metadata"]["initializers"].get("pending")
            finally:
                await ccm.stop()
                await ccm.client.close()
    run(go(), 90)


def test_cloud_controller_manager_controller_set():
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-m", "amdkube", "cloud-controller-manager", "--cloud-provider", "baremetal",
                        "--controllers", "*,-nope", "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--cloud-config" in r.stdout
    from amdkube.controllers import ALL, CLOUD_CONTROLLERS, Options, default_controllers
    assert set(CLOUD_CONTROLLERS) <= set(ALL)
    assert not set(CLOUD_CONTROLLERS) & set(default_controllers(Options()))   # kube-controller-manager without a cloud
