"""Volume-aware scheduling (predicates_test.go TestVolumeZonePredicate / TestEBSVolumeCountConflicts,
scheduler_binder_test.go, test/integration/scheduler/volume_binding_test.go): zone labels of
bound PVs, cloud-disk count limits, local-PV node affinity, and delayed binding of
WaitForFirstConsumer claims to a PV on the node the scheduler picks."""
import asyncio
import json
import os

import pytest

from amdkube.api import meta as m
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.scheduler.generic import FitError
from amdkube.scheduler.volumes import NODE_AFFINITY_ANN, VolumeLister
from tests.conftest import run
from tests.test_scheduler import node, pod, sched


def _pv(name, size="10Gi", cls="", zone=None, host=None, claim=None, **src):
    md = {"name": name, "labels": {}, "annotations": {}}
    if zone:
        md["labels"]["failure-domain.beta.kubernetes.io/zone"] = zone
    if host:
        md["annotations"][NODE_AFFINITY_ANN] = json.dumps({"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": [{"matchExpressions": [{"key": "kubernetes.io/hostname", "operator": "In", "values": [host]}]}]}})
    spec = {"capacity": {"storage": size}, "accessModes": ["ReadWriteOnce"], "storageClassName": cls, **src}
    if claim:
        spec["claimRef"] = {"namespace": "default", "name": claim}
    return {"kind": "PersistentVolume", "metadata": md, "spec": spec, "status": {"phase": "Bound" if claim else "Available"}}


def _pvc(name, size="5Gi", cls="", volume=None):
    return {"kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}"},
            "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": size}}, "storageClassName": cls,
                     **({"volumeName": volume} if volume else {})}}


def _vpod(name, *claims, inline=()):
    p = pod(name)
    p["spec"]["volumes"] = [{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}} for i, c in enumerate(claims)] + list(inline)
    return p


def _nodes(*zones):
    out = []
    for i, z in enumerate(zones):
        n = node(f"n{i}", gpus=0, topo=False)
        n["metadata"]["labels"]["kubernetes.io/hostname"] = f"n{i}"
        if z:
            n["metadata"]["labels"]["failure-domain.beta.kubernetes.io/zone"] = z
        out.append(n)
    return out


def _sched(nodes, pvs=(), pvcs=(), classes=(), gate=True):
    c, g = sched(nodes)
    g.volumes = VolumeLister({f"default/{m.name_of(x)}": x for x in pvcs}, {m.name_of(x): x for x in pvs},
                             {m.name_of(x): x for x in classes})
    g.volume_scheduling = gate
    return c, g


def test_zone_conflict_and_missing_claims():
    pv = _pv("pv-a", zone="rack-a__rack-b", claim="data")
    c, g = _sched(_nodes("rack-a", "rack-c", None), [pv], [_pvc("data", volume="pv-a")])
    fit, failed, _ = asyncio.run(g.find_nodes_that_fit(_pi(g, _vpod("p", "data")), c.ready_nodes()))
    assert sorted(ni.name for ni in fit) == ["n0", "n2"]        # rack-a is one of the PV's zones; n2 has no zone
    assert failed["n1"] == ["NoVolumeZoneConflict"]
    with pytest.raises(FitError) as e:
        asyncio.run(g.schedule(_vpod("q", "nope")))
    assert 'persistentvolumeclaim "nope" not found' in str(e.value)


def _pi(g, p):
    from amdkube.scheduler.predicates import PodInfo
    from amdkube.scheduler.volumes import pod_volumes
    pi = PodInfo(p)
    pi.lister, pi.volume_scheduling, pi.vol = g.volumes, g.volume_scheduling, pod_volumes(p, g.volumes)
    return pi


def test_max_cloud_disk_count_and_disk_conflicts(monkeypatch):
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", "2")
    c, g = _sched(_nodes(None), [_pv("gce-pv", claim="g3", gcePersistentDisk={"pdName": "pd-3"})],
                  [_pvc("g3", volume="gce-pv")])
    gce = lambda i, ro=True: {"name": f"d{i}", "gcePersistentDisk": {"pdName": f"pd-{i}", "readOnly": ro}}   # noqa: E731
    for i in (1, 2):
        p = _vpod(f"p{i}", inline=[gce(i)])
        p["spec"]["nodeName"] = "n0"
        c.add_pod(p)
    asyncio.run(g.schedule(_vpod("same", inline=[gce(1)])))             # shared read-only, already counted
    with pytest.raises(FitError) as e:
        asyncio.run(g.schedule(_vpod("same-rw", inline=[gce(1, False)])))
    assert "NoDiskConflict" in str(e.value)                      # NoDiskConflict: a writer needs it alone
    with pytest.raises(FitError) as e:
        asyncio.run(g.schedule(_vpod("third", inline=[gce(9)])))
    assert "MaxVolumeCount" in str(e.value)
    with pytest.raises(FitError):
        asyncio.run(g.schedule(_vpod("via-pv", "g3")))                 # counted through its PV too
    asyncio.run(g.schedule(_vpod("ebs", inline=[{"name": "e", "awsElasticBlockStore": {"volumeID": "v"}}])))   # other kind
    p = _vpod("ebs-user", inline=[{"name": "e", "awsElasticBlockStore": {"volumeID": "v", "readOnly": True}}])
    p["spec"]["nodeName"] = "n0"
    c.add_pod(p)
    with pytest.raises(FitError):    # EBS cannot be shared at all, read-only or not
        asyncio.run(g.schedule(_vpod("ebs2", inline=[{"name": "e", "awsElasticBlockStore": {"volumeID": "v", "readOnly": True}}])))


def test_local_pv_affinity_and_delayed_binding_choice():
    wffc = {"kind": "StorageClass", "metadata": {"name": "local"}, "provisioner": "kubernetes.io/no-provisioner",
            "volumeBindingMode": "WaitForFirstConsumer"}
    pvs = [_pv("small-on-n0", "20Gi", "local", host="n0", local={"path": "/mnt/a"}),
           _pv("big-on-n1", "500Gi", "local", host="n1", local={"path": "/mnt/b"}),
           _pv("mid-on-n1", "100Gi", "local", host="n1", local={"path": "/mnt/c"}),
           _pv("bound-on-n0", "1Gi", host="n0", claim="pinned", local={"path": "/mnt/d"})]
    pvcs = [_pvc("scratch", "50Gi", "local"), _pvc("pinned", volume="bound-on-n0"), _pvc("imm", "1Gi", "")]
    c, g = _sched(_nodes(None, None), pvs, pvcs, [wffc])
    host, _ = asyncio.run(g.schedule(_vpod("p", "scratch")))
    assert host == "n1" and [(m.name_of(a), m.name_of(b)) for a, b in g.volume_binds["default/p"]] == [("scratch", "mid-on-n1")]
    host, _ = asyncio.run(g.schedule(_vpod("q", "pinned")))          # bound local PV pins the pod to its node
    assert host == "n0"
    with pytest.raises(FitError) as e:
        asyncio.run(g.schedule(_vpod("r", "pinned", "scratch")))     # n0 has no 50Gi volume; n1 is not the pinned node
    assert "VolumeNodeAffinityConflict" in str(e.value) and "VolumeBindingNoMatch" in str(e.value)
    with pytest.raises(FitError) as e:
        asyncio.run(g.schedule(_vpod("s", "imm")))
    assert "unbound PersistentVolumeClaims" in str(e.value)
    g.volume_scheduling = False                                       # gate off: binding is the PV controller's
    assert asyncio.run(g.schedule(_vpod("t", "scratch")))[0] in ("n0", "n1")


def test_wait_for_first_consumer_end_to_end(tmp_path):
    path = tmp_path / "nvme0"
    path.mkdir()

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, scheduler_kw={"feature_gates": "VolumeScheduling=true"},
                                kubelet_kw={"volume_reconcile_period": 0.2}) as lc:
            c = lc.client
            await c.create({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": "local-nvme"},
                            "provisioner": "kubernetes.io/no-provisioner", "volumeBindingMode": "WaitForFirstConsumer"})
            for name, host, size, p in (("elsewhere", "other-node", "100Gi", "/nonexistent"),
                                        ("here", lc.node_name, "200Gi", str(path))):
                pv = _pv(name, size, "local-nvme", host=host, local={"path": p})
                pv["apiVersion"] = "v1"
                pv.pop("status")
                await c.create(pv)
            await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "ds"},
                            "spec": {"accessModes": ["ReadWriteOnce"], "storageClassName": "local-nvme",
                                     "resources": {"requests": {"storage": "50Gi"}}}}, "default")
            await asyncio.sleep(1.0)
            claim = await c.get("persistentvolumeclaims", "ds", "default")
            assert not claim["spec"].get("volumeName")                  # not bound before a consumer exists
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "reader"}, "spec": {
                "volumes": [{"name": "d", "persistentVolumeClaim": {"claimName": "ds"}}],
                "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "echo hi > $AMDKUBE_ROOTFS/d/out; sleep 30"],
                                "volumeMounts": [{"name": "d", "mountPath": "/d"}]}]}}, "default")
            p = await wait_pod(c, "default", "reader", timeout=40)
            assert p["spec"]["nodeName"] == lc.node_name
            claim = await c.get("persistentvolumeclaims", "ds", "default")
            assert claim["spec"]["volumeName"] == "here" and claim["status"]["phase"] == "Bound"
            for _ in range(100):
                if os.path.exists(path / "out"):
                    break
                await asyncio.sleep(0.1)
            assert (path / "out").read_text().strip() == "hi"
    run(go(), 90)
