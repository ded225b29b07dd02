"""QoS classes, OOM score adjustment and cgroup parents (reference
pkg/apis/core/helper/qos/qos_test.go, pkg/kubelet/qos/policy_test.go)."""
import asyncio

from amdkube.kubelet.qos import BEST_EFFORT, BURSTABLE, GUARANTEED, cgroup_parent, oom_score_adj, pod_qos
from amdkube.localcluster import LocalCluster, wait_pod


def _pod(*resources, uid="u1"):
    return {"metadata": {"uid": uid, "namespace": "default"},
            "spec": {"containers": [{"name": f"c{i}", "resources": r} for i, r in enumerate(resources)]}}


def test_qos_classes_and_oom_scores():
    # API-defaulted shapes: requests filled from limits (GetPodQOS itself does not default)
    g = _pod({"requests": {"cpu": "2", "memory": "4Gi"}, "limits": {"cpu": "2", "memory": "4Gi"}})
    b = _pod({"requests": {"memory": "1Gi"}})
    e = _pod({}, {"limits": {"amd.com/gpu": "1"}})
    assert (pod_qos(g), pod_qos(b), pod_qos(e)) == (GUARANTEED, BURSTABLE, BEST_EFFORT)
    assert pod_qos(_pod({"limits": {"cpu": "1", "memory": "1Gi"}}, {"limits": {"cpu": "1"}})) == BURSTABLE
    assert pod_qos(_pod({"requests": {"cpu": "1", "memory": "1Gi"}, "limits": {"cpu": "2", "memory": "1Gi"}})) == BURSTABLE
    cap = 8 << 30
    assert oom_score_adj(g, g["spec"]["containers"][0], cap) == -998
    assert oom_score_adj(e, e["spec"]["containers"][0], cap) == 1000
    assert oom_score_adj(b, b["spec"]["containers"][0], cap) == 875           # 1000 - 1000 * 1Gi / 8Gi
    huge = _pod({"requests": {"memory": "16Gi"}})
    assert oom_score_adj(huge, huge["spec"]["containers"][0], cap) == 2
    assert cgroup_parent(g) == "kubepods/podu1" and cgroup_parent(b) == "kubepods/burstable/podu1"
    assert cgroup_parent(e) == "kubepods/besteffort/podu1"


async def test_best_effort_container_gets_oom_score_1000():
    async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
        c = lc.client
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "be"},
                        "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"]}]}}, "default")
        await wait_pod(c, "default", "be", ("Running",), 20)
        [ct] = [x for x in lc.shim.containers.values() if x.name == "c"]
        for _ in range(50):
            if open(f"/proc/{ct.pid}/oom_score_adj").read().strip() == "1000":
                break
            await asyncio.sleep(0.05)
        assert open(f"/proc/{ct.pid}/oom_score_adj").read().strip() == "1000"
        assert ct.resources["cgroup_parent"].startswith("kubepods/besteffort/pod")
