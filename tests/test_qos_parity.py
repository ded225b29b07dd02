"""QoS class and OOM score adjustment held to the reference's tables.

* pkg/apis/core/v1/helper/qos/qos_test.go TestGetPodQOS :30 — every case (the `nvidia-gpu`
  extended resource of the reference is carried as written; it is not a QoS compute resource).
* pkg/kubelet/qos/policy_test.go TestGetContainerOOMScoreAdjust :147 — every case, with the
  reference's low/high bounds.
Both feed pods as the tests build them, without API defaulting.
"""
from __future__ import annotations

import pytest

from amdkube.kubelet.qos import BEST_EFFORT, BURSTABLE, GUARANTEED, oom_score_adj, pod_qos


def rl(cpu="", memory="", **extra):
    out = {}
    if cpu:
        out["cpu"] = cpu
    if memory:
        out["memory"] = memory
    out.update({k.replace("_", "-"): v for k, v in extra.items()})
    return out


def gpu(r):
    return {**r, "nvidia-gpu": "2"}


def pod(*containers):
    return {"metadata": {"name": "p"}, "spec": {"containers": [{"name": f"c{i}", "resources": {"requests": rq, "limits": li}}
                                                               for i, (rq, li) in enumerate(containers)]}}


HP = {"hugepages_2Mi": "1Gi"}
QOS = [
    ("guaranteed", [(rl("100m", "100Mi"), rl("100m", "100Mi"))], GUARANTEED),
    ("guaranteed-with-gpu", [(rl("100m", "100Mi"), gpu(rl("100m", "100Mi")))], GUARANTEED),
    ("guaranteed-guaranteed", [(rl("100m", "100Mi"), rl("100m", "100Mi"))] * 2, GUARANTEED),
    ("guaranteed-guaranteed-with-gpu", [(rl("100m", "100Mi"), gpu(rl("100m", "100Mi"))), (rl("100m", "100Mi"), rl("100m", "100Mi"))],
     GUARANTEED),
    ("best-effort-best-effort", [(rl(), rl())] * 2, BEST_EFFORT),
    ("best-effort-best-effort-with-gpu", [(rl(), gpu(rl())), (rl(), rl())], BEST_EFFORT),
    ("best-effort-with-gpu", [(rl(), gpu(rl()))], BEST_EFFORT),
    ("best-effort-burstable", [(rl(), gpu(rl())), (rl("1"), rl("2"))], BURSTABLE),
    ("best-effort-guaranteed", [(rl(), gpu(rl())), (rl("10m", "100Mi"), rl("10m", "100Mi"))], BURSTABLE),
    ("burstable-cpu-guaranteed-memory", [(rl("", "100Mi"), rl("", "100Mi"))], BURSTABLE),
    ("burstable-no-limits", [(rl("100m", "100Mi"), rl())], BURSTABLE),
    ("burstable-guaranteed", [(rl("1", "100Mi"), rl("2", "100Mi")), (rl("100m", "100Mi"), rl("100m", "100Mi"))], BURSTABLE),
    ("burstable-unbounded-but-requests-match-limits", [(rl("100m", "100Mi"), rl("200m", "200Mi")), (rl("100m", "100Mi"), rl())],
     BURSTABLE),
    ("burstable-1", [(rl("10m", "100Mi"), rl("100m", "200Mi"))], BURSTABLE),
    ("burstable-2", [(rl("0", "0"), gpu(rl("100m", "200Mi")))], BURSTABLE),
    ("burstable-hugepages", [(rl("0", "0", **HP), rl("0", "0", **HP))], BURSTABLE),
]


@pytest.mark.parametrize("name,containers,expected", QOS, ids=[q[0] for q in QOS])
def test_get_pod_qos(name, containers, expected):
    assert pod_qos(pod(*containers)) == expected


STANDARD = 8000000000
OOM = [
    ("cpuLimit", (rl(), rl("10")), 4000000000, 999, 999),
    ("memoryLimitCPURequest", (rl("0"), rl("", "10G")), 8000000000, 999, 999),
    ("zeroMemoryLimit", (rl(), rl("", "0")), 7230457451, 1000, 1000),
    ("noRequestLimit", (rl(), rl()), 4000000000, 1000, 1000),
    ("equalRequestLimitCPUMemory", (rl("5m", "10G"), rl("5m", "10G")), 123456789, -998, -998),
    ("cpuUnlimitedMemoryLimitedWithRequests", (rl("5m", str(STANDARD // 2)), rl("", "10G")), STANDARD, 495, 505),
    ("requestNoLimit", (rl("5m", str(STANDARD - 1)), rl()), STANDARD, 2, 2),
]


@pytest.mark.parametrize("name,container,capacity,low,high", OOM, ids=[o[0] for o in OOM])
def test_get_container_oom_score_adjust(name, container, capacity, low, high):
    p = pod(container)
    assert low <= oom_score_adj(p, p["spec"]["containers"][0], capacity) <= high
