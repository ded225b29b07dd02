"""pkg/api/v1/pod/util_test.go held against amdkube's pod helpers: TestFindPort :32 (every case;
an error is `None`, whose port the reference reports as 0) and TestIsPodAvailable :371."""
from __future__ import annotations

import pytest

from amdkube.api import meta as m
from amdkube.controllers.networking import find_port
from amdkube.controllers.replicaset import is_pod_available


def _ports(*ps):
    return [{}, {"ports": [dict(zip(("name", "containerPort", "protocol"), p[:3]), **(p[3] if len(p) > 3 else {})) for p in ps]}]


@pytest.mark.parametrize("name,containers,port,expected", [
    ("valid int, no ports", [{}], 93, 93),
    ("valid int, with ports", [{"ports": [{"name": "", "containerPort": 11, "protocol": "TCP"},
                                          {"name": "p", "containerPort": 22, "protocol": "TCP"}]}], 93, 93),
    ("valid str, no ports", [{}], "p", None),
    ("valid str, one ctr with ports", _ports(("", 11, "UDP"), ("p", 22, "TCP"), ("q", 33, "TCP"))[1:], "q", 33),
    ("valid str, two ctr with ports", _ports(("", 11, "UDP"), ("p", 22, "TCP"), ("q", 33, "TCP")), "q", 33),
    ("valid str, two ctr with same port", _ports(("", 11, "UDP"), ("p", 22, "TCP"), ("q", 22, "TCP")), "q", 22),
    ("valid str, invalid protocol", _ports(("a", 11, "snmp")), "a", None),
    ("valid hostPort", _ports(("a", 11, "TCP", {"hostPort": 81})), "a", 11),
    ("invalid hostPort", _ports(("a", 11, "TCP", {"hostPort": -1})), "a", 11),
    ("invalid ContainerPort", _ports(("a", -1, "TCP")), "a", -1),
    ("HostIP Address", _ports(("a", 11, "TCP", {"hostIP": "192.168.1.1"})), "a", 11),
])
def test_find_port(name, containers, port, expected):
    assert find_port({"spec": {"containers": containers}}, {"protocol": "TCP", "targetPort": port}) == expected


NOW = 1_700_000_000.0


def _pod(ready, seconds_ago):
    return {"status": {"conditions": [{"type": "Ready", "status": "True" if ready else "False",
                                       "lastTransitionTime": m.format_time(NOW - seconds_ago)}]}}


@pytest.mark.parametrize("ready,ago,min_ready,expected", [
    (False, 0, 0, False), (True, 0, 1, False), (True, 0, 0, True), (True, 51, 50, True),
])
def test_is_pod_available(ready, ago, min_ready, expected):
    assert is_pod_available(_pod(ready, ago), min_ready, NOW) is expected


def test_available_needs_strictly_more_than_min_ready():
    """IsPodAvailable uses Time.Before: a pod ready exactly minReadySeconds ago is not yet available."""
    assert is_pod_available(_pod(True, 50), 50, NOW) is False
