"""Services, endpoints, kube-proxy and pod networking (reference
pkg/registry/core/service/rest_test.go, pkg/controller/endpoint/endpoints_controller_test.go,
pkg/proxy/iptables/proxier_test.go, pkg/proxy/userspace/roundrobin_test.go,
pkg/kubelet/network/cni/cni_test.go)."""
from __future__ import annotations

import asyncio
import json
import os
import socket
import urllib.request

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import APIServer
from amdkube.proxy import ProxyServer
from amdkube.proxy.config import ServiceInfo, ServicePortName, endpoints_map, service_infos
from amdkube.proxy.iptables import render, sep_chain, svc_chain
from amdkube.proxy.userspace import LoadBalancerRR
from amdkube.runtime.images import NATIVE_BIN
from amdkube.runtime.network import CNINetwork, NetworkError
from amdkube.store import MVCCStore


def _svc(name, ports, typ="ClusterIP", **spec):
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name},
            "spec": {"type": typ, "selector": {"app": name}, "ports": ports, **spec}}


def test_service_cluster_ip_and_node_port_allocation(tmp_path):
    store = MVCCStore(str(tmp_path / "s"))
    api = APIServer(store, service_cidr="10.96.0.0/29", node_port_range="30000-30002")
    rs = api.registry.rs("services")
    a = rs.create("default", _svc("a", [{"port": 80, "targetPort": 8080}], "NodePort"))
    ip_a, np_a = a["spec"]["clusterIP"], a["spec"]["ports"][0]["nodePort"]
    assert ip_a.startswith("10.96.0.") and ip_a not in ("10.96.0.0", "10.96.0.7")
    assert 30000 <= np_a <= 30002 and a["spec"]["ports"][0]["protocol"] == "TCP"
    # a requested IP that is taken, or outside the range, is rejected (rest.go Create)
    for bad in (ip_a, "10.97.0.1", "not-an-ip"):
        with pytest.raises(m.StatusError) as ei:
            rs.create("default", _svc("b", [{"port": 80}], clusterIP=bad))
        assert ei.value.code == 422
    # clusterIP is immutable; a PUT without clusterIP keeps it; the nodePort survives an update
    cur = rs.get("default", "a")
    cur["spec"]["clusterIP"] = "10.96.0.6" if ip_a != "10.96.0.6" else "10.96.0.5"
    with pytest.raises(m.StatusError):
        rs.update("default", "a", cur)
    cur = rs.get("default", "a")
    del cur["spec"]["clusterIP"]
    cur["spec"]["ports"][0].pop("nodePort")
    upd, _ = rs.update("default", "a", cur)
    assert upd["spec"]["clusterIP"] == ip_a and upd["spec"]["ports"][0]["nodePort"] == np_a
    # headless and ExternalName services get no IP; ClusterIP services get no node ports
    h = rs.create("default", _svc("h", [{"port": 80}], clusterIP="None"))
    assert h["spec"]["clusterIP"] == "None"
    e = rs.create("default", {"metadata": {"name": "ext"}, "spec": {"type": "ExternalName", "externalName": "example.com"}})
    assert "clusterIP" not in e["spec"]
    with pytest.raises(m.StatusError):
        rs.create("default", _svc("np", [{"port": 80, "nodePort": 30001}]))   # nodePort on ClusterIP
    # exhaust the node-port range (3 ports), then deletion releases one
    rs.create("default", _svc("b", [{"port": 80}], "NodePort"))
    rs.create("default", _svc("c", [{"port": 80}], "NodePort"))
    with pytest.raises(m.StatusError) as ei:
        rs.create("default", _svc("d", [{"port": 80}], "NodePort"))
    assert ei.value.code == 500
    rs.delete("default", "c")
    d = rs.create("default", _svc("d", [{"port": 80}], "NodePort"))
    # repair: a restarted apiserver on the same store sees every allocation
    store.close()
    api2 = APIServer(MVCCStore(str(tmp_path / "s")), service_cidr="10.96.0.0/29", node_port_range="30000-30002")
    alloc = api2.registry.services
    assert ip_a in alloc.ips and d["spec"]["clusterIP"] in alloc.ips
    assert {p for _, p in alloc.ports} == {30000, 30001, 30002}


def test_service_validation():
    api = APIServer()
    rs = api.registry.rs("services")
    for spec, frag in (({"ports": [{"port": 0}]}, "spec.ports[0].port"),
                       ({"ports": [{"port": 80, "protocol": "SCTP"}]}, "protocol"),
                       ({"ports": [{"port": 80}, {"port": 81}]}, "name: Required"),
                       ({"ports": [{"name": "a", "port": 80}, {"name": "a", "port": 81}]}, "Duplicate"),
                       ({"type": "Bogus", "ports": [{"port": 80}]}, "spec.type"),
                       ({"type": "ExternalName"}, "externalName"),
                       ({"ports": [{"port": 80}], "sessionAffinity": "Cookie"}, "sessionAffinity")):
        with pytest.raises(m.StatusError) as ei:
            rs.create("default", {"metadata": {"name": "v"}, "spec": spec})
        assert frag in str(ei.value.status()), (spec, ei.value.status())


async def test_kubernetes_master_service():
    api = await APIServer(service_cidr="10.0.0.0/24").start()
    try:
        svc = api.registry.rs("services").get("default", "kubernetes")
        assert svc["spec"]["clusterIP"] == "10.0.0.1" and svc["spec"]["ports"][0]["port"] == 443
        ep = api.registry.rs("endpoints").get("default", "kubernetes")
        assert ep["subsets"][0]["ports"][0]["port"] == api.port
    finally:
        await api.stop()


def test_iptables_ruleset():
    web = ServicePortName("default", "web", "http")
    lonely = ServicePortName("default", "lonely", "")
    svcs = {web: ServiceInfo("10.0.0.10", 80, "TCP", node_port=30080, session_affinity="ClientIP", affinity_timeout=600,
                             external_ips=["192.168.1.5"]),
            lonely: ServiceInfo("10.0.0.11", 53, "UDP")}
    eps = {web: [("10.244.0.2", 8080, "n1"), ("10.244.0.3", 8080, "n1"), ("10.244.1.2", 8080, "n2")]}
    rules = render(svcs, eps, cluster_cidr="10.244.0.0/16")
    assert rules == render(svcs, eps, cluster_cidr="10.244.0.0/16")  # deterministic
    sc = svc_chain(web, "TCP")
    assert sc.startswith("KUBE-SVC-") and len(sc) == len("KUBE-SVC-") + 16
    lines = rules.splitlines()
    assert lines[0] == "*filter" and "*nat" in lines and lines[-1] == "COMMIT"
    assert f"-A KUBE-SERVICES -m comment --comment \"default/web:http cluster IP\" -m tcp -p tcp -d 10.0.0.10/32 --dport 80 -j {sc}" in lines
    assert any("! -s 10.244.0.0/16" in ln and "-j KUBE-MARK-MASQ" in ln for ln in lines)
    assert any("-A KUBE-NODEPORTS" in ln and "--dport 30080" in ln and sc in ln for ln in lines)
    assert any("-d 192.168.1.5/32" in ln and sc in ln for ln in lines)
    split = [ln for ln in lines if ln.startswith(f"-A {sc}") and "statistic" in ln]
    assert [ln.split("--probability ")[1].split()[0] for ln in split] == ["0.3333333333", "0.5000000000"]
    last = [ln for ln in lines if ln.startswith(f"-A {sc}") and "statistic" not in ln and "recent" not in ln]
    assert len(last) == 1 and last[0].endswith(sep_chain(web, "TCP", "10.244.1.2:8080"))
    assert sum(1 for ln in lines if ln.startswith(f"-A {sc}") and "--rcheck --seconds 600" in ln) == 3
    assert any("DNAT --to-destination 10.244.0.3:8080" in ln and "--set" in ln for ln in lines)
    # no endpoints → filter REJECT; the SVC chain is declared but empty (TestClusterIPReject)
    assert any(ln.startswith("-A KUBE-SERVICES") and "lonely has no endpoints" in ln and "-j REJECT" in ln for ln in lines)
    assert f":{svc_chain(lonely, 'UDP')} - [0:0]" in lines
    assert not any(ln.startswith(f"-A {svc_chain(lonely, 'UDP')}") for ln in lines)
    nat_commit = len(lines) - 1 - lines[::-1].index("COMMIT")
    assert lines[nat_commit - 1].endswith("-j KUBE-NODEPORTS")


def test_proxy_config_maps():
    svc = {"metadata": {"name": "web", "namespace": "ns"},
           "spec": {"clusterIP": "10.0.0.3", "type": "NodePort", "sessionAffinity": "ClientIP",
                    "ports": [{"name": "http", "port": 80, "nodePort": 30001, "protocol": "TCP"},
                              {"name": "dns", "port": 53, "protocol": "UDP"}]}}
    infos = service_infos(svc)
    assert infos[ServicePortName("ns", "web", "http")].node_port == 30001
    assert infos[ServicePortName("ns", "web", "dns")].protocol == "UDP"
    assert service_infos({"metadata": {"name": "h", "namespace": "ns"}, "spec": {"clusterIP": "None", "ports": []}}) == {}
    ep = {"metadata": {"name": "web", "namespace": "ns"},
          "subsets": [{"addresses": [{"ip": "10.1.0.2"}], "notReadyAddresses": [{"ip": "10.1.0.9"}],
                       "ports": [{"name": "http", "port": 8080}]}]}
    assert endpoints_map(ep) == {ServicePortName("ns", "web", "http"): [("10.1.0.2", 8080, "")]}


def test_round_robin_and_client_ip_affinity():
    spn = ServicePortName("ns", "s", "")
    lb = LoadBalancerRR()
    lb.new_service(spn)
    with pytest.raises(LookupError):
        lb.next_endpoint(spn, "1.1.1.1")
    lb.on_endpoints_update({spn: [("10.0.0.1", 80, ""), ("10.0.0.2", 80, ""), ("10.0.0.3", 80, "")]})
    picks = [lb.next_endpoint(spn, "1.1.1.1") for _ in range(6)]
    assert set(picks) == {"10.0.0.1:80", "10.0.0.2:80", "10.0.0.3:80"} and picks[:3] == picks[3:]
    sticky = ServicePortName("ns", "sticky", "")
    lb.new_service(sticky, "ClientIP", 60)
    lb.on_endpoints_update({spn: [("10.0.0.1", 80, "")], sticky: [("10.0.0.1", 80, ""), ("10.0.0.2", 80, "")]})
    first = lb.next_endpoint(sticky, "2.2.2.2")
    assert all(lb.next_endpoint(sticky, "2.2.2.2") == first for _ in range(5))
    other = lb.next_endpoint(sticky, "3.3.3.3")
    assert other != first
    # the affinity entry dies with its endpoint
    keep = [e for e in ("10.0.0.1:80", "10.0.0.2:80") if e != first][0]
    lb.on_endpoints_update({sticky: [(keep.split(":")[0], 80, "")]})
    assert lb.next_endpoint(sticky, "2.2.2.2") == keep


def _cni_conf(d, data_dir, subnet="usePodCidr"):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "10-amdkube.conflist"), "w") as f:
        json.dump({"cniVersion": "0.3.1", "name": "amdkube",
                   "plugins": [{"type": "amdkube-cni", "ipam": {"subnet": subnet, "dataDir": data_dir}}]}, f)


async def test_cni_network_plugin_ipam(tmp_path):
    conf = tmp_path / "net.d"
    _cni_conf(str(conf), str(tmp_path / "ipam"))
    net = CNINetwork(str(conf), [os.path.join(NATIVE_BIN, "cni")])
    ok, msg = net.status()
    assert not ok and "pod CIDR" in msg          # usePodCidr before UpdateRuntimeConfig
    with pytest.raises(NetworkError):
        await net.setup("sb0", {"name": "p", "namespace": "default"}, "")
    net.set_pod_cidr("10.244.3.0/24")
    assert net.status()[0]
    ips = [await net.setup(f"sb{i}", {"name": f"p{i}", "namespace": "default"}, "") for i in range(5)]
    assert len(set(ips)) == 5 and all(ip.startswith("10.244.3.") and ip != "10.244.3.1" for ip in ips)
    assert await net.setup("sb0", {"name": "p0", "namespace": "default"}, "") == ips[0]   # ADD is idempotent
    await net.teardown("sb1", {}, "")
    assert ips[1] not in os.listdir(tmp_path / "ipam" / "amdkube")
    bad = CNINetwork(str(tmp_path / "empty"), [os.path.join(NATIVE_BIN, "cni")])
    assert not bad.status()[0]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


async def _until(fn, timeout=20.0, every=0.05):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        v = await fn()
        if v:
            return v
        await asyncio.sleep(every)
    raise TimeoutError("condition not met")


async def test_service_routes_to_pods_through_userspace_proxy(tmp_path):
    """End to end: node IPAM → CNI pod IPs, endpoints controller, userspace kube-proxy; the
    service CIDR sits in 127/8 so the proxier binds ClusterIPs directly."""
    from amdkube.client import Client
    from amdkube.localcluster import LocalCluster, wait_pod
    conf = tmp_path / "net.d"
    _cni_conf(str(conf), str(tmp_path / "ipam"))
    net = CNINetwork(str(conf), [os.path.join(NATIVE_BIN, "cni")])
    async with LocalCluster(gpus="none", api_kw={"service_cidr": "127.0.10.0/24", "node_port_range": "31000-31999"},
                            controllers_kw={"allocate_node_cidrs": True, "cluster_cidr": "10.244.0.0/16"},
                            shim_kw={"network": net}, node_status_update_frequency=0.3, relist_period=0.3) as lc:
        c = lc.client
        node = await _until(lambda: _pod_cidr(c, lc.node_name))
        await _until(lambda: _true(net.pod_cidr == node))
        # a pod-network pod gets an address from the node's pod CIDR via CNI
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "cni-pod", "labels": {"app": "cni"}},
                        "spec": {"containers": [{"name": "c", "image": "amdkube/pause:3.1"}]}}, "default")
        p = await wait_pod(c, "default", "cni-pod", ("Running",), 20)
        assert p["status"]["podIP"].startswith(node.rsplit(".", 2)[0]) and p["status"]["hostIP"] == "127.0.0.1"
        # a host-network web server behind a NodePort service
        port = _free_port()
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web", "labels": {"app": "web"}},
                        "spec": {"hostNetwork": True, "containers": [{
                            "name": "http", "image": "python:3", "args": ["-u", "-m", "http.server", "--bind", "127.0.0.1", str(port)],
                            "ports": [{"name": "http", "containerPort": port}],
                            "readinessProbe": {"tcpSocket": {"port": port}, "periodSeconds": 1}}]}}, "default")
        svc = await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web"},
                              "spec": {"type": "NodePort", "selector": {"app": "web"},
                                       "ports": [{"name": "http", "port": 80, "targetPort": "http"}]}}, "default")
        cip, nport = svc["spec"]["clusterIP"], svc["spec"]["ports"][0]["nodePort"]
        assert cip.startswith("127.0.10.") and 31000 <= nport <= 31999
        ep = await _until(lambda: _ready_eps(c, "web"), timeout=30)
        assert ep == [("127.0.0.1", port)]
        proxy = await ProxyServer(Client(lc.api.url), "userspace", node_ip="127.0.0.1", healthz_port=0).start()
        try:
            loop = asyncio.get_running_loop()
            for url in (f"http://{cip}:80/", f"http://127.0.0.1:{nport}/"):
                body = await loop.run_in_executor(None, lambda u=url: urllib.request.urlopen(u, timeout=5).read())
                assert b"Directory listing" in body, url
            hz = await loop.run_in_executor(None, lambda: urllib.request.urlopen(
                f"http://127.0.0.1:{proxy.healthz_port}/healthz", timeout=5).status)
            assert hz == 200 and proxy.proxier.connections >= 2
            # deleting the service closes its portal and removes its endpoints
            await c.delete("services", "web", "default")
            await _until(lambda: _gone(c, "endpoints", "web"))
            await _until(lambda: _true(not proxy.proxier.sockets or all(s.name != "web" for s in proxy.proxier.sockets)))
            with pytest.raises(OSError):
                await loop.run_in_executor(None, lambda: urllib.request.urlopen(f"http://{cip}:80/", timeout=2).read())
        finally:
            await proxy.stop()
            await proxy.client.close()


async def _true(v):
    return v


async def _pod_cidr(c, node):
    n = await c.get_or_none("nodes", node)
    return ((n or {}).get("spec") or {}).get("podCIDR")


async def _ready_eps(c, name):
    ep = await c.get_or_none("endpoints", name, "default")
    out = [(a["ip"], p["port"]) for s in ((ep or {}).get("subsets") or []) for a in s.get("addresses") or []
           for p in s.get("ports") or []]
    return out or None


async def _gone(c, res, name):
    return await c.get_or_none(res, name, "default") is None


def test_ipvs_proxier_state_diff_and_restore():
    """pkg/proxy/ipvs/proxier_test.go: virtual servers per cluster/external/LB/node-port
    address, endpoints as real servers, ClientIP persistence, minimal diffs on change."""
    import asyncio
    from amdkube.proxy.config import ServiceInfo, ServicePortName
    from amdkube.proxy.ipvs import IPVSProxier, parse_save, render_iptables, render_restore

    web = ServicePortName("default", "web", "http")
    dns = ServicePortName("kube-system", "dns", "dns")
    services = {web: ServiceInfo("10.0.0.10", 80, "TCP", node_port=30080, external_ips=["192.168.1.50"]),
                dns: ServiceInfo("10.0.0.53", 53, "UDP", session_affinity="ClientIP", affinity_timeout=600)}
    eps = {web: [("10.244.0.5", 8080, "n1"), ("10.244.0.6", 8080, "n1")], dns: [("10.244.0.9", 53, "n1")]}
    px = IPVSProxier("10.244.0.0/16", node_ips=["172.16.0.2"], dry_run=True)

    async def go():
        await px.sync(services, eps)
        first = list(px.last_commands)
        assert "-A -t 10.0.0.10:80 -s rr" in first and "-A -t 172.16.0.2:30080 -s rr" in first
        assert "-A -t 192.168.1.50:80 -s rr" in first and "-A -u 10.0.0.53:53 -s rr -p 600" in first
        assert "-a -t 10.0.0.10:80 -r 10.244.0.5:8080 -m -w 1" in first
        assert px.addrs == {"10.0.0.10", "192.168.1.50", "10.0.0.53"}
        eps[web] = [("10.244.0.6", 8080, "n1"), ("10.244.0.7", 8080, "n1")]
        await px.sync(services, eps)
        assert sorted(px.last_commands) == sorted([
            "-a -t 10.0.0.10:80 -r 10.244.0.7:8080 -m -w 1", "-d -t 10.0.0.10:80 -r 10.244.0.5:8080",
            "-a -t 192.168.1.50:80 -r 10.244.0.7:8080 -m -w 1", "-d -t 192.168.1.50:80 -r 10.244.0.5:8080",
            "-a -t 172.16.0.2:30080 -r 10.244.0.7:8080 -m -w 1", "-d -t 172.16.0.2:30080 -r 10.244.0.5:8080"])
        del services[dns]
        await px.sync(services, eps)
        assert px.last_commands == ["-D -u 10.0.0.53:53"] and "10.0.0.53" not in px.addrs
        vs, rs = parse_save(render_restore(px.vs, px.rs))
        assert vs == px.vs and rs == px.rs
        assert "! -s 10.244.0.0/16" in render_iptables(services, "10.244.0.0/16")
    asyncio.run(go())
