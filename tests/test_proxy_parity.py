"""kube-proxy's iptables/ipvs rulesets against the reference's proxier tests.

Ported from pkg/proxy/iptables/proxier_test.go — TestClusterIPReject (:584),
TestClusterIPEndpointsJump (:618), TestLoadBalancer (:675), TestNodePort (:736),
TestExternalIPsReject (:786), TestNodePortReject (:820), TestOnlyLocalLoadBalancing (:857),
TestOnlyLocalNodePortsNoClusterCIDR (:947), TestOnlyLocalNodePorts (:955) — over the rendered
restore input, read back per chain the way iptablestest.FakeIPTables.GetRules does
(hasJump / hasDNAT / hasSessionAffinityRule, :447-583). There is no iptables binary here, so the
jumps from the built-in chains are checked as the list the proxier ensures.
"""
from __future__ import annotations

import shlex

import aiohttp

from amdkube.proxy.config import ServicePortName, endpoints_map, service_infos
from amdkube.proxy.iptables import (ENSURED_JUMPS, IptablesProxier, cleanup_rules, fw_chain, health_check_state,
                                    render, sep_chain, svc_chain, xlb_chain)
from tests.conftest import run

HOST = "test-hostname"          # proxier_test.go testHostname
SPN = ServicePortName("ns1", "svc1", "p80")


def rules_by_chain(text: str) -> dict[str, list[dict]]:
    """iptablestest.GetRules: every `-A CHAIN ...` line as {jump, destination, dport, todest, recent}."""
    out: dict[str, list[dict]] = {}
    for line in text.splitlines():
        if not line.startswith("-A "):
            continue
        tok = shlex.split(line)
        r = {"recent": "recent" in tok, "source": ""}
        for flag, key in (("-j", "jump"), ("-d", "destination"), ("--dport", "dport"), ("--to-destination", "todest")):
            r[key] = tok[tok.index(flag) + 1] if flag in tok else ""
        if "-s" in tok:
            r["source"] = tok[tok.index("-s") + 1]
        out.setdefault(tok[1], []).append(r)
    return out


def has_jump(rules, dest_chain, dest_ip="", dest_port=0) -> bool:
    """proxier_test.go hasJump (same semantics, including its fall-through)."""
    port = str(dest_port)
    match = False
    for r in rules:
        if r["jump"] == dest_chain:
            match = True
            if dest_ip:
                if dest_ip in r["destination"] and (port in r["dport"] or r["dport"] == ""):
                    return True
                match = False
            if dest_port:
                if port in r["dport"] and (dest_ip in r["destination"] or r["destination"] == ""):
                    return True
                match = False
    return match


def has_dnat(rules, endpoint) -> bool:
    return any(r["todest"] == endpoint for r in rules)


def svc(typ="ClusterIP", node_port=0, ingress=None, local=False, affinity=False, external_ips=None, ranges=None, hc=0):
    port = {"name": "p80", "port": 80, "protocol": "TCP"}
    if node_port:
        port["nodePort"] = node_port
    spec = {"type": typ, "clusterIP": "10.20.30.41", "ports": [port]}
    if local:
        spec["externalTrafficPolicy"] = "Local"
    if affinity:
        spec["sessionAffinity"] = "ClientIP"
        spec["sessionAffinityConfig"] = {"clientIP": {"timeoutSeconds": 10800}}
    if external_ips:
        spec["externalIPs"] = list(external_ips)
    if ranges:
        spec["loadBalancerSourceRanges"] = list(ranges)
    if hc:
        spec["healthCheckNodePort"] = hc
    obj = {"metadata": {"name": "svc1", "namespace": "ns1"}, "spec": spec}
    if ingress:
        obj["status"] = {"loadBalancer": {"ingress": [{"ip": ingress}]}}
    return service_infos(obj)


def eps(*addrs):
    """addrs: (ip, nodeName or None)."""
    ep = {"metadata": {"name": "svc1", "namespace": "ns1"},
          "subsets": [{"addresses": [{"ip": ip, **({"nodeName": n} if n else {})} for ip, n in addrs],
                       "ports": [{"name": "p80", "port": 80}]}]}
    return endpoints_map(ep)


def sync(services, endpoints, cluster_cidr="10.0.0.0/24", node_ip=""):
    return rules_by_chain(render(services, endpoints, cluster_cidr, hostname=HOST, node_ip=node_ip))


def test_cluster_ip_reject():
    r = sync(svc(), {})
    assert r.get(svc_chain(SPN, "tcp"), []) == []
    assert has_jump(r["KUBE-SERVICES"], "REJECT", "10.20.30.41", 80)


def test_cluster_ip_endpoints_jump():
    r = sync(svc(), eps(("10.180.0.1", None)))
    sc, ec = svc_chain(SPN, "tcp"), sep_chain(SPN, "tcp", "10.180.0.1:80")
    assert has_jump(r["KUBE-SERVICES"], sc, "10.20.30.41", 80)
    assert has_jump(r[sc], ec)
    assert has_dnat(r[ec], "10.180.0.1:80")


def test_load_balancer():
    r = sync(svc("LoadBalancer", 3001, ingress="1.2.3.4"), eps(("10.180.0.1", None)))
    fw, sc = fw_chain(SPN, "tcp"), svc_chain(SPN, "tcp")
    assert has_jump(r["KUBE-SERVICES"], fw, "1.2.3.4", 80)
    assert has_jump(r[fw], sc) and has_jump(r[fw], "KUBE-MARK-MASQ")


def test_node_port():
    r = sync(svc("NodePort", 3001), eps(("10.180.0.1", None)))
    assert has_jump(r["KUBE-NODEPORTS"], svc_chain(SPN, "tcp"), "", 3001)


def test_external_ips_reject():
    r = sync(svc(external_ips=["50.60.70.81"]), {})
    assert has_jump(r["KUBE-SERVICES"], "REJECT", "50.60.70.81", 80)


def test_node_port_reject():
    r = sync(svc("NodePort", 3001), {})
    assert has_jump(r["KUBE-SERVICES"], "REJECT", "10.20.30.41", 3001)


def test_only_local_load_balancing():
    r = sync(svc("LoadBalancer", 3001, ingress="1.2.3.4", local=True, affinity=True),
             eps(("10.180.0.1", None), ("10.180.2.1", HOST)))
    fw, lb = fw_chain(SPN, "tcp"), xlb_chain(SPN, "tcp")
    non_local, local = sep_chain(SPN, "tcp", "10.180.0.1:80"), sep_chain(SPN, "tcp", "10.180.2.1:80")
    assert has_jump(r["KUBE-SERVICES"], fw, "1.2.3.4", 80)
    assert has_jump(r[fw], lb)
    assert not has_jump(r[fw], "KUBE-MARK-MASQ")
    assert not has_jump(r[lb], non_local)
    assert has_jump(r[lb], local)
    assert any(x["recent"] for x in r[lb])


def _only_local_node_ports(cluster_cidr):
    r = sync(svc("NodePort", 3001, local=True), eps(("10.180.0.1", None), ("10.180.2.1", HOST)), cluster_cidr)
    lb, sc = xlb_chain(SPN, "tcp"), svc_chain(SPN, "tcp")
    assert has_jump(r["KUBE-NODEPORTS"], lb, "", 3001)
    assert not has_jump(r[lb], sep_chain(SPN, "tcp", "10.180.0.1:80"))
    assert has_jump(r[lb], sc) == bool(cluster_cidr)
    assert has_jump(r[lb], sep_chain(SPN, "tcp", "10.180.2.1:80"))


def test_only_local_node_ports_no_cluster_cidr():
    _only_local_node_ports("")


def test_only_local_node_ports():
    _only_local_node_ports("10.0.0.0/24")


def test_only_local_without_local_endpoints_drops():
    r = sync(svc("NodePort", 3001, local=True), eps(("10.180.0.1", "other-node")))
    assert has_jump(r[xlb_chain(SPN, "tcp")], "KUBE-MARK-DROP")


def test_load_balancer_source_ranges():
    """KUBE-FW: only the listed sources reach the service, then drop; when the node itself is in
    a range, the LB IP as source (hairpin) is allowed too (proxier.go:1262-1290)."""
    r = sync(svc("LoadBalancer", 3001, ingress="1.2.3.4", ranges=["192.168.0.0/16", "10.1.0.0/16"]),
             eps(("10.180.0.1", None)), node_ip="10.1.2.3")
    fw, sc = fw_chain(SPN, "tcp"), svc_chain(SPN, "tcp")
    assert [x["source"] for x in r[fw] if x["jump"] == sc] == ["192.168.0.0/16", "10.1.0.0/16", "1.2.3.4/32"]
    assert r[fw][-1]["jump"] == "KUBE-MARK-DROP"
    r2 = sync(svc("LoadBalancer", 3001, ingress="1.2.3.4", ranges=["192.168.0.0/16"]), eps(("10.180.0.1", None)),
              node_ip="10.1.2.3")
    assert [x["source"] for x in r2[fw] if x["jump"] == sc] == ["192.168.0.0/16"]


def test_jump_rules_are_ensured_and_cleaned_up():
    """proxier.go:1007-1060: the built-in chains jump into KUBE-SERVICES / KUBE-POSTROUTING /
    KUBE-FORWARD; CleanupLeftovers removes exactly those jumps."""
    p = IptablesProxier("10.0.0.0/24", dry_run=True, hostname=HOST)
    run(p.sync(svc(), eps(("10.180.0.1", None))))
    got = {(t, c, a.split()[-1]) for t, c, a in p.ensured}
    assert got == {("filter", "INPUT", "KUBE-SERVICES"), ("filter", "OUTPUT", "KUBE-SERVICES"),
                   ("nat", "OUTPUT", "KUBE-SERVICES"), ("nat", "PREROUTING", "KUBE-SERVICES"),
                   ("nat", "POSTROUTING", "KUBE-POSTROUTING"), ("filter", "FORWARD", "KUBE-FORWARD")}
    saved = ["*nat", ":PREROUTING ACCEPT [0:0]", ":OUTPUT ACCEPT [0:0]", ":POSTROUTING ACCEPT [0:0]",
             ":KUBE-SERVICES - [0:0]", ":KUBE-POSTROUTING - [0:0]"]
    saved += [f"-A {c} {a}" for t, c, a in ENSURED_JUMPS if t == "nat"] + ["COMMIT", "*filter", ":INPUT ACCEPT [0:0]",
                                                                          ":KUBE-SERVICES - [0:0]", ":KUBE-FORWARD - [0:0]"]
    saved += [f"-A {c} {a}" for t, c, a in ENSURED_JUMPS if t == "filter"] + ["COMMIT"]
    out = cleanup_rules("\n".join(saved))
    for t, c, a in ENSURED_JUMPS:
        assert f"-D {c} {a}" in out


def test_ipvs_local_policy_and_links():
    from amdkube.proxy.ipvs import IPVS_JUMPS, IPVSProxier
    p = IPVSProxier("10.0.0.0/24", node_ips=["10.1.2.3"], dry_run=True, hostname=HOST)
    run(p.sync(svc("LoadBalancer", 3001, ingress="1.2.3.4", local=True), eps(("10.180.0.1", None), ("10.180.2.1", HOST))))
    assert p.rs[("TCP", "10.20.30.41", 80)] == {("10.180.0.1", 80), ("10.180.2.1", 80)}     # cluster IP: all
    assert p.rs[("TCP", "10.1.2.3", 3001)] == {("10.180.2.1", 80)}                          # node port: local only
    assert p.rs[("TCP", "1.2.3.4", 80)] == {("10.180.2.1", 80)}
    assert p.ensured == list(IPVS_JUMPS)


def test_health_check_node_port_served_by_kube_proxy():
    """A LoadBalancer with externalTrafficPolicy=Local gets a healthCheckNodePort from the
    apiserver; kube-proxy answers it with the node's local endpoint count (healthcheck.go
    :173-185): 200 while one runs here, 503 when none does."""
    from amdkube.localcluster import LocalCluster
    from amdkube.proxy import ProxyServer

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False) as lc:
            c = lc.client
            s = await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "lb", "namespace": "default"},
                                "spec": {"type": "LoadBalancer", "externalTrafficPolicy": "Local",
                                         "ports": [{"name": "http", "port": 80}]}}, "default")   # no selector: endpoints are ours
            hc = s["spec"]["healthCheckNodePort"]
            assert 30000 <= hc <= 32767 and hc not in [p["nodePort"] for p in s["spec"]["ports"]]
            await c.create({"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "lb", "namespace": "default"},
                            "subsets": [{"addresses": [{"ip": "10.244.0.9", "nodeName": HOST}],
                                         "ports": [{"name": "http", "port": 8080}]}]}, "default")
            px = await ProxyServer(c.__class__(lc.api.url, token=lc.api.loopback_token), mode="iptables",
                                   hostname=HOST, cluster_cidr="10.244.0.0/16").start()
            try:
                async with aiohttp.ClientSession() as http:
                    async with http.get(f"http://127.0.0.1:{hc}/") as r:
                        assert r.status == 200
                        body = await r.json(content_type=None)
                        assert body == {"service": {"namespace": "default", "name": "lb"}, "localEndpoints": 1}
                    ep = await c.get("endpoints", "lb", "default")
                    # the endpoint moves off this node (a new address: validation refuses re-homing an IP)
                    ep["subsets"][0]["addresses"][0] = {"ip": "10.244.1.9", "nodeName": "elsewhere"}
                    await c.update(ep)
                    for _ in range(100):
                        await px.sync()
                        async with http.get(f"http://127.0.0.1:{hc}/") as r:
                            if r.status == 503:
                                assert (await r.json(content_type=None))["localEndpoints"] == 0
                                break
                    else:
                        raise AssertionError("health check never turned 503")
                # the service's XLB chain only balances over local endpoints (none now): drop
                rules = rules_by_chain(px.proxier.last_rules)
                spn = ServicePortName("default", "lb", "http")
                assert has_jump(rules[xlb_chain(spn, "tcp")], "KUBE-MARK-DROP")
            finally:
                await px.stop()
                await px.client.close()
            assert not px.health.services
            hs, he = health_check_state(px.tracker.service_map(), px.tracker.endpoint_map(), HOST)
            assert hs == {("default", "lb"): hc} and he == {("default", "lb"): 0}
    run(go(), 60)
