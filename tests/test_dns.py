"""Cluster DNS and pod resolv.conf (reference pkg/kubelet/network/dns/dns_test.go:
TestGetPodDNS / TestGetPodDNSCustom / search-limit cases; the DNS record schema the kube-dns
addon serves: service A, headless A + hostnames, SRV for named ports, pod A, PTR, NXDOMAIN)."""
import asyncio
import os

from amdkube.dns import A, CNAME, NXDOMAIN, PTR, SRV, DNSServer, resolve
from amdkube.kubelet.dns import DNSConfigurer, parse_resolv_conf
from amdkube.localcluster import LocalCluster, wait_pod


def test_pod_dns_policies(tmp_path):
    rc = tmp_path / "resolv.conf"
    rc.write_text("nameserver 10.0.0.2\nsearch corp.example\noptions timeout:2\n")
    assert parse_resolv_conf(rc.read_text()) == (["10.0.0.2"], ["corp.example"], ["timeout:2"])
    d = DNSConfigurer(["10.96.0.10"], "cluster.local", str(rc))
    pod = lambda **spec: {"metadata": {"namespace": "ml"}, "spec": spec}
    assert d.pod_dns(pod()) == {"servers": ["10.96.0.10"], "searches": ["ml.svc.cluster.local", "svc.cluster.local",
                                                                       "cluster.local", "corp.example"], "options": ["ndots:5"]}
    assert d.pod_dns(pod(hostNetwork=True))["servers"] == ["10.0.0.2"]                 # ClusterFirst + hostNetwork → Default
    assert d.pod_dns(pod(hostNetwork=True, dnsPolicy="ClusterFirstWithHostNet"))["servers"] == ["10.96.0.10"]
    assert d.pod_dns(pod(dnsPolicy="Default")) == {"servers": ["10.0.0.2"], "searches": ["corp.example"], "options": ["timeout:2"]}
    custom = d.pod_dns(pod(dnsPolicy="None", dnsConfig={"nameservers": ["1.1.1.1"], "searches": ["a.b"],
                                                         "options": [{"name": "ndots", "value": "2"}, {"name": "edns0"}]}))
    assert custom == {"servers": ["1.1.1.1"], "searches": ["a.b"], "options": ["ndots:2", "edns0"]}
    many = d.pod_dns(pod(dnsConfig={"nameservers": ["1.1.1.1", "2.2.2.2", "3.3.3.3"], "searches": [f"s{i}.x" for i in range(8)]}))
    assert len(many["servers"]) == 3 and len(many["searches"]) == 6
    assert DNSConfigurer([], "cluster.local", str(rc)).pod_dns(pod())["servers"] == ["10.0.0.2"]   # no cluster DNS: Default


async def test_cluster_dns_records_and_pod_resolv_conf(tmp_path):
    async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=True,
                            kubelet_kw={"cluster_dns": ["127.0.0.1"], "cluster_domain": "cluster.local"}) as lc:
        c = lc.client
        dns = await DNSServer(c, "cluster.local", "127.0.0.1", 0, upstream=[]).start()
        try:
            srv = ("127.0.0.1", dns.port)
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "api"},
                            "spec": {"selector": {"app": "api"}, "ports": [{"name": "http", "port": 80, "targetPort": 8080}]}},
                           "default")
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "workers"},
                            "spec": {"clusterIP": "None", "selector": {"app": "w"},
                                     "ports": [{"name": "rccl", "port": 29500}]}}, "default")
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "ext"},
                            "spec": {"type": "ExternalName", "externalName": "models.example.com"}}, "default")
            for i in range(2):
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"w{i}", "labels": {"app": "w"}},
                                "spec": {"hostname": f"w{i}", "subdomain": "workers",
                                         "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"],
                                                         "ports": [{"name": "rccl", "containerPort": 29500}]}]}}, "default")
            for i in range(2):
                await wait_pod(c, "default", f"w{i}", ("Running",), 20)
            cip = (await c.get("services", "api", "default"))["spec"]["clusterIP"]

            async def q(name, t=A, nx=False):
                for _ in range(100):   # records follow the service/endpoints watch: poll until present
                    rcode, ans = await resolve(name, t, srv)
                    if ans or (nx and rcode == NXDOMAIN):
                        return rcode, ans
                    await asyncio.sleep(0.1)
                return rcode, ans
            assert (await q("api.default.svc.cluster.local"))[1] == [("api.default.svc.cluster.local", A, cip)]
            rcode, ans = await q("_http._tcp.api.default.svc.cluster.local", SRV)
            assert ans[0][2][2:] == (80, "api.default.svc.cluster.local")
            pod_ips = {(await c.get("pods", f"w{i}", "default"))["status"]["podIP"] for i in range(2)}
            rcode, ans = await q("workers.default.svc.cluster.local")      # headless: the endpoint IPs
            assert {v for _, t, v in ans if t == A} == pod_ips
            # LocalCluster pods share the host network (one IP), so per-hostname records are
            # covered with distinct IPs in test_headless_hostnames_and_srv below
            rcode, ans = await q("w1.workers.default.svc.cluster.local")
            assert ans and ans[0][2] in pod_ips
            assert (await q("ext.default.svc.cluster.local"))[1] == [("ext.default.svc.cluster.local", CNAME, "models.example.com")]
            assert (await q("10-1-2-3.default.pod.cluster.local"))[1][0][2] == "10.1.2.3"
            rev = ".".join(reversed(cip.split("."))) + ".in-addr.arpa"
            assert (await q(rev, PTR))[1] == [(rev, PTR, "api.default.svc.cluster.local")]
            assert (await q("nope.default.svc.cluster.local", nx=True))[0] == NXDOMAIN
            # the pod's resolv.conf (rocshim writes it per sandbox and mounts it at /etc/resolv.conf)
            sbs = [s for s in lc.shim.sandboxes.values() if s.meta["name"] == "w0"]
            text = open(os.path.join(lc.shim.state_dir, "rootfs", sbs[0].id, "resolv.conf")).read()
            assert "nameserver 127.0.0.1" in text and "search default.svc.cluster.local svc.cluster.local cluster.local" in text
            assert "options ndots:5" in text
        finally:
            await dns.stop()


def test_headless_hostnames_and_srv():
    from amdkube.dns import Records
    r = Records("cluster.local")
    svc = {"metadata": {"name": "workers", "namespace": "ml"},
           "spec": {"clusterIP": "None", "ports": [{"name": "rccl", "port": 29500, "protocol": "TCP"}]}}
    ep = {"metadata": {"name": "workers", "namespace": "ml"},
          "subsets": [{"addresses": [{"ip": "10.244.1.5", "hostname": "w0"}, {"ip": "10.244.2.7", "hostname": "w1"},
                                     {"ip": "10.244.3.9"}],
                       "ports": [{"name": "rccl", "port": 29500, "protocol": "TCP"}]}]}
    r.rebuild([svc], [ep])
    rcode, ans = r.lookup("workers.ml.svc.cluster.local", A)
    assert rcode == 0 and len(ans) == 3
    assert r.lookup("w1.workers.ml.svc.cluster.local", A)[1][0][2] == bytes([10, 244, 2, 7])
    rcode, ans = r.lookup("_rccl._tcp.workers.ml.svc.cluster.local", SRV)
    targets = sorted(a[2][6:] for a in ans)
    from amdkube.dns import encode_name
    assert targets == sorted(encode_name(n) for n in ("w0.workers.ml.svc.cluster.local", "w1.workers.ml.svc.cluster.local",
                                                       "10-244-3-9.workers.ml.svc.cluster.local"))
    assert r.lookup("10-244-3-9.workers.ml.svc.cluster.local", A)[1]
    assert r.lookup("9.3.244.10.in-addr.arpa", PTR)[0] == NXDOMAIN          # no hostname: no PTR
    assert r.lookup("5.1.244.10.in-addr.arpa", PTR)[1]
    assert r.lookup("svc.cluster.local", A) == (0, [])                       # empty non-terminal: NODATA


def test_corefile_parse_and_kubeadm_coredns_addon(tmp_path):
    """The CoreDNS feature gate (kubeadm addons/dns coreDNSAddon): the Corefile kubeadm writes
    parses to the cluster domain, port and resolv.conf upstreams; the addon objects."""
    from amdkube.dns.corefile import CorefileError, parse
    from amdkube.kubeadm import phases as ph
    rc = tmp_path / "resolv.conf"
    rc.write_text("nameserver 10.0.0.2\nnameserver 10.0.0.3\n")
    text = ph.COREFILE.format(domain="corp.local", cidr="10.96.0.0/12").replace("/etc/resolv.conf", str(rc))
    cf = parse(text)
    assert (cf["domain"], cf["port"], cf["upstream"], cf["cache"]) == ("corp.local", 53, ["10.0.0.2", "10.0.0.3"], 30)
    assert cf["plugins"] == ["errors", "log", "health", "kubernetes", "prometheus", "proxy", "cache"]
    assert parse(".:1053 {\n kubernetes a.b\n forward . dns://9.9.9.9\n}\n")["upstream"] == ["9.9.9.9"]
    for bad in (".:53 {\n errors\n}\n", ".:53 {\n kubernetes x\n", "nothing"):
        try:
            parse(bad)
            raise AssertionError(bad)
        except CorefileError:
            pass
    mc = {"networking": {"dnsDomain": "corp.local", "serviceSubnet": "10.96.0.0/12"}, "kubernetesVersion": "v1.9.0",
          "featureGates": {"CoreDNS": True}}
    objs = {(o["kind"], o["metadata"]["name"]): o for o in ph.addon_objects(mc, {"base": "/k"}, "kube-dns")}
    assert set(objs) == {("ConfigMap", "coredns"), ("ServiceAccount", "coredns"), ("ClusterRole", "system:coredns"),
                         ("ClusterRoleBinding", "system:coredns"), ("Deployment", "coredns"), ("Service", "kube-dns")}
    assert "kubernetes corp.local 10.96.0.0/12" in objs[("ConfigMap", "coredns")]["data"]["Corefile"]
    tpl = objs[("Deployment", "coredns")]["spec"]["template"]
    assert tpl["metadata"]["labels"] == objs[("Service", "kube-dns")]["spec"]["selector"] == {"k8s-app": "kube-dns"}
    args = tpl["spec"]["containers"][0]["args"]
    assert args[args.index("-conf") + 1] == "/etc/coredns/Corefile"
    assert objs[("Service", "kube-dns")]["spec"]["clusterIP"] == "10.96.0.10"
    mc["featureGates"] = {}
    assert [o["metadata"]["name"] for o in ph.addon_objects(mc, {"base": "/k"}, "kube-dns")] == ["kube-dns", "kube-dns"]


async def test_dns_component_serves_from_a_corefile_in_the_container_view(tmp_path):
    """`amdkube dns -conf /etc/coredns/Corefile` as the CoreDNS addon pod runs it: the ConfigMap
    volume sits under $AMDKUBE_ROOTFS, the zone comes from the Corefile."""
    import socket
    import subprocess
    import sys
    from amdkube.apiserver import APIServer
    from amdkube.kubeadm import phases as ph
    root = tmp_path / "root"
    (root / "etc" / "coredns").mkdir(parents=True)
    (root / "etc" / "coredns" / "Corefile").write_text(
        ph.COREFILE.format(domain="corp.local", cidr="10.96.0.0/12").replace("proxy . /etc/resolv.conf", ""))
    # the server binds UDP and TCP on the same port: pick one free for both
    for _ in range(50):
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            try:
                with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as t:
                    t.bind(("127.0.0.1", port))
                break
            except OSError:
                continue
    srv = await APIServer().start()
    proc = None
    try:
        from amdkube.client import Client
        c = Client(srv.url, token=srv.loopback_token)
        await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "api"},
                        "spec": {"ports": [{"port": 80}]}}, "default")
        cip = (await c.get("services", "api", "default"))["spec"]["clusterIP"]
        env = dict(os.environ, AMDKUBE_ROOTFS=str(root))
        proc = subprocess.Popen([sys.executable, "-m", "amdkube", "dns", "-conf", "/etc/coredns/Corefile", "--master", srv.url,
                                 "--token", srv.loopback_token, "--dns-bind-address", "127.0.0.1", "--dns-port", str(port)],
                                env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        for _ in range(200):
            try:
                _, ans = await resolve("api.default.svc.corp.local", A, ("127.0.0.1", port))
            except (OSError, asyncio.TimeoutError):
                ans = []
            if ans:
                break
            assert proc.poll() is None, proc.stderr.read().decode()[-2000:]
            await asyncio.sleep(0.1)
        assert cip in str(ans), ans
        await c.close()
    finally:
        if proc is not None:
            proc.terminate()
            proc.wait(10)
        await srv.stop()
