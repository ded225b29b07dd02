"""kube-proxy options (cmd/kube-proxy/app/server.go, conntrack.go; proxy/iptables/proxier.go
masqueradeAll / masqueradeBit / CleanupLeftovers)."""
import argparse
import os
import subprocess
import sys

import yaml

from amdkube.proxy import config_file
from amdkube.proxy.config import ServiceInfo, ServicePortName
from amdkube.proxy.iptables import cleanup_rules, masq_mark, render

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_masquerade_all_and_bit():
    spn = ServicePortName("default", "web", "http")
    svc = {spn: ServiceInfo("10.96.0.20", 80, "TCP")}
    eps = {spn: [("10.244.1.5", 8080, True)]}
    plain = render(svc, eps, "10.244.0.0/16")
    assert "! -s 10.244.0.0/16" in plain and "0x4000/0x4000" in plain
    allm = render(svc, eps, "10.244.0.0/16", masquerade_all=True, masq=masq_mark(10))
    assert "! -s 10.244.0.0/16" not in allm and "-d 10.96.0.20/32 --dport 80 -j KUBE-MARK-MASQ" in allm
    assert "0x400/0x400" in allm and "0x4000/0x4000" not in allm


def test_cleanup_rules_from_iptables_save():
    saved = "\n".join(["*nat", ":PREROUTING ACCEPT [0:0]", ":KUBE-SERVICES - [0:0]", ":KUBE-SVC-ABC - [0:0]",
                       '-A PREROUTING -m comment --comment "kubernetes service portals" -j KUBE-SERVICES',
                       "-A KUBE-SERVICES -d 10.96.0.1/32 -j KUBE-SVC-ABC", "COMMIT",
                       "*filter", ":INPUT ACCEPT [0:0]", ":KUBE-FORWARD - [0:0]", "-A FORWARD -j KUBE-FORWARD", "COMMIT"])
    out = cleanup_rules(saved)
    assert '-D PREROUTING -m comment --comment "kubernetes service portals" -j KUBE-SERVICES' in out
    assert "-X KUBE-SERVICES" in out and "-X KUBE-SVC-ABC" in out and "-X KUBE-FORWARD" in out and "-D FORWARD -j KUBE-FORWARD" in out
    assert "-X PREROUTING" not in out and out.count("COMMIT") == 2


def test_config_file_and_conntrack(tmp_path):
    cfg = tmp_path / "kp.yaml"
    cfg.write_text(yaml.safe_dump({"apiVersion": "kubeproxy.config.k8s.io/v1alpha1", "kind": "KubeProxyConfiguration",
                                   "mode": "iptables", "clusterCIDR": "10.244.0.0/16", "healthzBindAddress": "0.0.0.0:10266",
                                   "iptables": {"masqueradeAll": True, "masqueradeBit": 12, "syncPeriod": "10s"},
                                   "conntrack": {"maxPerCore": 1000, "min": 5000, "tcpEstablishedTimeout": "2h0m0s"}}))
    out = tmp_path / "effective.yaml"
    r = subprocess.run([sys.executable, "-m", "amdkube", "proxy", "--config", str(cfg), "--write-config-to", str(out)],
                       cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    eff = yaml.safe_load(out.read_text())
    assert eff["mode"] == "iptables" and eff["clusterCIDR"] == "10.244.0.0/16" and eff["healthzBindAddress"] == "0.0.0.0:10266"
    assert eff["iptables"] == {"masqueradeAll": True, "masqueradeBit": 12, "syncPeriod": "0h0m10s", "minSyncPeriod": "0ms"}
    assert eff["conntrack"]["tcpEstablishedTimeout"] == "2h0m0s"
    # conntrack: max(maxPerCore × cores, min), written where the kernel would take it
    a = argparse.Namespace(conntrack_max=0, conntrack_max_per_core=1000, conntrack_min=5000,
                           conntrack_tcp_timeout_established=7200, conntrack_tcp_timeout_close_wait=3600)
    assert config_file.conntrack_max(a, cores=2) == 5000 and config_file.conntrack_max(a, cores=16) == 16000
    root = tmp_path / "nf"
    root.mkdir()
    for k in ("nf_conntrack_max", "nf_conntrack_tcp_timeout_established", "nf_conntrack_tcp_timeout_close_wait"):
        (root / k).write_text("1\n")
    want = config_file.apply_conntrack(a, str(root))
    assert (root / "nf_conntrack_tcp_timeout_established").read_text() == "7200"
    assert int((root / "nf_conntrack_max").read_text()) == want["nf_conntrack_max"]
