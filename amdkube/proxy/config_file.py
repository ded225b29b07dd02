"""KubeProxyConfiguration (pkg/proxy/apis/kubeproxyconfig/v1alpha1; cmd/kube-proxy/app/server.go
--config / --write-config-to) and the conntrack settings kube-proxy applies at start
(cmd/kube-proxy/app/conntrack.go: nf_conntrack_max from max(maxPerCore × cores, min) and the TCP
established / close-wait timeouts)."""
from __future__ import annotations

import logging
import os
import re

import yaml

log = logging.getLogger("amdkube.proxy")

API_VERSION = "kubeproxy.config.k8s.io/v1alpha1"


def _secs(v) -> float:
    """A Go duration ("30s", "1h0m0s", "500ms") or a number of seconds."""
    if isinstance(v, (int, float)):
        return float(v)
    tot = 0.0
    for n, u in re.findall(r"([\d.]+)(ms|h|m|s)", str(v)):
        tot += float(n) * {"h": 3600, "m": 60, "s": 1, "ms": 0.001}[u]
    return tot


def _dur(sec: float) -> str:
    sec = float(sec)
    if sec < 1:
        return f"{int(sec * 1000)}ms"
    h, rem = divmod(int(sec), 3600)
    mi, s = divmod(rem, 60)
    return f"{h}h{mi}m{s}s"


def load(path: str) -> dict:
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    if cfg.get("kind") not in (None, "KubeProxyConfiguration"):
        raise SystemExit(f"error: {path}: expected kind KubeProxyConfiguration, got {cfg.get('kind')}")
    return cfg


def apply(a, cfg: dict):
    """The file's fields over the parsed flags (the reference makes --config exclusive)."""
    cc = cfg.get("clientConnection") or {}
    a.kubeconfig = cc.get("kubeconfig") or a.kubeconfig
    a.kube_api_qps = float(cc.get("qps", a.kube_api_qps))
    a.kube_api_burst = int(cc.get("burst", a.kube_api_burst))
    a.bind_address = cfg.get("bindAddress", a.bind_address)
    a.cluster_cidr = cfg.get("clusterCIDR", a.cluster_cidr)
    if cfg.get("mode"):
        a.proxy_mode = cfg["mode"]
    if cfg.get("healthzBindAddress"):
        host, _, port = cfg["healthzBindAddress"].rpartition(":")
        a.healthz_bind_address, a.healthz_port = host or a.healthz_bind_address, int(port)
    a.metrics_bind_address = cfg.get("metricsBindAddress", a.metrics_bind_address)
    a.hostname_override = cfg.get("hostnameOverride", a.hostname_override)
    if cfg.get("oomScoreAdj") is not None:
        a.oom_score_adj = int(cfg["oomScoreAdj"])
    if cfg.get("udpIdleTimeout"):
        a.udp_timeout = _secs(cfg["udpIdleTimeout"])
    ipt = cfg.get("iptables") or {}
    a.masquerade_all = bool(ipt.get("masqueradeAll", a.masquerade_all))
    if ipt.get("masqueradeBit") is not None:
        a.iptables_masquerade_bit = int(ipt["masqueradeBit"])
    if ipt.get("syncPeriod"):
        a.iptables_sync_period = _secs(ipt["syncPeriod"])
    if ipt.get("minSyncPeriod"):
        a.iptables_min_sync_period = _secs(ipt["minSyncPeriod"])
    ipvs = cfg.get("ipvs") or {}
    if ipvs.get("syncPeriod"):
        a.ipvs_sync_period = _secs(ipvs["syncPeriod"])
    if ipvs.get("minSyncPeriod"):
        a.ipvs_min_sync_period = _secs(ipvs["minSyncPeriod"])
    a.ipvs_scheduler = ipvs.get("scheduler") or a.ipvs_scheduler
    ct = cfg.get("conntrack") or {}
    if ct.get("max") is not None:
        a.conntrack_max = int(ct["max"])
    if ct.get("maxPerCore") is not None:
        a.conntrack_max_per_core = int(ct["maxPerCore"])
    if ct.get("min") is not None:
        a.conntrack_min = int(ct["min"])
    if ct.get("tcpEstablishedTimeout"):
        a.conntrack_tcp_timeout_established = _secs(ct["tcpEstablishedTimeout"])
    if ct.get("tcpCloseWaitTimeout"):
        a.conntrack_tcp_timeout_close_wait = _secs(ct["tcpCloseWaitTimeout"])


def effective(a) -> dict:
    return {"apiVersion": API_VERSION, "kind": "KubeProxyConfiguration",
            "bindAddress": a.bind_address, "clusterCIDR": a.cluster_cidr, "mode": a.proxy_mode,
            "healthzBindAddress": f"{a.healthz_bind_address}:{a.healthz_port}", "metricsBindAddress": a.metrics_bind_address,
            "hostnameOverride": a.hostname_override, "oomScoreAdj": a.oom_score_adj, "udpIdleTimeout": _dur(a.udp_timeout),
            "clientConnection": {"kubeconfig": a.kubeconfig or "", "qps": a.kube_api_qps, "burst": a.kube_api_burst},
            "iptables": {"masqueradeAll": a.masquerade_all, "masqueradeBit": a.iptables_masquerade_bit,
                         "syncPeriod": _dur(a.iptables_sync_period), "minSyncPeriod": _dur(a.iptables_min_sync_period)},
            "ipvs": {"syncPeriod": _dur(a.ipvs_sync_period), "minSyncPeriod": _dur(a.ipvs_min_sync_period),
                     "scheduler": a.ipvs_scheduler},
            "conntrack": {"max": a.conntrack_max, "maxPerCore": a.conntrack_max_per_core, "min": a.conntrack_min,
                          "tcpEstablishedTimeout": _dur(a.conntrack_tcp_timeout_established),
                          "tcpCloseWaitTimeout": _dur(a.conntrack_tcp_timeout_close_wait)}}


def write(a, path: str):
    with open(path, "w") as f:
        yaml.safe_dump(effective(a), f, sort_keys=False)


def conntrack_max(a, cores: int | None = None) -> int:
    if a.conntrack_max:
        return a.conntrack_max
    cores = cores or os.cpu_count() or 1
    return max(a.conntrack_max_per_core * cores, a.conntrack_min) if a.conntrack_max_per_core else 0


def apply_conntrack(a, root: str = "/proc/sys/net/netfilter") -> dict:
    """Writes what it may; returns {setting: value} of what it attempted."""
    want = {}
    mx = conntrack_max(a)
    if mx:
        want["nf_conntrack_max"] = mx
    if a.conntrack_tcp_timeout_established:
        want["nf_conntrack_tcp_timeout_established"] = int(a.conntrack_tcp_timeout_established)
    if a.conntrack_tcp_timeout_close_wait:
        want["nf_conntrack_tcp_timeout_close_wait"] = int(a.conntrack_tcp_timeout_close_wait)
    for k, v in want.items():
        path = os.path.join(root, k)
        try:
            with open(path) as f:
                if int(f.read().strip()) >= v and k == "nf_conntrack_max":
                    continue
            with open(path, "w") as f:
                f.write(str(v))
        except (OSError, ValueError) as e:
            log.info("conntrack %s=%s not applied: %s", k, v, e)
    return want
