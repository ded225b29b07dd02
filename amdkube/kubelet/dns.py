"""Pod DNS configuration (the resolv.conf a pod's containers see).

Reference: pkg/kubelet/network/dns/dns.go — GetPodDNS (:325): dnsPolicy ClusterFirst (default;
host-network pods fall back to Default), ClusterFirstWithHostNet, Default (the node's
--resolv-conf), None (only spec.dnsConfig, CustomPodDNS); cluster pods get the --cluster-dns
servers, search `<ns>.svc.<domain> svc.<domain> <domain>` + the host's searches and
`options ndots:5`; spec.dnsConfig is appended (appendDNSConfig :317, option merge :286); the
result is clipped to validation limits (3 nameservers, 6 search paths, 256 chars).
"""
from __future__ import annotations

import os

from ..grpcdesc.cri import CRI as C

MAX_NAMESERVERS, MAX_SEARCH_PATHS, MAX_SEARCH_CHARS = 3, 6, 256
DEFAULT_OPTIONS = ["ndots:5"]


def parse_resolv_conf(text: str) -> tuple[list[str], list[str], list[str]]:
    servers, searches, options = [], [], []
    for line in text.splitlines():
        line = line.split("#", 1)[0].split(";", 1)[0].strip()
        if not line:
            continue
        f = line.split()
        if f[0] == "nameserver" and len(f) > 1:
            servers.append(f[1])
        elif f[0] in ("search", "domain"):
            searches = f[1:]          # the last search/domain line wins
        elif f[0] == "options":
            options = f[1:]
    return servers, searches, options


def _dedup(xs):
    out = []
    for x in xs:
        if x not in out:
            out.append(x)
    return out


def _merge_options(existing, extra) -> list[str]:
    opts = {}
    for o in existing:
        k, _, v = o.partition(":")
        opts[k] = v
    for o in extra or []:
        opts[o["name"]] = o.get("value") or ""
    return [f"{k}:{v}" if v else k for k, v in opts.items()]


class DNSConfigurer:
    def __init__(self, cluster_dns: list[str] | None = None, cluster_domain: str = "", resolv_conf: str = "/etc/resolv.conf",
                 node_ip: str = "127.0.0.1", recorder=None):
        self.cluster_dns = [x for x in (cluster_dns or []) if x]
        self.cluster_domain = cluster_domain
        self.resolv_conf = resolv_conf
        self.node_ip = node_ip
        self.recorder = recorder

    _cache: tuple | None = None     # ((mtime_ns, size), parsed) of --resolv-conf

    def _host(self):
        if not self.resolv_conf:
            return [], [], []
        try:
            st = os.stat(self.resolv_conf)
            key = (st.st_mtime_ns, st.st_size, st.st_ino)
            if self._cache is not None and self._cache[0] == key:
                return tuple(list(x) for x in self._cache[1])
            with open(self.resolv_conf) as f:
                parsed = parse_resolv_conf(f.read())
            self._cache = (key, parsed)
            return tuple(list(x) for x in parsed)
        except OSError:
            return [], [], []

    def pod_dns(self, pod: dict) -> dict:
        """{"servers", "searches", "options"} for the pod's sandbox."""
        spec = pod.get("spec") or {}
        policy = spec.get("dnsPolicy") or "ClusterFirst"
        servers, searches, options = self._host()
        if policy == "None":
            kind = "none"
        elif policy == "ClusterFirstWithHostNet":
            kind = "cluster"
        elif policy == "ClusterFirst":
            kind = "host" if spec.get("hostNetwork") else "cluster"
        else:
            kind = "host"
        if kind == "none":
            servers, searches, options = [], [], []
        elif kind == "cluster" and self.cluster_dns:
            ns = (pod.get("metadata") or {}).get("namespace") or "default"
            servers = list(self.cluster_dns)
            if self.cluster_domain:
                d = self.cluster_domain
                searches = _dedup([f"{ns}.svc.{d}", f"svc.{d}", d] + searches)
            options = list(DEFAULT_OPTIONS)
        elif kind == "cluster":
            if self.recorder is not None:
                self.recorder.event(pod, "Warning", "MissingClusterDNS",
                                    "kubelet does not have ClusterDNS IP configured and cannot create Pod using "
                                    '"ClusterFirst" policy. Falling back to "Default" policy.')
            kind = "host"
        if kind == "host" and not self.resolv_conf:
            servers, searches = ["127.0.0.1"], ["."]
        extra = spec.get("dnsConfig")
        if extra:
            servers = _dedup(servers + list(extra.get("nameservers") or []))
            searches = _dedup(searches + list(extra.get("searches") or []))
            options = _merge_options(options, extra.get("options"))
        servers = servers[:MAX_NAMESERVERS]
        searches = searches[:MAX_SEARCH_PATHS]
        while searches and len(" ".join(searches)) > MAX_SEARCH_CHARS:
            searches = searches[:-1]
        return {"servers": servers, "searches": searches, "options": options}

    def cri_config(self, pod: dict) -> "C.DNSConfig":
        d = self.pod_dns(pod)
        return C.DNSConfig(servers=d["servers"], searches=d["searches"], options=d["options"])
