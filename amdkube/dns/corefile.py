"""The part of CoreDNS's Corefile that the kubeadm CoreDNS addon writes, read by `amdkube dns
-conf <Corefile>` (reference: cmd/kubeadm/app/phases/addons/dns/manifests.go CoreDNSConfigMap;
the `kubernetes`, `proxy`/`forward`, `cache`, `prometheus`, `health` and `errors` plugins).

    .:53 {
        errors
        health
        kubernetes cluster.local 10.96.0.0/12 {
           pods insecure
           upstream /etc/resolv.conf
        }
        prometheus :9153
        proxy . /etc/resolv.conf
        cache 30
    }

Only the first server block is served. `kubernetes <zone> [reverse zones...]` gives the cluster
domain, `proxy|forward . <to...>` the upstream servers (a path reads that resolv.conf), `.:<port>`
the port. Other plugins are recorded under `plugins` and otherwise not acted on.
"""
from __future__ import annotations

import os
import re


class CorefileError(ValueError):
    pass


def _tokens(text: str):
    for line in text.splitlines():
        line = line.split("#", 1)[0]
        for tok in re.findall(r"[{}]|[^\s{}]+", line):
            yield tok
        yield "\n"


def _blocks(toks: list[str], i: int) -> tuple[list[list], int]:
    """Parse `plugin args... [{ nested }]` lines until the closing brace."""
    out, cur = [], []
    while i < len(toks):
        t = toks[i]
        if t == "}":
            if cur:
                out.append(cur)
            return out, i + 1
        if t == "{":
            nested, i = _blocks(toks, i + 1)
            cur.append(nested)
            continue
        if t == "\n":
            if cur:
                out.append(cur)
            cur = []
        else:
            cur.append(t)
        i += 1
    raise CorefileError("unbalanced braces in the Corefile")


def parse(text: str) -> dict:
    toks = list(_tokens(text))
    i, keys = 0, []
    while i < len(toks) and toks[i] != "{":
        if toks[i] != "\n":
            keys.append(toks[i])
        i += 1
    if not keys or i == len(toks):
        raise CorefileError("the Corefile has no server block")
    plugins, _ = _blocks(toks, i + 1)
    zone, _, port = keys[0].rpartition(":")
    conf = {"zone": zone or keys[0], "port": int(port) if port.isdigit() else 53, "domain": None,
            "upstream": None, "cache": None, "plugins": [p[0] for p in plugins]}
    for p in plugins:
        name, args = p[0], [a for a in p[1:] if isinstance(a, str)]
        if name == "kubernetes" and args:
            conf["domain"] = args[0].rstrip(".")
        elif name in ("proxy", "forward") and len(args) >= 2:
            up = []
            for to in args[1:]:
                if to.startswith("/"):
                    from ..kubelet.dns import parse_resolv_conf
                    if os.path.exists(to):
                        up += parse_resolv_conf(open(to).read())[0]
                else:
                    up.append(to.split("://", 1)[-1])
            conf["upstream"] = up
        elif name == "cache":
            conf["cache"] = int(args[0]) if args else 3600
    if conf["domain"] is None:
        raise CorefileError("the Corefile's server block has no kubernetes plugin")
    return conf
