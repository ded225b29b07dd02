"""iptables proxy mode: render the full nat/filter ruleset and apply it atomically.

Reference: pkg/proxy/iptables/proxier.go:973 syncProxyRules —
  * chains KUBE-SERVICES, KUBE-NODEPORTS, KUBE-POSTROUTING, KUBE-MARK-MASQ (+ KUBE-MARK-DROP);
  * per service port a KUBE-SVC-<hash> chain jumped to from KUBE-SERVICES on
    `-d clusterIP/32 -p proto --dport port` (plus externalIPs, LB ingress and, via
    KUBE-NODEPORTS, `--dport nodePort`), traffic from outside the cluster CIDR is marked for
    masquerade;
  * per endpoint a KUBE-SEP-<hash> chain that DNATs to ip:port; the SVC chain picks endpoint
    i of n with `-m statistic --mode random --probability 1/(n-i)` (the last one
    unconditionally); ClientIP affinity uses `-m recent --name KUBE-SEP-… --rcheck
    --seconds T --reap` ahead of the random split and `--set` in the SEP chain;
  * a service port with no endpoints gets a filter-table REJECT in KUBE-SERVICES;
  * chain names are "KUBE-SVC-"/"KUBE-SEP-" + base32(sha256(...))[:16]
    (servicePortChainName / servicePortEndpointChainName);
  * the result is fed to `iptables-restore --noflush --counters`.

amdkube renders the same ruleset deterministically (sorted service ports). `apply` runs
iptables-restore when it exists and the process may change the host's tables. Otherwise
it keeps the last ruleset in memory and, with `dump_path`, on disk (dry run: CI, the
unprivileged GPU box).
"""
from __future__ import annotations

import base64
import hashlib
import logging
import os
import shutil
import subprocess

from .config import ServiceInfo, ServicePortName

log = logging.getLogger("amdkube.proxy")

KUBE_MARK_MASQ = "KUBE-MARK-MASQ"
MASQ_MARK = "0x4000/0x4000"     # --iptables-masquerade-bit 14


def _hash(s: str) -> str:
    return base64.b32encode(hashlib.sha256(s.encode()).digest()).decode()[:16]


def svc_chain(spn: ServicePortName, proto: str) -> str:
    return "KUBE-SVC-" + _hash(str(spn) + proto.lower())


def sep_chain(spn: ServicePortName, proto: str, endpoint: str) -> str:
    return "KUBE-SEP-" + _hash(str(spn) + proto.lower() + endpoint)


def masq_mark(bit: int = 14) -> str:
    """--iptables-masquerade-bit: the fwmark bit that asks KUBE-POSTROUTING for SNAT."""
    if not 0 <= bit <= 31:
        raise ValueError("--iptables-masquerade-bit must be within [0, 31]")
    v = f"{1 << bit:#x}"
    return f"{v}/{v}"


def render(services: dict[ServicePortName, ServiceInfo], endpoints: dict[ServicePortName, list],
           cluster_cidr: str = "", node_ips: tuple = (), masquerade_all: bool = False, masq: str = MASQ_MARK) -> str:
    """masquerade_all (--masquerade-all): SNAT every packet sent to a service's cluster IP, not
    only those from outside --cluster-cidr."""
    mark = masq
    filt_chains = ["KUBE-SERVICES", "KUBE-FORWARD"]
    filt_rules: list[str] = []
    nat_chains = ["KUBE-SERVICES", "KUBE-NODEPORTS", "KUBE-POSTROUTING", KUBE_MARK_MASQ, "KUBE-MARK-DROP"]
    nat_rules = [
        f'-A KUBE-POSTROUTING -m comment --comment "kubernetes service traffic requiring SNAT" -m mark --mark {mark} -j MASQUERADE',
        f"-A {KUBE_MARK_MASQ} -j MARK --set-xmark {mark}",
        "-A KUBE-MARK-DROP -j MARK --set-xmark 0x8000/0x8000",
    ]
    filt_rules.append(f'-A KUBE-FORWARD -m comment --comment "kubernetes forwarding rules" -m mark --mark {mark} -j ACCEPT')
    for spn in sorted(services, key=str):
        info = services[spn]
        proto = info.protocol.lower()
        eps = endpoints.get(spn) or []
        comment = f'-m comment --comment "{spn} cluster IP"'
        if not eps:
            filt_rules.append(f'-A KUBE-SERVICES -m comment --comment "{spn} has no endpoints" -m {proto} -p {proto} '
                              f"-d {info.cluster_ip}/32 --dport {info.port} -j REJECT")
            if info.node_port:
                filt_rules.append(f'-A KUBE-SERVICES -m comment --comment "{spn} has no endpoints" -m addrtype --dst-type LOCAL '
                                  f"-m {proto} -p {proto} --dport {info.node_port} -j REJECT")
            continue
        sc = svc_chain(spn, info.protocol)
        nat_chains.append(sc)
        if masquerade_all:
            nat_rules.append(f"-A KUBE-SERVICES {comment} -m {proto} -p {proto} "
                             f"-d {info.cluster_ip}/32 --dport {info.port} -j {KUBE_MARK_MASQ}")
        elif cluster_cidr:
            nat_rules.append(f"-A KUBE-SERVICES ! -s {cluster_cidr} {comment} -m {proto} -p {proto} "
                             f"-d {info.cluster_ip}/32 --dport {info.port} -j {KUBE_MARK_MASQ}")
        nat_rules.append(f"-A KUBE-SERVICES {comment} -m {proto} -p {proto} -d {info.cluster_ip}/32 --dport {info.port} -j {sc}")
        for eip in info.external_ips:
            c = f'-m comment --comment "{spn} external IP"'
            nat_rules.append(f"-A KUBE-SERVICES {c} -m {proto} -p {proto} -d {eip}/32 --dport {info.port} -j {KUBE_MARK_MASQ}")
            nat_rules.append(f"-A KUBE-SERVICES {c} -m {proto} -p {proto} -d {eip}/32 --dport {info.port} -j {sc}")
        for ing in info.lb_ingress:
            c = f'-m comment --comment "{spn} loadbalancer IP"'
            nat_rules.append(f"-A KUBE-SERVICES {c} -m {proto} -p {proto} -d {ing}/32 --dport {info.port} -j {KUBE_MARK_MASQ}")
            nat_rules.append(f"-A KUBE-SERVICES {c} -m {proto} -p {proto} -d {ing}/32 --dport {info.port} -j {sc}")
        if info.node_port:
            c = f'-m comment --comment "{spn}"'
            nat_rules.append(f"-A KUBE-NODEPORTS {c} -m {proto} -p {proto} --dport {info.node_port} -j {KUBE_MARK_MASQ}")
            nat_rules.append(f"-A KUBE-NODEPORTS {c} -m {proto} -p {proto} --dport {info.node_port} -j {sc}")
        seps = [(f"{ip}:{port}", sep_chain(spn, info.protocol, f"{ip}:{port}")) for ip, port, _ in eps]
        nat_chains += [c for _, c in seps]
        if info.session_affinity == "ClientIP":
            for _, c in seps:
                nat_rules.append(f'-A {sc} -m comment --comment "{spn}" -m recent --name {c} --mask 255.255.255.255 '
                                 f"--rsource --rcheck --seconds {info.affinity_timeout} --reap -j {c}")
        n = len(seps)
        for i, (ep, c) in enumerate(seps):
            if i < n - 1:
                nat_rules.append(f'-A {sc} -m comment --comment "{spn}" -m statistic --mode random '
                                 f"--probability {1.0 / (n - i):.10f} -j {c}")
            else:
                nat_rules.append(f'-A {sc} -m comment --comment "{spn}" -j {c}')
        for ep, c in seps:
            ip = ep.rsplit(":", 1)[0]
            nat_rules.append(f'-A {c} -m comment --comment "{spn}" -s {ip}/32 -j {KUBE_MARK_MASQ}')
            aff = f"-m recent --name {c} --mask 255.255.255.255 --rsource --set " if info.session_affinity == "ClientIP" else ""
            nat_rules.append(f'-A {c} -m comment --comment "{spn}" {aff}-m {proto} -p {proto} -j DNAT --to-destination {ep}')
    nat_rules.append('-A KUBE-SERVICES -m comment --comment "kubernetes service nodeports; NOTE: this must be the last rule in '
                     'this chain" -m addrtype --dst-type LOCAL -j KUBE-NODEPORTS')
    out = ["*filter"] + [f":{c} - [0:0]" for c in filt_chains] + filt_rules + ["COMMIT", "*nat"]
    out += [f":{c} - [0:0]" for c in nat_chains] + nat_rules + ["COMMIT", ""]
    return "\n".join(out)


class IptablesProxier:
    mode = "iptables"

    def __init__(self, cluster_cidr: str = "", dry_run: bool | None = None, dump_path: str | None = None,
                 masquerade_all: bool = False, masquerade_bit: int = 14):
        self.cluster_cidr = cluster_cidr
        self.masquerade_all, self.masq = masquerade_all, masq_mark(masquerade_bit)
        self.binary = shutil.which("iptables-restore")
        self.dry_run = (self.binary is None or os.geteuid() != 0) if dry_run is None else dry_run
        self.dump_path = dump_path
        self.last_rules = ""
        self.syncs = 0

    async def sync(self, services, endpoints):
        rules = render(services, endpoints, self.cluster_cidr, masquerade_all=self.masquerade_all, masq=self.masq)
        self.syncs += 1
        if rules == self.last_rules:
            return
        self.last_rules = rules
        if self.dump_path:
            tmp = self.dump_path + ".tmp"
            with open(tmp, "w") as f:
                f.write(rules)
            os.replace(tmp, self.dump_path)
        if not self.dry_run:
            r = subprocess.run([self.binary, "--noflush", "--counters"], input=rules, text=True, capture_output=True)
            if r.returncode != 0:
                log.error("iptables-restore failed: %s", r.stderr.strip())
                raise RuntimeError(r.stderr.strip())

    async def stop(self):
        pass


def cleanup_rules(saved: str) -> str:
    """iptables-restore input that flushes and deletes every KUBE-* chain found in
    `iptables-save` output (proxier.go CleanupLeftovers), jump rules into them first."""
    out, table, chains, jumps = [], None, [], []

    def flush():
        if table is None:
            return
        out.append(f"*{table}")
        out.extend(f":{c} - [0:0]" for c in chains)
        out.extend(jumps)
        out.extend(f"-X {c}" for c in chains)
        out.append("COMMIT")
    for line in saved.splitlines():
        if line.startswith("*"):
            flush()
            table, chains, jumps = line[1:], [], []
        elif line.startswith(":KUBE-"):
            chains.append(line[1:].split()[0])
        elif line.startswith("-A ") and " -j KUBE-" in line and not line.split()[1].startswith("KUBE-"):
            jumps.append("-D" + line[2:])
    flush()
    return "\n".join(out) + "\n"


def cleanup(dry_run: bool = False) -> str:
    save, restore = shutil.which("iptables-save"), shutil.which("iptables-restore")
    if save is None or restore is None:
        return ""
    saved = subprocess.run([save], capture_output=True, text=True).stdout
    rules = cleanup_rules(saved)
    if not dry_run:
        subprocess.run([restore, "--noflush"], input=rules, text=True, capture_output=True)
    return rules
