"""iptables proxy mode: render the full nat/filter ruleset and apply it atomically.

Reference: pkg/proxy/iptables/proxier.go:973 syncProxyRules —
  * the built-in chains jump into kube-proxy's (nat PREROUTING/OUTPUT and filter INPUT/OUTPUT ->
    KUBE-SERVICES, nat POSTROUTING -> KUBE-POSTROUTING, filter FORWARD -> KUBE-FORWARD), ensured
    with -C/-I outside the restore (:1007-1060);
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
  * load-balancer ingress IPs go through KUBE-FW-<hash> (loadBalancerSourceRanges, else drop);
    externalTrafficPolicy=Local sends node-port and LB traffic to KUBE-XLB-<hash>, which only
    balances over this node's endpoints (pods of the cluster CIDR still go the cluster way, no
    local endpoint drops), and kube-proxy answers the service's healthCheckNodePort
    (proxy/healthcheck.py);
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


def fw_chain(spn: ServicePortName, proto: str) -> str:
    """serviceFirewallChainName: the load-balancer IP chain (loadBalancerSourceRanges)."""
    return "KUBE-FW-" + _hash(str(spn) + proto.lower())


def xlb_chain(spn: ServicePortName, proto: str) -> str:
    """serviceLBChainName: externalTrafficPolicy=Local — only this node's endpoints."""
    return "KUBE-XLB-" + _hash(str(spn) + proto.lower())


# the jumps from the built-in chains into kube-proxy's (proxier.go:1007-1060, EnsureRule with
# Prepend): kept outside the --noflush restore, checked with -C and inserted first with -I
ENSURED_JUMPS = (
    ("filter", "INPUT", '-m comment --comment "kubernetes service portals" -j KUBE-SERVICES'),
    ("filter", "OUTPUT", '-m comment --comment "kubernetes service portals" -j KUBE-SERVICES'),
    ("nat", "OUTPUT", '-m comment --comment "kubernetes service portals" -j KUBE-SERVICES'),
    ("nat", "PREROUTING", '-m comment --comment "kubernetes service portals" -j KUBE-SERVICES'),
    ("nat", "POSTROUTING", '-m comment --comment "kubernetes postrouting rules" -j KUBE-POSTROUTING'),
    ("filter", "FORWARD", '-m comment --comment "kubernetes forward rules" -j KUBE-FORWARD'),
)


def _cidr_contains(cidr: str, ip: str) -> bool:
    import ipaddress
    try:
        return ipaddress.ip_address(ip) in ipaddress.ip_network(cidr, strict=False)
    except ValueError:
        return False


def render(services: dict[ServicePortName, ServiceInfo], endpoints: dict[ServicePortName, list],
           cluster_cidr: str = "", node_ips: tuple = (), masquerade_all: bool = False, masq: str = MASQ_MARK,
           hostname: str = "", node_ip: str = "") -> str:
    """syncProxyRules (proxier.go:1081-1640) as iptables-restore input. masquerade_all
    (--masquerade-all): SNAT every packet sent to a cluster IP, not only those from outside
    --cluster-cidr. `hostname` decides which endpoints are local (endpoint nodeName) for
    externalTrafficPolicy=Local; `node_ip` is where loadBalancerSourceRanges may also allow the
    node itself."""
    mark = masq
    filt_chains = ["KUBE-SERVICES", "KUBE-FORWARD"]
    filt_rules: list[str] = []
    nat_chains = ["KUBE-SERVICES", "KUBE-NODEPORTS", "KUBE-POSTROUTING", KUBE_MARK_MASQ, "KUBE-MARK-DROP"]
    nat_rules = [
        f'-A KUBE-POSTROUTING -m comment --comment "kubernetes service traffic requiring SNAT" -m mark --mark {mark} -j MASQUERADE',
        f"-A {KUBE_MARK_MASQ} -j MARK --set-xmark {mark}",
        "-A KUBE-MARK-DROP -j MARK --set-xmark 0x8000/0x8000",
    ]
    for spn in sorted(services, key=str):
        info = services[spn]
        proto = info.protocol.lower()
        eps = endpoints.get(spn) or []
        sc, xlb = svc_chain(spn, info.protocol), xlb_chain(spn, info.protocol)
        nat_chains.append(sc)
        if info.only_local:
            nat_chains.append(xlb)
        # cluster IP
        base = f'-A KUBE-SERVICES -m comment --comment "{spn} cluster IP" -m {proto} -p {proto} -d {info.cluster_ip}/32 --dport {info.port}'
        if masquerade_all:
            nat_rules.append(f"{base} -j {KUBE_MARK_MASQ}")
        elif cluster_cidr:
            nat_rules.append(f"{base} ! -s {cluster_cidr} -j {KUBE_MARK_MASQ}")
        nat_rules.append(f"{base} -j {sc}")
        # external IPs: traffic arriving from outside the node, or addressed to a local IP
        for eip in info.external_ips:
            b = f'-A KUBE-SERVICES -m comment --comment "{spn} external IP" -m {proto} -p {proto} -d {eip}/32 --dport {info.port}'
            nat_rules.append(f"{b} -j {KUBE_MARK_MASQ}")
            nat_rules.append(f"{b} -m physdev ! --physdev-is-in -m addrtype ! --src-type LOCAL -j {sc}")
            nat_rules.append(f"{b} -m addrtype --dst-type LOCAL -j {sc}")
            if not eps:
                filt_rules.append(f'-A KUBE-SERVICES -m comment --comment "{spn} has no endpoints" -m {proto} -p {proto} '
                                  f"-d {eip}/32 --dport {info.port} -j REJECT")
        # load-balancer ingress through the firewall chain
        fw = fw_chain(spn, info.protocol)
        for ing in info.lb_ingress:
            if fw not in nat_chains:
                nat_chains.append(fw)
            nat_rules.append(f'-A KUBE-SERVICES -m comment --comment "{spn} loadbalancer IP" -m {proto} -p {proto} '
                             f"-d {ing}/32 --dport {info.port} -j {fw}")
            fb = f'-A {fw} -m comment --comment "{spn} loadbalancer IP"'
            chosen = xlb
            if not info.only_local:
                nat_rules.append(f"{fb} -j {KUBE_MARK_MASQ}")
                chosen = sc
            if not info.source_ranges:
                nat_rules.append(f"{fb} -j {chosen}")
            else:
                allow_node = False
                for src in info.source_ranges:
                    nat_rules.append(f"{fb} -s {src} -j {chosen}")
                    allow_node = allow_node or bool(node_ip and _cidr_contains(src, node_ip))
                if allow_node:
                    # the node reaching its own LB (hairpin) arrives with the LB IP as source
                    nat_rules.append(f"{fb} -s {ing}/32 -j {chosen}")
            nat_rules.append(f"{fb} -j KUBE-MARK-DROP")
        # node ports
        if info.node_port:
            nb = f'-A KUBE-NODEPORTS -m comment --comment "{spn}" -m {proto} -p {proto} --dport {info.node_port}'
            if not info.only_local:
                nat_rules.append(f"{nb} -j {KUBE_MARK_MASQ}")
                nat_rules.append(f"{nb} -j {sc}")
            else:
                nat_rules.append(f"{nb} -j {xlb}")
            if not eps:
                filt_rules.append(f'-A KUBE-SERVICES -m comment --comment "{spn} has no endpoints" -m addrtype --dst-type LOCAL '
                                  f"-m {proto} -p {proto} --dport {info.node_port} -j REJECT")
        if not eps:
            filt_rules.append(f'-A KUBE-SERVICES -m comment --comment "{spn} has no endpoints" -m {proto} -p {proto} '
                              f"-d {info.cluster_ip}/32 --dport {info.port} -j REJECT")
            continue
        # endpoints
        seps = [(f"{ip}:{port}", sep_chain(spn, info.protocol, f"{ip}:{port}"), node) for ip, port, node in eps]
        nat_chains += [c for _, c, _ in seps]
        rec = f"--mask 255.255.255.255 --rsource"
        if info.session_affinity == "ClientIP":
            for _, c, _ in seps:
                nat_rules.append(f'-A {sc} -m comment --comment "{spn}" -m recent --name {c} {rec} --rcheck '
                                 f"--seconds {info.affinity_timeout} --reap -j {c}")
        n = len(seps)
        for i, (ep, c, _) in enumerate(seps):
            if i < n - 1:
                nat_rules.append(f'-A {sc} -m comment --comment "{spn}" -m statistic --mode random '
                                 f"--probability {1.0 / (n - i):.10f} -j {c}")
            else:
                nat_rules.append(f'-A {sc} -m comment --comment "{spn}" -j {c}')
        for ep, c, _ in seps:
            ip = ep.rsplit(":", 1)[0]
            nat_rules.append(f'-A {c} -m comment --comment "{spn}" -s {ip}/32 -j {KUBE_MARK_MASQ}')
            aff = f"-m recent --name {c} {rec} --set " if info.session_affinity == "ClientIP" else ""
            nat_rules.append(f'-A {c} -m comment --comment "{spn}" {aff}-m {proto} -p {proto} -j DNAT --to-destination {ep}')
        if not info.only_local:
            continue
        # KUBE-XLB: pods reaching the LB VIP go the cluster way; outside traffic only to local endpoints
        local = [c for _, c, node in seps if hostname and node == hostname]
        if cluster_cidr:
            nat_rules.append(f'-A {xlb} -m comment --comment "Redirect pods trying to reach external loadbalancer VIP '
                             f'to clusterIP" -s {cluster_cidr} -j {sc}')
        if not local:
            nat_rules.append(f'-A {xlb} -m comment --comment "{spn} has no local endpoints" -j KUBE-MARK-DROP')
            continue
        if info.session_affinity == "ClientIP":
            for c in local:
                nat_rules.append(f'-A {xlb} -m comment --comment "{spn}" -m recent --name {c} {rec} --rcheck '
                                 f"--seconds {info.affinity_timeout} --reap -j {c}")
        for i, c in enumerate(local):
            stat = (f" -m statistic --mode random --probability {1.0 / (len(local) - i):.10f}"
                    if i < len(local) - 1 else "")
            nat_rules.append(f'-A {xlb} -m comment --comment "Balancing rule {i} for {spn}"{stat} -j {c}')
    nat_rules.append('-A KUBE-SERVICES -m comment --comment "kubernetes service nodeports; NOTE: this must be the last rule in '
                     'this chain" -m addrtype --dst-type LOCAL -j KUBE-NODEPORTS')
    filt_rules.append(f'-A KUBE-FORWARD -m comment --comment "kubernetes forwarding rules" -m mark --mark {mark} -j ACCEPT')
    if cluster_cidr:
        filt_rules.append(f'-A KUBE-FORWARD -s {cluster_cidr} -m comment --comment "kubernetes forwarding conntrack pod '
                          'source rule" -m conntrack --ctstate RELATED,ESTABLISHED -j ACCEPT')
        filt_rules.append('-A KUBE-FORWARD -m comment --comment "kubernetes forwarding conntrack pod destination rule" '
                          f"-d {cluster_cidr} -m conntrack --ctstate RELATED,ESTABLISHED -j ACCEPT")
    out = ["*filter"] + [f":{c} - [0:0]" for c in filt_chains] + filt_rules + ["COMMIT", "*nat"]
    out += [f":{c} - [0:0]" for c in nat_chains] + nat_rules + ["COMMIT", ""]
    return "\n".join(out)


def ensure_jumps(iptables: str | None, jumps, dry_run: bool) -> list:
    """EnsureChain + EnsureRule(Prepend, table, chain, args) for every jump: `iptables -N` the
    target, `iptables -C` the rule and, when missing, `iptables -I chain 1` it. Dry (no binary,
    no privilege): nothing runs and every jump is reported as what would be in place."""
    if dry_run or iptables is None:
        return list(jumps)
    import shlex
    for table, target in {(t, shlex.split(a)[-1]) for t, _c, a in jumps}:
        subprocess.run([iptables, "-w", "-t", table, "-N", target], capture_output=True)
    done = []
    for table, chain, args in jumps:
        a = shlex.split(args)
        if subprocess.run([iptables, "-w", "-t", table, "-C", chain, *a], capture_output=True).returncode != 0:
            r = subprocess.run([iptables, "-w", "-t", table, "-I", chain, "1", *a], capture_output=True, text=True)
            if r.returncode != 0:
                log.error("ensuring %s/%s -> %s failed: %s", table, chain, a[-1], r.stderr.strip())
                continue
        done.append((table, chain, args))
    return done


def health_check_state(services: dict[ServicePortName, ServiceInfo], endpoints: dict[ServicePortName, list],
                       hostname: str) -> tuple[dict, dict]:
    """(hcServices, hcEndpoints) for the health-check server: every Local LoadBalancer service's
    healthCheckNodePort, and how many of its endpoints run on this node (proxier.go:1688-1695,
    updateServiceMap / updateEndpointsMap)."""
    hc_svcs, hc_eps = {}, {}
    for spn, info in services.items():
        if info.only_local and info.health_check_node_port:
            nsn = (spn.namespace, spn.name)
            hc_svcs[nsn] = info.health_check_node_port
            local = sum(1 for _ip, _port, node in endpoints.get(spn) or [] if hostname and node == hostname)
            hc_eps[nsn] = max(hc_eps.get(nsn, 0), local)
    return hc_svcs, hc_eps


class IptablesProxier:
    mode = "iptables"

    def __init__(self, cluster_cidr: str = "", dry_run: bool | None = None, dump_path: str | None = None,
                 masquerade_all: bool = False, masquerade_bit: int = 14, hostname: str = "", node_ip: str = ""):
        self.cluster_cidr = cluster_cidr
        self.masquerade_all, self.masq = masquerade_all, masq_mark(masquerade_bit)
        self.hostname, self.node_ip = hostname, node_ip
        self.binary = shutil.which("iptables-restore")
        self.iptables = shutil.which("iptables")
        self.dry_run = (self.binary is None or os.geteuid() != 0) if dry_run is None else dry_run
        self.dump_path = dump_path
        self.last_rules = ""
        self.ensured: list[tuple[str, str, str]] = []     # the jump rules in place (or, dry, that would be)
        self.syncs = 0

    def ensure_jumps(self):
        self.ensured = ensure_jumps(self.iptables, ENSURED_JUMPS, self.dry_run)

    async def sync(self, services, endpoints):
        self.ensure_jumps()
        rules = render(services, endpoints, self.cluster_cidr, masquerade_all=self.masquerade_all, masq=self.masq,
                       hostname=self.hostname, node_ip=self.node_ip)
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
