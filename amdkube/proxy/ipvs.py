"""ipvs proxy mode (pkg/proxy/ipvs/proxier.go:929 syncProxyRules, SupportIPVSProxyMode gate).

Per service port one IPVS virtual server for every address it is reachable on — the cluster
IP, each external IP, each load-balancer ingress IP and, for NodePorts, every node IP — with
the --ipvs-scheduler (rr by default) and, for ClientIP affinity, persistence for the affinity
timeout; the ready endpoints are its real servers (masquerading forward, weight 1). Every
cluster/external/LB address is bound to the dummy interface kube-ipvs0 so the node accepts the
traffic. iptables only supplies the masquerade marks (KUBE-POSTROUTING, KUBE-MARK-MASQ for
traffic from outside --cluster-cidr or with --masquerade-all), linked from nat PREROUTING/OUTPUT
(-> KUBE-SERVICES) and POSTROUTING (-> KUBE-POSTROUTING) like the reference's
linkKubeServiceChain (proxier.go:1676-1700).

externalTrafficPolicy=Local: the virtual servers of the node ports, external IPs and load-balancer
IPs get only this node's endpoints (syncEndpoint onlyNodeLocalEndpoints, :1565-1590); unlike
the v1.9 reference, the cluster IP keeps every endpoint (traffic inside the cluster is not
subject to the external traffic policy).

The proxier computes the desired state, diffs it with what it applied last (or with
`ipvsadm -Sn` when it owns the host) and emits the minimal ipvsadm-restore / ip-addr / iptables
changes; without root or the tools it runs dry (state kept for inspection, --ipvs-dump-file).
"""
from __future__ import annotations

import logging
import os
import shutil
import subprocess

from .config import ServiceInfo, ServicePortName
from .iptables import KUBE_MARK_MASQ, MASQ_MARK, ensure_jumps

IPVS_JUMPS = (
    ("nat", "OUTPUT", '-m comment --comment "kubernetes service portals" -j KUBE-SERVICES'),
    ("nat", "PREROUTING", '-m comment --comment "kubernetes service portals" -j KUBE-SERVICES'),
    ("nat", "POSTROUTING", '-m comment --comment "kubernetes postrouting rules" -j KUBE-POSTROUTING'),
)

log = logging.getLogger("amdkube.proxy.ipvs")
DUMMY = "kube-ipvs0"
SCHEDULERS = ("rr", "wrr", "lc", "wlc", "lblc", "lblcr", "dh", "sh", "sed", "nq")


def _flag(proto: str) -> str:
    return {"TCP": "-t", "UDP": "-u", "SCTP": "--sctp-service"}.get(proto.upper(), "-t")


def desired(services: dict[ServicePortName, ServiceInfo], endpoints: dict[ServicePortName, list], node_ips=(),
            scheduler: str = "rr", hostname: str = ""):
    """(virtual servers {(proto, vip, port): {scheduler, persistent}}, real servers
    {(proto, vip, port): {(ip, port)}}, addresses bound to kube-ipvs0)."""
    vs, rs, addrs = {}, {}, set()
    for spn, info in sorted(services.items(), key=lambda kv: str(kv[0])):
        eps = {(ip, port) for ip, port, _node in endpoints.get(spn, [])}
        local = {(ip, port) for ip, port, node in endpoints.get(spn, []) if hostname and node == hostname}
        persist = info.affinity_timeout if info.session_affinity == "ClientIP" else 0
        vips = [info.cluster_ip] + list(info.external_ips) + list(info.lb_ingress)
        addrs.update(v for v in vips if v)
        targets = [(v, info.port, v != info.cluster_ip) for v in vips if v]
        if info.node_port:
            targets += [(nip, info.node_port, True) for nip in node_ips]
        for vip, port, external in targets:
            key = (info.protocol.upper(), vip, port)
            vs[key] = {"scheduler": scheduler, "persistent": persist}
            rs[key] = set(local if (external and info.only_local) else eps)
    return vs, rs, addrs


def render_restore(vs, rs) -> str:
    """The full state in `ipvsadm-restore` syntax."""
    out = []
    for (proto, vip, port), v in sorted(vs.items()):
        line = f"-A {_flag(proto)} {vip}:{port} -s {v['scheduler']}"
        if v["persistent"]:
            line += f" -p {v['persistent']}"
        out.append(line)
        for ip, rport in sorted(rs.get((proto, vip, port), ())):
            out.append(f"-a {_flag(proto)} {vip}:{port} -r {ip}:{rport} -m -w 1")
    return "\n".join(out) + ("\n" if out else "")


def diff(old_vs, old_rs, vs, rs) -> list[str]:
    """ipvsadm commands turning (old_vs, old_rs) into (vs, rs): edits, adds, then deletes."""
    cmds = []
    for key, v in sorted(vs.items()):
        proto, vip, port = key
        svc = f"{_flag(proto)} {vip}:{port}"
        opt = f"-s {v['scheduler']}" + (f" -p {v['persistent']}" if v["persistent"] else "")
        if key not in old_vs:
            cmds.append(f"-A {svc} {opt}")
        elif old_vs[key] != v:
            cmds.append(f"-E {svc} {opt}")
        have = old_rs.get(key, set()) if key in old_vs else set()
        for ip, rport in sorted(rs.get(key, set()) - have):
            cmds.append(f"-a {svc} -r {ip}:{rport} -m -w 1")
        for ip, rport in sorted(have - rs.get(key, set())):
            cmds.append(f"-d {svc} -r {ip}:{rport}")
    for key in sorted(set(old_vs) - set(vs)):
        proto, vip, port = key
        cmds.append(f"-D {_flag(proto)} {vip}:{port}")
    return cmds


def render_iptables(services, cluster_cidr: str = "", masquerade_all: bool = False, masq: str = MASQ_MARK) -> str:
    rules = ["*nat", ":KUBE-SERVICES - [0:0]", ":KUBE-POSTROUTING - [0:0]", f":{KUBE_MARK_MASQ} - [0:0]",
             f'-A KUBE-POSTROUTING -m comment --comment "kubernetes service traffic requiring SNAT" -m mark --mark {masq} -j MASQUERADE',
             f"-A {KUBE_MARK_MASQ} -j MARK --set-xmark {masq}"]
    for spn, info in sorted(services.items(), key=lambda kv: str(kv[0])):
        base = f'-A KUBE-SERVICES -m comment --comment "{spn} cluster IP" -p {info.protocol.lower()} -d {info.cluster_ip}/32 --dport {info.port}'
        if masquerade_all:
            rules.append(f"{base} -j {KUBE_MARK_MASQ}")
        elif cluster_cidr:
            rules.append(base.replace(" -p ", f" ! -s {cluster_cidr} -p ", 1) + f" -j {KUBE_MARK_MASQ}")
    rules.append("COMMIT")
    return "\n".join(rules) + "\n"


def parse_save(text: str):
    """`ipvsadm -Sn` output → (vs, rs) (the host's current state)."""
    vs, rs = {}, {}
    for line in text.splitlines():
        parts = line.split()
        if not parts:
            continue
        proto = {"-t": "TCP", "-u": "UDP"}.get(parts[1], "TCP")
        vip, _, port = parts[2].rpartition(":")
        key = (proto, vip, int(port))
        if parts[0] == "-A":
            sched = parts[parts.index("-s") + 1] if "-s" in parts else "wlc"
            persist = int(parts[parts.index("-p") + 1]) if "-p" in parts else 0
            vs[key] = {"scheduler": sched, "persistent": persist}
            rs.setdefault(key, set())
        elif parts[0] == "-a":
            ip, _, rport = parts[parts.index("-r") + 1].rpartition(":")
            rs.setdefault(key, set()).add((ip, int(rport)))
    return vs, rs


class IPVSProxier:
    mode = "ipvs"

    def __init__(self, cluster_cidr: str = "", scheduler: str = "rr", node_ips=(), masquerade_all: bool = False,
                 dry_run: bool | None = None, dump_path: str | None = None, hostname: str = "", masquerade_bit: int = 14):
        from .iptables import masq_mark
        if scheduler not in SCHEDULERS:
            raise ValueError(f"unknown ipvs scheduler {scheduler!r}")
        self.cluster_cidr, self.scheduler, self.node_ips = cluster_cidr, scheduler, tuple(node_ips)
        self.masquerade_all, self.hostname, self.masq = masquerade_all, hostname, masq_mark(masquerade_bit)
        self.iptables = shutil.which("iptables")
        self.ensured: list = []
        self.ipvsadm = shutil.which("ipvsadm")
        self.dry_run = (self.ipvsadm is None or os.geteuid() != 0) if dry_run is None else dry_run
        self.dump_path = dump_path
        self.vs, self.rs, self.addrs = {}, {}, set()
        self.last_commands: list[str] = []
        self.syncs = 0

    def _host_state(self):
        if self.dry_run:
            return self.vs, self.rs
        r = subprocess.run([self.ipvsadm, "-Sn"], capture_output=True, text=True)
        return parse_save(r.stdout) if r.returncode == 0 else (self.vs, self.rs)

    async def sync(self, services, endpoints):
        vs, rs, addrs = desired(services, endpoints, self.node_ips, self.scheduler, self.hostname)
        self.ensured = ensure_jumps(self.iptables, IPVS_JUMPS, self.dry_run)
        old_vs, old_rs = self._host_state()
        cmds = diff(old_vs, old_rs, vs, rs)
        self.syncs += 1
        self.last_commands = cmds
        add_ips, del_ips = sorted(addrs - self.addrs), sorted(self.addrs - addrs)
        if self.dump_path:
            tmp = self.dump_path + ".tmp"
            with open(tmp, "w") as f:
                f.write(render_restore(vs, rs))
            os.replace(tmp, self.dump_path)
        if not self.dry_run:
            if cmds:
                r = subprocess.run([self.ipvsadm, "-R"], input="\n".join(cmds) + "\n", text=True, capture_output=True)
                if r.returncode != 0:
                    raise RuntimeError(f"ipvsadm -R failed: {r.stderr.strip()}")
            subprocess.run(["ip", "link", "add", DUMMY, "type", "dummy"], capture_output=True)
            for ip in add_ips:
                subprocess.run(["ip", "addr", "add", f"{ip}/32", "dev", DUMMY], capture_output=True)
            for ip in del_ips:
                subprocess.run(["ip", "addr", "del", f"{ip}/32", "dev", DUMMY], capture_output=True)
            ipt = shutil.which("iptables-restore")
            if ipt:
                subprocess.run([ipt, "--noflush"], input=render_iptables(services, self.cluster_cidr, self.masquerade_all,
                                                                         self.masq), text=True, capture_output=True)
        self.vs, self.rs, self.addrs = vs, rs, addrs

    async def stop(self):
        pass
