"""ip-masq-agent: which pod traffic leaving the node is masqueraded.

What cluster/addons/ip-masq-agent/ip-masq-agent.yaml runs on every node labelled
beta.kubernetes.io/masq-agent-ds-ready=true (the kubernetes-incubator/ip-masq-agent v2 image),
its config a YAML/JSON file mounted from the `ip-masq-agent` ConfigMap at
/etc/config/ip-masq-agent:
* nonMasqueradeCIDRs (default the RFC 1918 ranges 10.0.0.0/8, 172.16.0.0/12, 192.168.0.0/16),
  masqLinkLocal (default false: 169.254.0.0/16 is not masqueraded either), resyncInterval
  (default 60s);
* a missing file means the defaults; a file that does not parse or validate keeps the last good
  config;
* every resync the nat chain IP-MASQ-AGENT is rewritten whole through `iptables-restore
  --noflush`: a RETURN per non-masquerade CIDR, then MASQUERADE for everything else (last);
  POSTROUTING sends every non-LOCAL destination to the chain (ensured with -C, appended when
  missing).
Without an iptables binary or root the rules are rendered and kept (`last_rules`), as kube-proxy's
dry mode does, so the agent and its tests run on unprivileged nodes.
"""
from __future__ import annotations

import asyncio
import ipaddress
import logging
import os
import re
import shlex
import shutil
import subprocess

log = logging.getLogger("amdkube.ip-masq-agent")

CHAIN = "IP-MASQ-AGENT"
DEFAULT_NON_MASQ = ["10.0.0.0/8", "172.16.0.0/12", "192.168.0.0/16"]
LINK_LOCAL = "169.254.0.0/16"
POSTROUTING_ARGS = ('-m comment --comment "ip-masq-agent: ensure nat POSTROUTING directs all non-LOCAL destination '
                    f'traffic to our custom {CHAIN} chain" -m addrtype ! --dst-type LOCAL -j {CHAIN}')


class ConfigError(ValueError):
    pass


def _duration(v) -> float:
    if isinstance(v, (int, float)):
        return float(v) / 1e9 if v > 10_000 else float(v)     # Go time.Duration in ns, or seconds
    m = re.fullmatch(r"(?:(\d+(?:\.\d+)?)h)?(?:(\d+(?:\.\d+)?)m(?!s))?(?:(\d+(?:\.\d+)?)s)?(?:(\d+(?:\.\d+)?)ms)?", str(v).strip())
    if not m or not any(m.groups()):
        raise ConfigError(f"resyncInterval: invalid duration {v!r}")
    h, mi, s, ms = (float(x) if x else 0.0 for x in m.groups())
    return h * 3600 + mi * 60 + s + ms / 1000


def parse_config(text: str) -> dict:
    """The config file: YAML or JSON with the three fields (unknown fields are errors, as the
    agent's strict decoding)."""
    import yaml
    try:
        raw = yaml.safe_load(text) if text.strip() else {}
    except yaml.YAMLError as e:
        raise ConfigError(f"config does not parse: {e}") from e
    if raw is None:
        raw = {}
    if not isinstance(raw, dict):
        raise ConfigError("config must be a mapping")
    unknown = set(raw) - {"nonMasqueradeCIDRs", "masqLinkLocal", "resyncInterval"}
    if unknown:
        raise ConfigError(f"unknown config fields: {sorted(unknown)}")
    cfg = {"nonMasqueradeCIDRs": list(DEFAULT_NON_MASQ), "masqLinkLocal": False, "resyncInterval": 60.0}
    if "nonMasqueradeCIDRs" in raw:
        cidrs = raw["nonMasqueradeCIDRs"] or []
        if not isinstance(cidrs, list):
            raise ConfigError("nonMasqueradeCIDRs must be a list")
        for i, c in enumerate(cidrs):
            try:
                ipaddress.ip_network(str(c), strict=False)
            except ValueError:
                raise ConfigError(f"config.NonMasqueradeCIDRs[{i}]: invalid CIDR {c!r}") from None
            if "/" not in str(c):
                raise ConfigError(f"config.NonMasqueradeCIDRs[{i}]: invalid CIDR {c!r}")
        cfg["nonMasqueradeCIDRs"] = [str(c) for c in cidrs]
    if "masqLinkLocal" in raw:
        if not isinstance(raw["masqLinkLocal"], bool):
            raise ConfigError("masqLinkLocal must be a boolean")
        cfg["masqLinkLocal"] = raw["masqLinkLocal"]
    if "resyncInterval" in raw:
        cfg["resyncInterval"] = _duration(raw["resyncInterval"])
    return cfg


def render(cfg: dict) -> str:
    """iptables-restore input for the nat IP-MASQ-AGENT chain."""
    lines = ["*nat", f":{CHAIN} - [0:0]"]
    cidrs = ([] if cfg["masqLinkLocal"] else [LINK_LOCAL]) + cfg["nonMasqueradeCIDRs"]
    for c in cidrs:
        lines.append(f'-A {CHAIN} -d {c} -m comment --comment "ip-masq-agent: local traffic is not subject to MASQUERADE" '
                     "-j RETURN")
    lines.append(f'-A {CHAIN} -m comment --comment "ip-masq-agent: outbound traffic is subject to MASQUERADE (must be last '
                 'in chain)" -j MASQUERADE')
    lines += ["COMMIT", ""]
    return "\n".join(lines)


class MasqAgent:
    def __init__(self, config_path: str = "/etc/config/ip-masq-agent", dry_run: bool | None = None):
        self.config_path = config_path
        self.restore, self.iptables = shutil.which("iptables-restore"), shutil.which("iptables")
        self.dry_run = (self.restore is None or self.iptables is None or os.geteuid() != 0) if dry_run is None else dry_run
        self.config = parse_config("")
        self.last_rules = ""
        self.postrouting_ensured = False
        self.syncs = 0

    def load(self) -> dict:
        """The config file, or the defaults when it is absent; a bad file keeps the last config."""
        try:
            with open(self.config_path) as f:
                text = f.read()
        except FileNotFoundError:
            self.config = parse_config("")
            return self.config
        except OSError as e:
            log.error("reading %s: %r; keeping the previous config", self.config_path, e)
            return self.config
        try:
            self.config = parse_config(text)
        except ConfigError as e:
            log.error("%s: %s; keeping the previous config", self.config_path, e)
        return self.config

    def _ensure_postrouting(self):
        if self.dry_run:
            self.postrouting_ensured = True
            return
        a = shlex.split(POSTROUTING_ARGS)
        if subprocess.run([self.iptables, "-w", "-t", "nat", "-C", "POSTROUTING", *a], capture_output=True).returncode != 0:
            r = subprocess.run([self.iptables, "-w", "-t", "nat", "-A", "POSTROUTING", *a], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"ensuring nat POSTROUTING -> {CHAIN}: {r.stderr.strip()}")
        self.postrouting_ensured = True

    def sync(self) -> str:
        self.load()
        rules = render(self.config)
        if not self.dry_run:
            r = subprocess.run([self.restore, "--noflush", "--counters"], input=rules, text=True, capture_output=True)
            if r.returncode != 0:
                raise RuntimeError(f"iptables-restore: {r.stderr.strip()}")
        self._ensure_postrouting()
        self.last_rules = rules
        self.syncs += 1
        return rules

    async def run(self, stop: asyncio.Event | None = None):
        stop = stop or asyncio.Event()
        while not stop.is_set():
            try:
                await asyncio.to_thread(self.sync)
            except RuntimeError as e:
                log.error("sync: %s", e)
            try:
                await asyncio.wait_for(stop.wait(), self.config["resyncInterval"])
            except asyncio.TimeoutError:
                pass

