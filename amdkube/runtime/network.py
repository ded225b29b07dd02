"""Pod network plugins for rocshim: host network and CNI.

Reference: pkg/kubelet/network/plugins.go (NetworkPlugin: Init / Event(pod CIDR change) /
SetUpPod / TearDownPod / GetPodNetworkStatus), pkg/kubelet/network/cni/cni.go
(getDefaultCNINetwork: the first *.conf / *.conflist / *.json in --cni-conf-dir in lexical
order; plugins looked up in --cni-bin-dir; SetUpPod = AddNetworkList with
CNI_ARGS "IgnoreUnknown=1;K8S_POD_NAMESPACE=..;K8S_POD_NAME=..;K8S_POD_INFRA_CONTAINER_ID=..";
TearDownPod = DelNetworkList in reverse order), pkg/kubelet/network/kubenet (the pod CIDR
arrives through the CRI UpdateRuntimeConfig call and is substituted into the config).

In the reference dockershim owns the network plugin, and rocshim does the same here, so
PodSandboxStatus reports the IP. The CNI runner follows the libcni contract: each plugin
in a conflist gets `prevResult` from the previous one; the DEL of a failed ADD is best effort.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os

log = logging.getLogger("amdkube.rocshim.network")

POD_CIDR_PLACEHOLDER = "usePodCidr"     # kubenet-style substitution of the node's pod CIDR


class NetworkError(RuntimeError):
    pass


class HostNetwork:
    name = "host"

    def __init__(self, node_ip: str = "127.0.0.1"):
        self.node_ip = node_ip
        self.pod_cidr = ""

    def set_pod_cidr(self, cidr: str):
        self.pod_cidr = cidr

    async def setup(self, sid, meta, netns):
        return self.node_ip

    async def teardown(self, sid, meta, netns):
        pass

    def status(self):
        return True, ""


def _load_conf(conf_dir: str):
    try:
        files = sorted(f for f in os.listdir(conf_dir) if f.endswith((".conf", ".conflist", ".json")))
    except OSError:
        return None
    for f in files:
        try:
            with open(os.path.join(conf_dir, f)) as fh:
                d = json.load(fh)
        except (OSError, ValueError) as e:
            log.warning("error loading CNI config %s: %r", f, e)
            continue
        if "plugins" in d:
            if not d["plugins"]:
                continue
            return d
        # a single-plugin .conf becomes a one-element list (libcni ConfListFromConf)
        return {"cniVersion": d.get("cniVersion", "0.3.1"), "name": d.get("name", ""), "plugins": [d]}
    return None


def _substitute(obj, cidr):
    if isinstance(obj, dict):
        return {k: _substitute(v, cidr) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_substitute(v, cidr) for v in obj]
    if obj == POD_CIDR_PLACEHOLDER:
        return cidr
    return obj


class CNINetwork:
    name = "cni"

    def __init__(self, conf_dir: str, bin_dirs: list[str], node_ip: str = "127.0.0.1", timeout: float = 30.0):
        self.conf_dir = conf_dir
        self.bin_dirs = bin_dirs
        self.node_ip = node_ip
        self.pod_cidr = ""
        self.timeout = timeout

    def set_pod_cidr(self, cidr: str):
        if cidr != self.pod_cidr:
            log.info("pod CIDR set to %s", cidr)
        self.pod_cidr = cidr

    def _netconf(self):
        conf = _load_conf(self.conf_dir)
        if conf is None:
            raise NetworkError(f"no valid CNI network config in {self.conf_dir}")
        if self.pod_cidr:
            conf = _substitute(conf, self.pod_cidr)
        elif POD_CIDR_PLACEHOLDER in json.dumps(conf):
            raise NetworkError("CNI config wants the node's pod CIDR, which is not known yet")
        return conf

    def status(self):
        try:
            self._netconf()
            return True, ""
        except NetworkError as e:
            return False, str(e)

    def _find(self, typ):
        for d in self.bin_dirs:
            p = os.path.join(d, typ)
            if os.access(p, os.X_OK):
                return p
        raise NetworkError(f"failed to find plugin {typ!r} in path {self.bin_dirs}")

    async def _exec(self, plugin: dict, conf: dict, command: str, sid: str, meta: dict, netns: str, prev=None):
        cfg = dict(plugin)
        cfg.setdefault("cniVersion", conf.get("cniVersion", "0.3.1"))
        cfg["name"] = conf.get("name", "")
        if prev is not None:
            cfg["prevResult"] = prev
        env = dict(os.environ, CNI_COMMAND=command, CNI_CONTAINERID=sid, CNI_NETNS=netns or "", CNI_IFNAME="eth0",
                   CNI_PATH=":".join(self.bin_dirs),
                   CNI_ARGS=f"IgnoreUnknown=1;K8S_POD_NAMESPACE={meta.get('namespace', '')};"
                            f"K8S_POD_NAME={meta.get('name', '')};K8S_POD_INFRA_CONTAINER_ID={sid}")
        proc = await asyncio.create_subprocess_exec(self._find(cfg.get("type", "")), stdin=asyncio.subprocess.PIPE,
                                                    stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE, env=env)
        try:
            out, err = await asyncio.wait_for(proc.communicate(json.dumps(cfg).encode()), self.timeout)
        except asyncio.TimeoutError:
            proc.kill()
            raise NetworkError(f"CNI plugin {cfg.get('type')} {command} timed out")
        res = {}
        if out.strip():
            try:
                res = json.loads(out)
            except ValueError:
                raise NetworkError(f"CNI plugin {cfg.get('type')} returned invalid JSON: {out[:200]!r}")
        if proc.returncode != 0:
            raise NetworkError(f"CNI plugin {cfg.get('type')} {command} failed: {res.get('msg') or err.decode()[-300:]}")
        return res

    async def setup(self, sid, meta, netns):
        conf = self._netconf()
        prev = None
        for plugin in conf["plugins"]:
            prev = await self._exec(plugin, conf, "ADD", sid, meta, netns, prev)
        for ipc in (prev or {}).get("ips") or []:
            addr = ipc.get("address", "")
            if addr:
                return addr.split("/")[0]
        raise NetworkError("CNI result carries no IP address")

    async def teardown(self, sid, meta, netns):
        try:
            conf = self._netconf()
        except NetworkError as e:
            log.warning("skipping CNI DEL for %s: %s", sid, e)
            return
        for plugin in reversed(conf["plugins"]):
            try:
                await self._exec(plugin, conf, "DEL", sid, meta, netns)
            except NetworkError as e:
                log.warning("CNI DEL for %s: %s", sid, e)


class KubenetNetwork(CNINetwork):
    """pkg/kubelet/network/kubenet: the kubelet-managed pod network — one `cbr0` bridge owning
    the node's pod CIDR gateway, a veth pair per pod, host-local addresses, hairpin mode and the
    MTU — realised with amdkube's native `amdkube-bridge` + `amdkube-cni` plugins. The config is
    generated from the pod CIDR the kubelet pushes (UpdateRuntimeConfig); until it is known the
    network is not ready ("kubenet does not have netConfig")."""
    name = "kubenet"

    def __init__(self, bin_dirs: list[str], state_dir: str, bridge: str = "cbr0", mtu: int = 1460,
                 node_ip: str = "127.0.0.1", timeout: float = 30.0):
        super().__init__("", bin_dirs, node_ip, timeout)
        self.bridge, self.mtu, self.state_dir = bridge, mtu, state_dir

    def _netconf(self):
        if not self.pod_cidr:
            raise NetworkError("kubenet does not have netConfig: the node has no pod CIDR yet")
        return {"cniVersion": "0.3.1", "name": "kubenet", "plugins": [{
            "type": "amdkube-bridge", "bridge": self.bridge, "mtu": self.mtu, "isGateway": True, "hairpinMode": True,
            "ipam": {"type": "amdkube-cni", "subnet": self.pod_cidr, "dataDir": os.path.join(self.state_dir, "ipam")}}]}
