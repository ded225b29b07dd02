"""KubeletConfiguration files and dynamic kubelet config.

Reference:
  * pkg/kubelet/apis/kubeletconfig/v1alpha1 (KubeletConfiguration, kubeletconfig/v1alpha1):
    the config-file / ConfigMap form of the kubelet's flags; `--config` (KubeletConfigFile
    gate) loads one from disk (configfiles/configfiles.go);
  * pkg/kubelet/kubeletconfig (DynamicKubeletConfig gate, `--dynamic-config-dir`):
    Node.spec.configSource.configMapRef {namespace, name, uid} names a ConfigMap whose `kubelet`
    key holds a KubeletConfiguration; the controller downloads it (checkpoint/download.go,
    UID must match), checkpoints it (checkpoint/store: checkpoints/<uid>, meta/current,
    meta/last-known-good), points `current` at it and restarts the kubelet to apply it
    (configsync.go); at start-up `current` is loaded, parsed and validated, falling back to
    last-known-good (rollback.go) with ConfigOK=False; `current` becomes last-known-good once it
    survived ConfigTrialDuration (default 10 min) without exceeding CrashLoopThreshold restarts;
  * status/status.go: the ConfigOK node condition and its messages.
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
import time

import yaml


log = logging.getLogger("amdkube.kubelet.config")


def _dur(v) -> float:
    if isinstance(v, (int, float)):
        return float(v)
    from .eviction import _duration
    return _duration(str(v))


def _map_str(sep="<"):
    def conv(v):
        if isinstance(v, str):
            return v
        return ",".join(f"{k}{sep}{x}" for k, x in sorted(v.items()))
    return conv


def _gates(v):
    return v if isinstance(v, str) else ",".join(f"{k}={str(x).lower()}" for k, x in sorted(v.items()))


# KubeletConfiguration (v1alpha1 JSON names) → KubeletConfig attribute, converter
FIELDS = {
    "syncFrequency": ("sync_frequency", _dur),
    "fileCheckFrequency": ("file_check_frequency", _dur),
    "address": ("address", str),
    "port": ("port", int),
    "podManifestPath": ("pod_manifest_path", str),
    "nodeStatusUpdateFrequency": ("node_status_update_frequency", _dur),
    "imageMinimumGCAge": ("minimum_image_ttl_duration", _dur),
    "imageGCHighThresholdPercent": ("image_gc_high_threshold", int),
    "imageGCLowThresholdPercent": ("image_gc_low_threshold", int),
    "cpuManagerPolicy": ("cpu_manager_policy", str),
    "cpuManagerReconcilePeriod": ("cpu_manager_reconcile_period", _dur),
    "maxPods": ("max_pods", int),
    "clusterDomain": ("cluster_domain", str),
    "clusterDNS": ("cluster_dns", list),
    "resolvConf": ("resolv_conf", str),
    "evictionHard": ("eviction_hard", _map_str("<")),
    "evictionSoft": ("eviction_soft", _map_str("<")),
    "evictionSoftGracePeriod": ("eviction_soft_grace_period", _map_str("=")),
    "evictionMinimumReclaim": ("eviction_minimum_reclaim", _map_str("=")),
    "evictionPressureTransitionPeriod": ("eviction_pressure_transition_period", _dur),
    "evictionMaxPodGracePeriod": ("eviction_max_pod_grace_period", int),
    "kubeReserved": ("kube_reserved", _map_str("=")),
    "systemReserved": ("system_reserved", _map_str("=")),
    "enforceNodeAllocatable": ("enforce_node_allocatable", lambda v: v if isinstance(v, str) else ",".join(v)),
    "featureGates": ("feature_gates", _gates),
    "experimentalAllowedUnsafeSysctls": ("allowed_unsafe_sysctls", list),
    "maximumDeadContainersPerContainer": ("maximum_dead_containers_per_container", int),
    "maximumDeadContainers": ("maximum_dead_containers", int),
    "minimumGCAge": ("minimum_container_ttl_duration", _dur),
    "cgroupDriver": ("cgroup_driver", str),
}
# accepted for compatibility, no effect here (the reference's knobs for parts this kubelet
# implements differently: docker, the QoS cgroup root, authn/z webhooks, cAdvisor port, ...)
IGNORED = {"kind", "apiVersion", "configTrialDuration", "crashLoopThreshold", "authentication", "authorization",
           "cgroupsPerQOS", "cgroupRoot", "hairpinMode", "readOnlyPort", "tlsCertFile", "tlsPrivateKeyFile",
           "registryPullQPS", "registryBurst", "eventRecordQPS", "eventBurst", "enableDebuggingHandlers", "healthzPort",
           "healthzBindAddress", "oomScoreAdj", "streamingConnectionIdleTimeout", "volumeStatsAggPeriod",
           "runtimeRequestTimeout", "serializeImagePulls", "kubeAPIQPS", "kubeAPIBurst", "podPidsLimit", "hostnameOverride",
           "podCIDR", "rotateCertificates", "staticPodURL", "staticPodURLHeader", "manifestURL", "manifestURLHeader",
           "failSwapOn", "containerLogMaxSize", "containerLogMaxFiles", "contentType", "makeIPTablesUtilChains",
           "iptablesMasqueradeBit", "iptablesDropBit", "systemReservedCgroup", "kubeReservedCgroup", "kubeletCgroups",
           "systemCgroups", "cAdvisorPort"}


def validate(cfg) -> list[str]:
    """kubeletconfig/validation: the ranges a configuration must respect."""
    errs = []
    if cfg.max_pods < 0:
        errs.append("maxPods must not be a negative number")
    if not (0 <= cfg.image_gc_low_threshold <= cfg.image_gc_high_threshold <= 100):
        errs.append("imageGCLowThresholdPercent must be ≤ imageGCHighThresholdPercent, both in [0, 100]")
    if cfg.node_status_update_frequency <= 0 or cfg.sync_frequency <= 0:
        errs.append("nodeStatusUpdateFrequency and syncFrequency must be positive")
    if cfg.cpu_manager_policy not in ("none", "static"):
        errs.append(f"cpuManagerPolicy {cfg.cpu_manager_policy!r} is unknown")
    if not (0 <= cfg.port < 65536):
        errs.append("port must be in [0, 65535] (0: any free port)")
    try:
        from .eviction import parse_thresholds
        parse_thresholds(cfg.eviction_hard or "", cfg.eviction_soft, cfg.eviction_soft_grace_period, cfg.eviction_minimum_reclaim)
        from .cm import parse_reserved
        parse_reserved(cfg.kube_reserved)
        parse_reserved(cfg.system_reserved)
    except Exception as e:   # noqa: BLE001 — any parse error is a validation error
        errs.append(str(e))
    return errs


def apply(cfg, kc: dict):
    """A copy of `cfg` with a KubeletConfiguration applied (ValueError on unknown fields,
    bad values or a configuration that fails validation)."""
    if not isinstance(kc, dict):
        raise ValueError("KubeletConfiguration must be an object")
    if kc.get("kind", "KubeletConfiguration") != "KubeletConfiguration":
        raise ValueError(f"kind {kc.get('kind')!r} is not KubeletConfiguration")
    changes = {}
    for k, v in kc.items():
        if k in IGNORED:
            continue
        if k not in FIELDS:
            raise ValueError(f"unknown KubeletConfiguration field {k!r}")
        attr, conv = FIELDS[k]
        try:
            changes[attr] = conv(v)
        except (TypeError, ValueError) as e:
            raise ValueError(f"{k}: {e}") from e
    new = dataclasses.replace(cfg, **changes)
    errs = validate(new)
    if errs:
        raise ValueError("; ".join(errs))
    return new


def load_file(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f) or {}


# ------------------------------------------------------------------ dynamic config
class DynamicConfig:
    """The kubeletconfig controller: checkpoint store + current / last-known-good + trial."""

    def __init__(self, dirpath: str, trial: float = 600.0, crash_loop_threshold: int = 10, clock=time.time):
        self.dir, self.trial, self.crash_loop_threshold, self.clock = dirpath, trial, crash_loop_threshold, clock
        os.makedirs(os.path.join(dirpath, "checkpoints"), exist_ok=True)
        os.makedirs(os.path.join(dirpath, "meta"), exist_ok=True)
        self.condition = {"type": "ConfigOK", "status": "True", "message": "using current (default)",
                          "reason": "current is set to the local default, and no init config was provided"}
        self.using: dict | None = None

    # ------------------------------------------------------------- meta files
    def _meta(self, name) -> dict | None:
        p = os.path.join(self.dir, "meta", name)
        try:
            with open(p) as f:
                txt = f.read().strip()
            return json.loads(txt) if txt else None
        except (OSError, ValueError):
            return None

    def _set_meta(self, name, ref: dict | None):
        p = os.path.join(self.dir, "meta", name)
        with open(p + ".tmp", "w") as f:
            f.write(json.dumps(ref) if ref else "")
        os.replace(p + ".tmp", p)

    def _checkpoint(self, uid) -> str:
        return os.path.join(self.dir, "checkpoints", uid)

    def _load(self, ref: dict, base):
        with open(self._checkpoint(ref["uid"])) as f:
            cm = json.load(f)
        text = (cm.get("data") or {}).get("kubelet")
        if text is None:
            raise ValueError("ConfigMap has no `kubelet` key")
        return apply(base, yaml.safe_load(text) or {})

    # -------------------------------------------------------------- start-up
    def bootstrap(self, base):
        """Effective configuration at start-up: current if it loads, parses and validates and
        has not crash-looped in its trial, else last-known-good, else the local config."""
        cur, lkg = self._meta("current"), self._meta("last-known-good")
        if cur is None:
            self.using = None
            return base
        starts = (self._meta("startups") or {}).get(cur["uid"], [])
        now = self.clock()
        starts = [t for t in starts if now - t < self.trial] + [now]
        self._set_meta("startups", {cur["uid"]: starts})
        reason = None
        if len(starts) > self.crash_loop_threshold:
            reason = f"current failed trial period due to crash loop (UID: {cur['uid']!r})"
        else:
            try:
                cfg = self._load(cur, base)
                self.using = cur
                self.condition = {"type": "ConfigOK", "status": "True", "reason": "passing all checks",
                                  "message": f"using current (UID: {cur['uid']!r})"}
                meta_t = os.path.getmtime(os.path.join(self.dir, "meta", "current"))
                if now - meta_t >= self.trial and lkg != cur:
                    self._set_meta("last-known-good", cur)     # survived its trial period
                return cfg
            except FileNotFoundError:
                reason = f"failed to load current (UID: {cur['uid']!r})"
            except (ValueError, yaml.YAMLError) as e:
                reason = f"failed to validate current (UID: {cur['uid']!r})" if "must" in str(e) or ";" in str(e) \
                    else f"failed to parse current (UID: {cur['uid']!r})"
        log.warning("dynamic config: %s; rolling back to last-known-good", reason)
        self.last_error = reason
        if lkg is not None:
            try:
                cfg = self._load(lkg, base)
                self.using = lkg
                self.condition = {"type": "ConfigOK", "status": "False", "reason": reason,
                                  "message": f"using last-known-good (UID: {lkg['uid']!r})"}
                return cfg
            except (OSError, ValueError, yaml.YAMLError) as e:
                log.warning("dynamic config: last-known-good unusable: %r", e)
        self.using = None
        self.condition = {"type": "ConfigOK", "status": "False", "reason": reason, "message": "using last-known-good (default)"}
        return base

    # ------------------------------------------------------------------ sync
    async def sync(self, client, node: dict) -> bool:
        """configsync.go: True when the kubelet must restart to apply a new current."""
        src = ((node.get("spec") or {}).get("configSource")) or None
        cur = self._meta("current")
        if src is None:
            if cur is not None:
                self._set_meta("current", None)
                return True
            return False
        ref = src.get("configMapRef") or None
        if ref is None:
            self._fail("invalid NodeConfigSource, exactly one subfield must be non-nil, but all were nil")
            return False
        if not (ref.get("uid") and ref.get("name") and ref.get("namespace")):
            self._fail("invalid ObjectReference, all of UID, Name, and Namespace must be specified")
            return False
        if cur is not None and cur.get("uid") == ref["uid"]:
            return False
        try:
            cm = await client.get("configmaps", ref["name"], ref["namespace"])
        except Exception:   # noqa: BLE001
            self._fail(f"failed to download ConfigMap with name {ref['name']!r} from namespace {ref['namespace']!r}")
            return False
        if (cm.get("metadata") or {}).get("uid") != ref["uid"]:
            self._fail(f"invalid ObjectReference, UID {ref['uid']!r} does not match UID of downloaded ConfigMap "
                       f"{(cm.get('metadata') or {}).get('uid')!r}")
            return False
        p = self._checkpoint(ref["uid"])
        with open(p + ".tmp", "w") as f:
            json.dump(cm, f)
        os.replace(p + ".tmp", p)
        self._set_meta("current", {"namespace": ref["namespace"], "name": ref["name"], "uid": ref["uid"]})
        log.info("dynamic config: current is now ConfigMap %s/%s (UID %s); restarting to apply",
                 ref["namespace"], ref["name"], ref["uid"])
        return True

    def _fail(self, why: str):
        self.condition = dict(self.condition, status="False", reason=f"failed to sync, reason: {why}")
