"""Feature gates (`--feature-gates=A=true,B=false`).

Reference: pkg/features/kube_features.go:67-76 — `DevicePlugins` is Beta and **default
true** in the fork, `Accelerators` (legacy NVIDIA path) alpha/false (:251-252).
"""
from __future__ import annotations

KNOWN = {
    "DevicePlugins": (True, "Beta"),
    "Accelerators": (False, "Alpha"),            # legacy path: superseded, accepted for flag compatibility
    "TaintNodesByCondition": (False, "Alpha"),
    "PodPriority": (True, "Beta"),
    "GPUTopologyScheduling": (True, "Beta"),     # amdkube: xGMI/NUMA-aware device scoring
    "ReserveDevicesOnAssume": (True, "Beta"),    # amdkube: SURVEY §7.6 #1 fix
    "DeviceHealthFiltering": (True, "Beta"),     # amdkube: SURVEY §7.6 #6 fix
    "AppArmor": (True, "Beta"),                  # kubelet admit + CRI apparmor_profile (amdkube/security/apparmor.py)
}
# the rest of the reference's gate names (kube_features.go:196-240), accepted so a reference
# flag line parses; the behaviour they switch is either always on here or not applicable
for _name, _spec in {
    "ExternalTrafficLocalOnly": (True, "GA"), "DynamicKubeletConfig": (False, "Alpha"), "KubeletConfigFile": (False, "Alpha"),
    "ExperimentalHostUserNamespaceDefaulting": (False, "Beta"), "ExperimentalCriticalPodAnnotation": (False, "Alpha"),
    "TaintBasedEvictions": (False, "Alpha"), "RotateKubeletServerCertificate": (False, "Alpha"),
    "RotateKubeletClientCertificate": (True, "Beta"), "PersistentLocalVolumes": (False, "Alpha"),
    "LocalStorageCapacityIsolation": (False, "Alpha"), "HugePages": (False, "Alpha"), "DebugContainers": (False, "Alpha"),
    "EnableEquivalenceClassCache": (False, "Alpha"), "MountPropagation": (False, "Alpha"),
    "ExpandPersistentVolumes": (False, "Alpha"), "CPUManager": (False, "Alpha"), "ServiceNodeExclusion": (False, "Alpha"),
    "MountContainers": (False, "Alpha"), "VolumeScheduling": (False, "Alpha"), "CSIPersistentVolume": (False, "Alpha"),
    "CustomPodDNS": (False, "Alpha"), "BlockVolume": (False, "Alpha"), "PVCProtection": (False, "Alpha"),
    "ResourceLimitsPriorityFunction": (False, "Alpha"), "SupportIPVSProxyMode": (False, "Beta"), "VolumeSubpath": (True, "GA"),
    "StreamingProxyRedirects": (True, "Beta"), "AdvancedAuditing": (True, "Beta"), "APIResponseCompression": (False, "Alpha"),
    "Initializers": (False, "Alpha"), "APIListChunking": (True, "Beta"), "CustomResourceValidation": (True, "Beta"),
    "ServiceProxyAllowExternalIPs": (False, "Deprecated"), "ReadOnlyAPIDataVolumes": (True, "Deprecated"),
}.items():
    KNOWN.setdefault(_name, _spec)


class FeatureGate:
    def __init__(self, spec: str | dict | None = None):
        self.enabled = {k: v[0] for k, v in KNOWN.items()}
        if spec:
            self.set(spec)

    def set(self, spec):
        items = spec.items() if isinstance(spec, dict) else (kv.split("=", 1) for kv in spec.split(",") if kv.strip())
        for k, v in items:
            k = k.strip()
            if k not in KNOWN:
                raise ValueError(f"unrecognized feature gate: {k}")
            self.enabled[k] = v if isinstance(v, bool) else str(v).strip().lower() in ("true", "1", "yes")

    def __call__(self, name: str) -> bool:
        return self.enabled[name]


DEFAULT = FeatureGate()
