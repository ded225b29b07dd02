"""amdkube — an MI355X-native, GPU-aware Kubernetes-compatible cluster system.

Layers: api (object model) → store (MVCC + watch + WAL) →
apiserver (REST + watch + admission) → client (informers, workqueue, leader election) →
scheduler (device-granular, xGMI-topology aware) / controllers / kubelet (DeviceManager,
CRI runtime client) ↔ deviceplugin (v1alpha2 gRPC, AMD GPU plugin over amd-smi) ↔
runtime (rocshim CRI server) → native (C++ amd-smi shim, topology allocator, pause) and
kernels (HIP gfx950 validation workloads, RCCL xGMI probe).
"""
__version__ = "0.1.0"
GIT_VERSION = "v1.9.6-amdkube.0"
