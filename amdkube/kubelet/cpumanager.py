"""CPU manager (pkg/kubelet/cm/cpumanager), with MI355X GPU-NUMA alignment.

Reference:
  * policy_none.go / policy_static.go — `--cpu-manager-policy=none|static`. The static policy
    gives every container of a Guaranteed pod with an integer CPU request that many exclusive
    CPUs; all other containers run on the shared pool (all CPUs minus the exclusive ones). A
    reserved set (ceil(kube-reserved + system-reserved cpu) CPUs, taken by topology from the
    lowest ids) stays in the shared pool and is never handed out exclusively; the static policy
    requires that reservation to be > 0.
  * cpu_assignment.go takeByTopology — whole free sockets first when the request covers one,
    then whole free cores, then single threads, preferring partly used cores (less
    fragmentation).
  * state/state_checkpoint.go (`cpu_manager_state`: policyName, defaultCpuSet, entries) and
    the validation against the policy on restart.
  * cpu_manager.go reconcileState (`--cpu-manager-reconcile-period`): shared-pool containers
    are re-pinned (CRI UpdateContainerResources) whenever the shared pool changes.

MI355X-first addition: a container that holds GPUs takes its exclusive CPUs from the NUMA
node(s) of those GPUs (`amd.com/numa-node` device attribute from the AMD plugin) when they have
room — the host-side half of GPU locality (DMA staging, launch threads, RCCL proxies) that the
reference release only gained later through the topology manager.
"""
from __future__ import annotations

import json
import logging
import math
import os
from dataclasses import dataclass

log = logging.getLogger("amdkube.kubelet.cpumanager")


# ----------------------------------------------------------------------- cpusets
def parse_cpuset(s: str) -> set[int]:
    out: set[int] = set()
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def format_cpuset(cpus) -> str:
    xs = sorted(cpus)
    out, i = [], 0
    while i < len(xs):
        j = i
        while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
            j += 1
        out.append(str(xs[i]) if i == j else f"{xs[i]}-{xs[j]}")
        i = j + 1
    return ",".join(out)


# ---------------------------------------------------------------------- topology
@dataclass(frozen=True)
class CPUInfo:
    cpu: int
    socket: int
    core: int        # globally unique core key: socket * 100000 + core_id
    numa: int


class CPUTopology:
    """topology.Discover from sysfs: logical CPU → (socket, core, NUMA node)."""

    def __init__(self, cpus: list[CPUInfo]):
        self.cpus = {c.cpu: c for c in cpus}
        self.sockets = sorted({c.socket for c in cpus})
        self.cores = sorted({c.core for c in cpus})

    @property
    def num_cpus(self):
        return len(self.cpus)

    def cpus_per_core(self):
        return max(1, self.num_cpus // max(1, len(self.cores)))

    def cpus_per_socket(self):
        return max(1, self.num_cpus // max(1, len(self.sockets)))

    @classmethod
    def discover(cls, sysfs: str = "/sys") -> "CPUTopology":
        base = os.path.join(sysfs, "devices", "system", "cpu")
        numa_of: dict[int, int] = {}
        nodes = os.path.join(sysfs, "devices", "system", "node")
        if os.path.isdir(nodes):
            for n in os.listdir(nodes):
                if n.startswith("node") and n[4:].isdigit():
                    try:
                        with open(os.path.join(nodes, n, "cpulist")) as f:
                            for c in parse_cpuset(f.read().strip()):
                                numa_of[c] = int(n[4:])
                    except OSError:
                        pass
        try:
            with open(os.path.join(base, "online")) as f:
                online = parse_cpuset(f.read().strip())
        except OSError:
            online = set(range(os.cpu_count() or 1))
        try:   # only the CPUs this kubelet may hand out (its cgroup cpuset / affinity)
            online &= os.sched_getaffinity(0)
        except (AttributeError, OSError):
            pass
        out = []
        for c in sorted(online):
            t = os.path.join(base, f"cpu{c}", "topology")
            try:
                sock = int(open(os.path.join(t, "physical_package_id")).read())
                core = int(open(os.path.join(t, "core_id")).read())
            except (OSError, ValueError):
                sock, core = 0, c
            out.append(CPUInfo(c, sock, sock * 100000 + core, numa_of.get(c, sock)))
        return cls(out)

    @classmethod
    def synthetic(cls, sockets: int, cores_per_socket: int, threads: int = 2, numa_per_socket: int = 1) -> "CPUTopology":
        """Linux numbering: thread t of core k on socket s is cpu t*S*C + s*C + k."""
        out = []
        n_cores = sockets * cores_per_socket
        for t in range(threads):
            for s in range(sockets):
                for k in range(cores_per_socket):
                    numa = s * numa_per_socket + (k * numa_per_socket) // cores_per_socket
                    out.append(CPUInfo(t * n_cores + s * cores_per_socket + k, s, s * 100000 + k, numa))
        return cls(out)


def take_by_topology(topo: CPUTopology, available: set[int], n: int) -> set[int]:
    """cpu_assignment.go takeByTopology: n CPUs from `available` — whole free sockets, then
    whole free cores, then threads of the cores with the fewest free threads first."""
    if n > len(available):
        raise ValueError(f"not enough cpus available to satisfy request: requested {n}, available {len(available)}")
    if n == 0:
        return set()
    avail = set(available)
    result: set[int] = set()
    by_socket: dict[int, list[int]] = {}
    by_core: dict[int, list[int]] = {}
    for c in avail:
        info = topo.cpus[c]
        by_socket.setdefault(info.socket, []).append(c)
        by_core.setdefault(info.core, []).append(c)
    need = n
    per_socket, per_core = topo.cpus_per_socket(), topo.cpus_per_core()
    if need >= per_socket:
        for s in sorted(by_socket):
            if len(by_socket[s]) == per_socket and need >= per_socket:
                result.update(by_socket[s])
                need -= per_socket
    if need >= per_core:
        free_cores = sorted((core for core, cs in by_core.items() if len(cs) == per_core and not (set(cs) & result)),
                            key=lambda k: (topo.cpus[by_core[k][0]].socket, k))
        for core in free_cores:
            if need < per_core:
                break
            result.update(by_core[core])
            need -= per_core
    if need:
        rest = [c for c in avail - result]
        # threads of partly used cores first (keeps whole cores free), then by socket and id
        used = {topo.cpus[c].core for c in topo.cpus if c not in avail} | {topo.cpus[c].core for c in result}
        rest.sort(key=lambda c: (topo.cpus[c].core not in used, len(by_core[topo.cpus[c].core]),
                                 topo.cpus[c].socket, topo.cpus[c].core, c))
        result.update(rest[:need])
    return result


# ------------------------------------------------------------------------- manager
class CPUManager:
    """One node's CPU manager: `none` records nothing; `static` keeps exclusive assignments
    keyed by <pod uid>/<container name> and checkpoints them."""

    def __init__(self, policy: str = "none", topology: CPUTopology | None = None, reserved_cpus_milli: int = 0,
                 state_file: str | None = None):
        if policy not in ("none", "static"):
            raise ValueError(f"unknown cpu manager policy {policy!r}")
        self.policy = policy
        self.topo = topology or (CPUTopology.discover() if policy == "static" else CPUTopology([]))
        self.state_file = state_file
        self.all = set(self.topo.cpus)
        self.assignments: dict[str, set[int]] = {}
        self.reserved: set[int] = set()
        if policy == "static":
            n = math.ceil(reserved_cpus_milli / 1000)
            if n <= 0:
                raise ValueError("the static policy requires systemreserved.cpu + kubereserved.cpu to be greater than zero")
            self.reserved = take_by_topology(self.topo, self.all, n)
            self._load()
        self.last_default: str | None = None

    # ------------------------------------------------------------------ state
    def _load(self):
        if not self.state_file or not os.path.exists(self.state_file):
            self._save()
            return
        try:
            with open(self.state_file) as f:
                st = json.load(f)
        except (OSError, ValueError) as e:
            raise RuntimeError(f"could not restore state from checkpoint: {e}")
        if st.get("policyName") != self.policy:
            raise RuntimeError(f"configured policy {self.policy!r} differs from state checkpoint policy "
                               f"{st.get('policyName')!r}; remove {self.state_file} to switch")
        entries = {k: parse_cpuset(v) for k, v in (st.get("entries") or {}).items()}
        # policy_static.go validateState: assignments disjoint, inside the machine, off the reserved set
        seen: set[int] = set()
        for k, cs in entries.items():
            if cs & seen or cs & self.reserved or not cs <= self.all:
                raise RuntimeError(f"invalid state: assignment {k}={format_cpuset(cs)} overlaps or is out of range")
            seen |= cs
        self.assignments = entries

    def _save(self):
        if not self.state_file:
            return
        os.makedirs(os.path.dirname(self.state_file) or ".", exist_ok=True)
        tmp = self.state_file + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"policyName": self.policy, "defaultCpuSet": format_cpuset(self.default_set()),
                       "entries": {k: format_cpuset(v) for k, v in sorted(self.assignments.items())}}, f)
        os.replace(tmp, self.state_file)

    # ---------------------------------------------------------------- policy
    def default_set(self) -> set[int]:
        used = set().union(*self.assignments.values()) if self.assignments else set()
        return self.all - used

    def assignable(self) -> set[int]:
        return self.default_set() - self.reserved

    @staticmethod
    def guaranteed_cpus(pod: dict, container: dict) -> int:
        """policy_static.go guaranteedCPUs: integer CPU count of a Guaranteed pod's container."""
        from .qos import pod_qos
        if pod_qos(pod) != "Guaranteed":
            return 0
        from ..api.quantity import Quantity
        req = ((container.get("resources") or {}).get("requests") or {}).get("cpu") or \
            ((container.get("resources") or {}).get("limits") or {}).get("cpu")
        if not req:
            return 0
        milli = Quantity(req).milli_value()
        return milli // 1000 if milli % 1000 == 0 else 0

    def allocate(self, pod: dict, container: dict, prefer_numa: set[int] | None = None) -> str:
        """The cpuset the container must run on (exclusive CPUs or the shared pool); '' with
        the none policy (no pinning)."""
        if self.policy != "static":
            return ""
        key = f"{pod['metadata']['uid']}/{container['name']}"
        n = self.guaranteed_cpus(pod, container)
        if n == 0:
            return format_cpuset(self.default_set())
        if key in self.assignments:
            return format_cpuset(self.assignments[key])
        avail = self.assignable()
        cs = None
        if prefer_numa:
            local = {c for c in avail if self.topo.cpus[c].numa in prefer_numa}
            if len(local) >= n:
                cs = take_by_topology(self.topo, local, n)
        if cs is None:
            cs = take_by_topology(self.topo, avail, n)
        self.assignments[key] = cs
        self._save()
        log.info("cpu manager: %s gets exclusive cpus %s%s", key, format_cpuset(cs),
                 f" (GPU NUMA {sorted(prefer_numa)})" if prefer_numa else "")
        return format_cpuset(cs)

    def exclusive(self, uid: str, name: str) -> bool:
        return f"{uid}/{name}" in self.assignments

    def release_pod(self, uid: str):
        gone = [k for k in self.assignments if k.startswith(uid + "/")]
        for k in gone:
            del self.assignments[k]
        if gone:
            self._save()

    def retain_only(self, active_uids: set[str]):
        """Drop assignments of pods no longer on the node (restart reconciliation)."""
        gone = [k for k in self.assignments if k.split("/", 1)[0] not in active_uids]
        for k in gone:
            del self.assignments[k]
        if gone:
            self._save()
