"""Kubelet stats provider: the /stats/summary API (pkg/kubelet/apis/stats/v1alpha1/types.go,
pkg/kubelet/stats/{cri_stats_provider,cadvisor_stats_provider}.go, server/stats/summary.go)
and the /metrics/cadvisor exposition, built from the runtime's CRI container stats plus the
node-side collectors in monitoring/cadvisor.py.

Node: cpu, memory, network (physical interfaces), fs (the kubelet root's filesystem),
runtime.imageFs (the runtime's image store), rlimit, systemContainers (kubelet, pods) and the
MI355X accelerators. Pod: containers (cpu with usageNanoCores, memory with usage / working set /
rss / page faults, rootfs = writable layer, logs, accelerators), network (the sandbox's own
network namespace when it has one), volume (du for node-local plugins, statvfs for mounted
ones — metrics_du / metrics_statfs), ephemeral-storage (rootfs + logs + local volumes).
"""
from __future__ import annotations

import asyncio
import os
import time

from ..api import meta as m
from ..grpcdesc.cri import CRI as C
from ..monitoring import cadvisor as cad
from .kuberuntime import L_POD_UID

DU_PLUGINS = ("kubernetes.io/empty-dir", "kubernetes.io/secret", "kubernetes.io/configmap", "kubernetes.io/downward-api",
              "kubernetes.io/projected", "kubernetes.io/git-repo")


class StatsProvider:
    def __init__(self, kubelet, du_ttl: float = 10.0):
        self.k = kubelet
        self.du = cad.DuCache(du_ttl)
        self._cpu_prev: dict[str, tuple[float, int]] = {}
        self._sandbox_pid: dict[str, int] = {}

    def rate(self, key: str, used_ns: int) -> int:
        """usageNanoCores: CPU time per wall time since the previous sample (cAdvisor's rate)."""
        t = time.monotonic()
        prev = self._cpu_prev.get(key)
        self._cpu_prev[key] = (t, used_ns)
        if prev is None or t <= prev[0] or used_ns < prev[1]:
            return 0
        return int((used_ns - prev[1]) / (t - prev[0]))

    async def _pod_network(self, sid: str) -> dict:
        pid = self._sandbox_pid.get(sid)
        if pid is None:
            try:
                info = await self.k.cri.pod_sandbox_info(sid)
                pid = int(info.get("pid") or 0)
            except Exception:
                pid = 0
            self._sandbox_pid[sid] = pid
        if not pid:
            return {}
        if os.path.realpath(f"/proc/{pid}/ns/net") == os.path.realpath("/proc/self/ns/net"):
            return {}          # host network: the node's counters, not the pod's
        return cad.network_stats(f"/proc/{pid}/net/dev", prefer="eth0")

    def _volume_stats(self, uid: str, now: str) -> tuple[list[dict], int]:
        """(VolumeStats of the pod's set-up volumes, bytes of those on the node's local disk)."""
        out, local = [], 0
        for (pu, _outer), mv in list(self.k.volume_manager.mounted.items()):
            if pu != uid or mv.reconstructed:
                continue
            if mv.plugin.name in DU_PLUGINS:
                used, inodes = self.du.get(mv.path)
                fs = cad.fs_stats(mv.path)
                st = {"capacityBytes": fs.get("capacityBytes", 0), "availableBytes": fs.get("availableBytes", 0),
                      "usedBytes": used, "inodesUsed": inodes, "inodes": fs.get("inodes", 0), "inodesFree": fs.get("inodesFree", 0)}
                local += used
            else:
                st = cad.fs_stats(mv.path)
            out.append({"name": mv.outer, "time": now, **st})
        return out, local

    def _logs(self, uid: str, cname: str) -> int:
        """Bytes of the container's log files: pods/<uid>/logs/<container>/<restart>.log."""
        d = os.path.join(self.k.cfg.root_dir, "pods", uid, "logs", cname)
        tot = 0
        try:
            for e in os.scandir(d):
                if e.is_file():
                    tot += e.stat().st_size
        except OSError:
            pass
        return tot

    async def _container_pids(self, cid: str) -> set[int] | None:
        """The container's process tree (CRI ContainerStatus verbose info carries its pid)."""
        from ..monitoring.collector import container_pids
        try:
            _, info = await self.k.cri.container_status(cid, verbose=True)
            pid = int((info or {}).get("pid") or 0)
        except Exception:
            return None
        return container_pids(pid) if pid else None

    async def summary(self) -> dict:
        import psutil
        now = m.now_rfc3339()
        stats = {s.attributes.id: s for s in await self.k.cri.list_container_stats()}
        conts = await self.k.cri.list_containers()
        from ..monitoring.collector import AcceleratorCollector
        accel = AcceleratorCollector(self.k.smi, self.k.node_name)
        dev_map = {(d["namespace"], d["pod"], d["container"]): d["devices"] for d in self.k.server._pod_devices()} \
            if self.k.server is not None else {}
        pods: dict[str, dict] = {}
        sandbox_of: dict[str, str] = {}
        for c in conts:
            if c.state != C.CONTAINER_RUNNING:
                continue
            uid = c.labels.get(L_POD_UID, "")
            p = self.k.pods.get(uid)
            if p is None:
                continue
            sandbox_of.setdefault(uid, c.pod_sandbox_id)
            ent = pods.setdefault(uid, {"podRef": {"name": m.name_of(p), "namespace": m.namespace_of(p), "uid": uid},
                                        "startTime": (p.get("status") or {}).get("startTime"), "containers": []})
            s = stats.get(c.id)
            used = s.cpu.usage_core_nano_seconds.value if s else 0
            mem = s.memory if s else None
            cont = {"name": c.metadata.name, "startTime": now,
                    "cpu": {"time": now, "usageCoreNanoSeconds": used, "usageNanoCores": self.rate(c.id, used)},
                    "memory": {"time": now, "workingSetBytes": mem.working_set_bytes.value if mem else 0,
                               "usageBytes": mem.usage_bytes.value if mem else 0, "rssBytes": mem.rss_bytes.value if mem else 0,
                               "pageFaults": mem.page_faults.value if mem else 0,
                               "majorPageFaults": mem.major_page_faults.value if mem else 0}}
            if s is not None and s.HasField("writable_layer"):
                cont["rootfs"] = {"time": now, "usedBytes": s.writable_layer.used_bytes.value,
                                  "inodesUsed": s.writable_layer.inodes_used.value}
            cont["logs"] = {"time": now, "usedBytes": self._logs(uid, c.metadata.name)}
            ids = dev_map.get((m.namespace_of(p), m.name_of(p), c.metadata.name))
            if ids:
                cont["accelerators"] = accel.accelerator_stats(ids, await self._container_pids(c.id))
            ent["containers"].append(cont)
        for uid, ent in pods.items():
            vols, local = await asyncio.to_thread(self._volume_stats, uid, now)
            if vols:
                ent["volume"] = vols
            net = await self._pod_network(sandbox_of[uid])
            if net:
                ent["network"] = {"time": now, **net}
            ent["ephemeral-storage"] = {"time": now, "usedBytes": local + sum(
                (c.get("rootfs") or {}).get("usedBytes", 0) + (c.get("logs") or {}).get("usedBytes", 0) for c in ent["containers"])}
        live = {c.id for c in conts} | {"__node__"}
        for key in [key for key in self._cpu_prev if key not in live]:
            del self._cpu_prev[key]
        vm = psutil.virtual_memory()
        cpu = psutil.cpu_times()
        node_used = int((cpu.user + cpu.system) * 1e9)
        me = psutil.Process()
        kcpu = me.cpu_times()
        image_fs = {}
        try:
            fsu = (await self.k.cri.image_fs_info())[0]
            image_fs = {**cad.fs_stats(fsu.storage_id.uuid or self.k.cfg.root_dir), "usedBytes": fsu.used_bytes.value,
                        "inodesUsed": fsu.inodes_used.value, "time": now}
        except Exception:
            pass
        node = {"nodeName": self.k.node_name, "startTime": m.now_rfc3339(),
                "cpu": {"time": now, "usageCoreNanoSeconds": node_used, "usageNanoCores": self.rate("__node__", node_used)},
                "memory": {"time": now, "availableBytes": vm.available, "usageBytes": vm.total - vm.available,
                           "workingSetBytes": vm.total - vm.available},
                "fs": {"time": now, **cad.fs_stats(self.k.cfg.root_dir if os.path.isdir(self.k.cfg.root_dir) else "/")},
                "runtime": {"imageFs": image_fs},
                "rlimit": {"time": now, **cad.rlimit()},
                "systemContainers": [{"name": "kubelet", "startTime": m.now_rfc3339(),
                                      "cpu": {"time": now, "usageCoreNanoSeconds": int((kcpu.user + kcpu.system) * 1e9)},
                                      "memory": {"time": now, "usageBytes": me.memory_info().rss,
                                                 "workingSetBytes": me.memory_info().rss}}],
                "accelerators": accel.accelerator_stats(None)}
        net = cad.network_stats()
        if net:
            node["network"] = {"time": now, **net}
        return {"node": node, "pods": list(pods.values())}

    async def render_cadvisor(self) -> str:
        """/metrics/cadvisor: cAdvisor's container_* families (labels container_name, pod_name,
        namespace, id, name, image) plus machine_* and container_accelerator_*."""
        from ..monitoring.collector import AcceleratorCollector
        summ = await self.summary()
        info = cad.machine_info()
        L = []
        fams = [("machine_cpu_cores", "gauge", "Number of CPU cores on the machine."),
                ("machine_memory_bytes", "gauge", "Amount of memory installed on the machine."),
                ("container_cpu_usage_seconds_total", "counter", "Cumulative cpu time consumed in seconds."),
                ("container_memory_usage_bytes", "gauge", "Current memory usage in bytes, including all memory regardless of when it was accessed"),
                ("container_memory_working_set_bytes", "gauge", "Current working set in bytes."),
                ("container_memory_rss", "gauge", "Size of RSS in bytes."),
                ("container_memory_failures_total", "counter", "Cumulative count of memory allocation failures."),
                ("container_fs_usage_bytes", "gauge", "Number of bytes that are consumed by the container on this filesystem."),
                ("container_network_receive_bytes_total", "counter", "Cumulative count of bytes received"),
                ("container_network_transmit_bytes_total", "counter", "Cumulative count of bytes transmitted")]
        for name, typ, hlp in fams:
            L += [f"# HELP {name} {hlp}", f"# TYPE {name} {typ}"]
        L.append(f"machine_cpu_cores {info['num_cores']}")
        L.append(f"machine_memory_bytes {info['memory_capacity']}")
        for p in summ["pods"]:
            ref = p["podRef"]
            for c in p["containers"]:
                lab = f'container_name="{c["name"]}",pod_name="{ref["name"]}",namespace="{ref["namespace"]}"'
                L.append(f'container_cpu_usage_seconds_total{{{lab},cpu="total"}} {c["cpu"]["usageCoreNanoSeconds"] / 1e9:.9f}')
                mem = c["memory"]
                L.append(f"container_memory_usage_bytes{{{lab}}} {mem.get('usageBytes', 0)}")
                L.append(f"container_memory_working_set_bytes{{{lab}}} {mem.get('workingSetBytes', 0)}")
                L.append(f"container_memory_rss{{{lab}}} {mem.get('rssBytes', 0)}")
                L.append(f'container_memory_failures_total{{{lab},type="pgfault",scope="container"}} {mem.get("pageFaults", 0)}')
                L.append(f'container_memory_failures_total{{{lab},type="pgmajfault",scope="container"}} {mem.get("majorPageFaults", 0)}')
                L.append(f"container_fs_usage_bytes{{{lab}}} {(c.get('rootfs') or {}).get('usedBytes', 0)}")
            net = p.get("network")
            if net:
                lab = f'container_name="POD",pod_name="{ref["name"]}",namespace="{ref["namespace"]}",interface="{net.get("name", "eth0")}"'
                L.append(f"container_network_receive_bytes_total{{{lab}}} {net.get('rxBytes', 0)}")
                L.append(f"container_network_transmit_bytes_total{{{lab}}} {net.get('txBytes', 0)}")
        text = "\n".join(L) + "\n"
        if self.k.server is not None:     # the summary's per-container stats (process-attributed VRAM)
            pd = [{"namespace": p["podRef"]["namespace"], "pod": p["podRef"]["name"], "container": c["name"],
                   "devices": [a["id"] for a in c["accelerators"]], "stats": c["accelerators"]}
                  for p in summ["pods"] for c in p["containers"] if c.get("accelerators")]
            text += AcceleratorCollector(self.k.smi, self.k.node_name).render_container_metrics(pd)
        return text
