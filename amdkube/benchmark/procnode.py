"""A one-node cluster with every node daemon in its own process (the deployment shape).

LocalCluster runs the whole node on one event loop, which is right for tests. A real MI355X
node runs rocshim, the AMD device plugin and the kubelet as separate daemons, as the
reference runs dockerd, the NVIDIA plugin DaemonSet and the kubelet. Under a 30-pods-per-step
density load the single loop becomes the bottleneck. ProcessNode keeps the control plane
(apiserver + scheduler) in the calling process and spawns the three daemons:

  python -m amdkube rocshim           --listen <sock> --state-dir ...
  python -m amdkube amd-device-plugin --backend <b> --max-gpus N --plugins-dir ...
  python -m amdkube kubelet           --server <url> --container-runtime-endpoint <sock> ...

Used by bench.py / podbench (`--procs`, the default).
"""
from __future__ import annotations

import asyncio
import os
import shutil
import signal
import subprocess
import sys
import tempfile

from ..apiserver import APIServer
from ..client import Client
from ..scheduler import Scheduler

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Backend:
    def __init__(self, name):
        self.name = name


class _SchedulerStats:
    """Stand-in for the in-process Scheduler's counters when it runs as its own process."""
    scheduled = bind_errors = 0

    def __init__(self, client):
        self.client = client

    async def stop(self):
        pass


class ProcessNode:
    def __init__(self, backend: str = "auto", n_gpus: int | None = None, node_name: str = "mi355x-node-0",
                 relist_period: float = 1.0, health_probe: str = "none", scheduler_process: bool = True,
                 isolation: str | None = None):
        self.scheduler_process = scheduler_process
        # real GPUs: the strongest device isolation the node offers; the fake backend: advisory env
        self.isolation = isolation or ("env" if backend in ("fake", "none") else "auto")
        self.backend_name, self.n_gpus, self.node_name = backend, n_gpus, node_name
        self.relist_period, self.health_probe = relist_period, health_probe
        self.base = tempfile.mkdtemp(prefix="ak-proc-", dir="/tmp")
        self.procs: list[subprocess.Popen] = []
        self.api = self.client = self.scheduler = None
        self.backend = _Backend(backend)

    def _spawn(self, name, args):
        log = open(os.path.join(self.base, f"{name}.log"), "ab")
        env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        prof = os.environ.get("AMDKUBE_PROFILE_DIR")     # cProfile every daemon (<dir>/<name>.prof)
        pre = ["-m", "cProfile", "-o", os.path.join(prof, f"{name}.prof")] if prof else []
        p = subprocess.Popen([sys.executable, *pre, "-m", "amdkube", *args], stdout=log, stderr=subprocess.STDOUT, env=env,
                             start_new_session=True, cwd=ROOT)
        self.procs.append(p)
        return p

    async def start(self):
        b = self.base
        self.api = await APIServer().start()
        self.client = Client(self.api.url, token=self.api.loopback_token, pool=256)
        if self.scheduler_process:
            self._spawn("scheduler", ["scheduler", "--server", self.api.url, "--token", self.api.loopback_token, "--port", "0"])
            self.scheduler = _SchedulerStats(self.client)
        else:
            self.scheduler = await Scheduler(Client(self.api.url, token=self.api.loopback_token, pool=256)).start()
        sock = os.path.join(b, "rocshim.sock")
        plugins = os.path.join(b, "plugins")
        self._spawn("rocshim", ["rocshim", "--listen", sock, "--state-dir", os.path.join(b, "rocshim"),
                                "--hooks-dir", os.path.join(b, "hooks.d"), "--isolation", self.isolation])
        dp = ["amd-device-plugin", "--backend", self.backend_name, "--plugins-dir", plugins, "--health-interval", "5",
              "--health-probe", self.health_probe]
        if self.n_gpus:
            dp += ["--max-gpus", str(self.n_gpus)]
        for _ in range(400):
            if os.path.exists(sock):
                break
            await asyncio.sleep(0.025)
        self._spawn("amd-device-plugin", dp)
        self._spawn("kubelet", ["kubelet", "--server", self.api.url, "--token", self.api.loopback_token,
                                "--node-name", self.node_name, "--root-dir", os.path.join(b, "kubelet"),
                                "--device-plugin-dir", plugins, "--container-runtime-endpoint", sock, "--port", "0",
                                "--pleg-relist-period", str(self.relist_period), "--gpu-stats-backend", "none"])
        return self

    async def wait_gpus(self, n: int, timeout: float = 60.0, resource: str = "amd.com/gpu"):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end:
            for p in self.procs:
                if p.poll() is not None:
                    raise RuntimeError(f"{p.args[3]} exited with {p.returncode}; see {self.base}")
            node = await self.client.get_or_none("nodes", self.node_name)
            if node and int(((node.get("status") or {}).get("allocatable") or {}).get(resource, 0)) >= n:
                return node
            await asyncio.sleep(0.05)
        raise TimeoutError(f"node never advertised {n} GPUs (logs in {self.base})")

    def daemon_pids(self) -> dict[str, int]:
        """{"kubelet": pid, "runtime": pid (rocshim), "device-plugin": pid, "scheduler": pid}."""
        role = {"kubelet": "kubelet", "rocshim": "runtime", "amd-device-plugin": "device-plugin", "scheduler": "scheduler"}
        out = {}
        for p in self.procs:
            args = p.args
            i = args.index("amdkube") + 1 if "amdkube" in args else None
            if i is not None and i < len(args) and args[i] in role:
                out[role[args[i]]] = p.pid
        return out

    def cpu_seconds(self) -> dict:
        """user+system CPU seconds of each node daemon so far (per-pod cost accounting)."""
        import psutil
        out = {}
        for p in self.procs:
            try:
                t = psutil.Process(p.pid).cpu_times()
                out[" ".join(p.args[2:4]) if "-m" in p.args[:2] else str(p.pid)] = round(t.user + t.system, 3)
            except psutil.Error:
                pass
        t = psutil.Process().cpu_times()       # this process: the apiserver and the bench driver
        out["amdkube apiserver+bench"] = round(t.user + t.system, 3)
        return out

    async def stop(self):
        for p in reversed(self.procs):     # kubelet, plugin, then rocshim
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
                try:
                    await asyncio.get_running_loop().run_in_executor(None, p.wait, 10)
                except subprocess.TimeoutExpired:
                    p.kill()
        # containers run in their own sessions; rocshim keeps them on SIGTERM (restart safety)
        import json
        for kind in ("containers", "sandboxes"):
            d = os.path.join(self.base, "rocshim", kind)
            for f in [x for x in os.listdir(d) if x.endswith(".json")] if os.path.isdir(d) else ():
                try:
                    pid = json.load(open(os.path.join(d, f))).get("pid") or 0
                    if pid > 1:
                        os.killpg(pid, signal.SIGKILL)
                except (OSError, ValueError):
                    pass
        if self.scheduler:
            await self.scheduler.stop()
            await self.scheduler.client.close()
        if self.client:
            await self.client.close()
        if self.api:
            await self.api.stop()
        shutil.rmtree(self.base, ignore_errors=True)
