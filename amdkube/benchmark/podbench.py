"""GPU-pod density / startup benchmark driver (runs the whole node in one process).

Metric (BASELINE.json): p50 GPU-pod startup latency + sustained GPU-pod throughput at
1/2/4/8 allocatable MI355X. One "step" = a burst of `pods_per_gpu × N` GPU pods, each
requesting `amd.com/gpu: 1` through the legacy limits path (ResourceV2 → device-granular
binding), each running the real gfx950 `rocm/vector-add` workload (the reference's
cuda-vector-add e2e image, 50,000 fp32 elements) on exactly its assigned GPU; the step ends
when every pod has Succeeded. Pods are deleted as they finish. Measured per pod from a
watch (the density test's method, test/e2e/scalability/density.go:771-819):
  create → scheduled (bind observed) → started (container running/terminated observed) → Succeeded.

Startup latency (the SLO metric, ≤ 5 s p50/p90/p99) is reported for the first wave of each
burst (pods that found a free GPU at creation, i.e. no queueing); node-side latency
(bind → start) is reported for every pod.

Node density (test/e2e_node/density_test.go, {"cmd":"node_density"}): the reference's two
limit-checked tests on this node — a batch of 10 pods created at once (startup p50/p90/p99 ≤
16/18/20 s, whole batch ≤ 25 s, :72-92) and 10 pods created in sequence beside 50 running
background pods (p50/p90/p99 ≤ 5/9/10 s, :213-229) — run with pause pods as in the reference
and again with GPU pods, while the kubelet's and the runtime's CPU (cores, per 1 s window,
p50/p95 ≤ 0.30/0.50 and 0.40/0.60) and RSS (≤ 100 / 500 MiB, :76-83) are sampled, plus the
apiserver's API call p99 (≤ 1 s, test/e2e/framework/metrics_util.go:52).

Protocol (stdin/stdout JSON lines, used by bench.py): {"cmd":"run","steps":K} → result line;
{"cmd":"node_density"} → result line; {"cmd":"quit"}.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from amdkube.utils.trace import POD_TRACE
from amdkube.api import meta as m  # noqa: E402
from amdkube.localcluster import LocalCluster  # noqa: E402

log = logging.getLogger("amdkube.podbench")


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))
    return xs[k]


# test/e2e_node/density_test.go:72-92, 76-83, 213-229; test/e2e/framework/metrics_util.go:52
DENSITY_LIMITS = {"batch10_startup_ms": {"p50": 16000, "p90": 18000, "p99": 20000}, "batch10_batch_ms": 25000,
                  "seq10_bg50_startup_ms": {"p50": 5000, "p90": 9000, "p99": 10000},
                  "kubelet_cpu_cores": {"p50": 0.30, "p95": 0.50}, "runtime_cpu_cores": {"p50": 0.40, "p95": 0.60},
                  "kubelet_rss_mib": 100, "runtime_rss_mib": 500, "api_p99_ms": 1000}


class ResourceSampler:
    """density_test.go's ResourceCollector (1 s housekeeping): CPU cores per 1 s window and RSS
    of named node daemons, sampled with psutil."""

    def __init__(self, pids: dict[str, int], period: float = 1.0):
        import psutil
        self.period = period
        self.procs = {}
        for name, pid in pids.items():
            try:
                self.procs[name] = psutil.Process(pid)
            except psutil.Error:
                pass
        self.cores: dict[str, list] = {n: [] for n in self.procs}
        self.rss: dict[str, list] = {n: [] for n in self.procs}
        self._task = None

    def _times(self):
        import psutil
        out = {}
        for n, p in self.procs.items():
            try:
                t = p.cpu_times()
                out[n] = (t.user + t.system, p.memory_info().rss)
            except psutil.Error:
                pass
        return out

    def _window(self):
        cur, t1 = self._times(), time.monotonic()
        for n, (cpu, rss) in cur.items():
            if n in self._prev:
                self.cores[n].append((cpu - self._prev[n][0]) / max(1e-6, t1 - self._t0))
            self.rss[n].append(rss)
        self._prev, self._t0 = cur, t1

    async def _run(self):
        while True:
            await asyncio.sleep(self.period)
            self._window()

    def start(self):
        self._prev, self._t0 = self._times(), time.monotonic()
        self._task = asyncio.create_task(self._run())

    async def stop(self) -> dict:
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
        if time.monotonic() - self._t0 >= 0.2 or not any(self.cores.values()):
            self._window()                      # the last (partial) window
        out = {}
        for n in self.procs:
            cs, rs = self.cores[n], self.rss[n]
            out[n] = {"cpu_cores_p50": round(pct(cs, 50), 3) if cs else None,
                      "cpu_cores_p95": round(pct(cs, 95), 3) if cs else None,
                      "rss_mib_max": round(max(rs) / 2**20, 1) if rs else None,
                      "rss_mib_last": round(rs[-1] / 2**20, 1) if rs else None, "windows": len(cs)}
        return out


def cpu_pods_for(n_gpus: int) -> int:
    """Density composition: the reference's 30 pods per node (density.go) as 8 GPU pods (one
    per MI355X of a full node) + 22 pause pods, scaled to N allocatable GPUs (weak scaling)."""
    return int(round(22 * n_gpus / 8.0 + 1e-9)) if n_gpus != 1 else 3


class PodBench:
    def __init__(self, lc: LocalCluster, n_gpus: int, pods_per_gpu: int, image: str, args: list[str], mode: str = "density"):
        self.lc, self.n, self.ppg, self.image, self.args = lc, n_gpus, pods_per_gpu, image, args
        self.mode = mode
        self.cpu_per_step = cpu_pods_for(n_gpus)
        self.pending_cleanup: list[str] = []
        self.seq = 0
        self.t: dict[str, dict] = {}
        self.done_events: dict[str, asyncio.Event] = {}
        self.failed: list[str] = []
        self._watch_task = None
        self.deleting: set = set()
        self.step_devices: list[list[str]] = []      # per density step: the distinct GPUs its pods ran on

    def cpu_pod(self, name):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "labels": {"app": "podbench"}},
                "spec": {"terminationGracePeriodSeconds": 0,
                         "containers": [{"name": "pause", "image": "amdkube/pause:3.1",
                                         "resources": {"requests": {"cpu": "10m", "memory": "10Mi"}}}]}}

    def pod(self, name):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "labels": {"app": "podbench"}},
                "spec": {"restartPolicy": "Never", "terminationGracePeriodSeconds": 0,
                         # IfNotPresent, as for the reference's tagged e2e image (k8s.gcr.io/cuda-vector-add:v0.1):
                         # an untagged image defaults to Always, and every start would then queue
                         # behind the kubelet's serialized, --registry-qps=5 limited puller
                         "containers": [{"name": "vector-add", "image": self.image, "args": self.args,
                                         "imagePullPolicy": "IfNotPresent",
                                         "resources": {"limits": {"amd.com/gpu": "1"}}}]}}

    async def start(self):
        self._watch_task = asyncio.create_task(self._watch())
        await asyncio.sleep(0.2)

    async def _watch(self):
        c = self.lc.client
        while True:
            try:
                async for typ, obj in c.watch("pods", "default", "", label_selector="app=podbench", timeout_seconds=3600):
                    self._observe(typ, obj)
            except asyncio.CancelledError:
                raise
            except Exception:
                await asyncio.sleep(0.05)

    def _observe(self, typ, obj):
        name = m.name_of(obj)
        rec = self.t.get(name)
        if rec is None:
            return
        now = time.perf_counter()
        uid = m.uid_of(obj)
        if "bound" not in rec and (obj.get("spec") or {}).get("nodeName"):
            rec["bound"] = now
            POD_TRACE(uid, "bench_bound")
        if "devices" not in rec:
            ids = [d for er in (obj.get("spec") or {}).get("extendedResources") or [] for d in er.get("assigned") or []]
            if ids:
                rec["devices"] = ids
        st = obj.get("status") or {}
        if "started" not in rec:
            for cs in st.get("containerStatuses") or []:
                s = cs.get("state") or {}
                if "running" in s or "terminated" in s:
                    rec["started"] = now
                    POD_TRACE(uid, "bench_started")
        ph = st.get("phase")
        if rec.get("cpu"):
            if ph == "Running" and "started" in rec and "done" not in rec:
                rec["done"] = now
                ev = self.done_events.get(name)
                if ev:
                    ev.set()
            elif ph == "Failed" and "done" not in rec:
                rec["done"] = now
                self.failed.append(f"{name}: {st.get('reason')} {st.get('message')}")
                self.done_events[name].set()
            return
        if ph in ("Succeeded", "Failed") and "done" not in rec:
            rec["done"] = now
            rec.setdefault("started", now)
            rec.setdefault("bound", now)
            if ph == "Failed":
                self.failed.append(f"{name}: {st.get('reason')} {st.get('message')} {json.dumps(st.get('containerStatuses'))[:300]}")
            ev = self.done_events.get(name)
            if ev:
                ev.set()
            if name not in self.deleting:
                self.deleting.add(name)
                asyncio.create_task(self._delete(name))

    async def _delete(self, name):
        try:
            await self.lc.client.delete("pods", name, "default", grace=0)
        except Exception:
            pass

    async def step(self, timeout=300.0):
        total = self.n * self.ppg
        names = []
        for i in range(total):
            self.seq += 1
            names.append(f"vadd-{self.seq:06d}")
        for nm in names:
            self.t[nm] = {"wave": 0}
            self.done_events[nm] = asyncio.Event()
        for i, nm in enumerate(names):
            self.t[nm]["wave"] = i // self.n
        creates = []
        for nm in names:
            self.t[nm]["create"] = time.perf_counter()
            creates.append(self.lc.client.create(self.pod(nm), "default"))
        await asyncio.gather(*creates)
        await asyncio.wait_for(asyncio.gather(*(self.done_events[nm].wait() for nm in names)), timeout)
        return names

    async def density_step(self, timeout=300.0):
        """density.go on the real node: N GPU pods (one per MI355X, real vector-add run to
        completion on its assigned GPU) + the density share of pause pods, created at once; the
        step ends when every pause pod is Running and every GPU pod has Succeeded. The previous
        step's pause pods are deleted while this one runs."""
        old, self.pending_cleanup = self.pending_cleanup, []
        gpu, cpu = [], []
        for _ in range(self.n):
            self.seq += 1
            gpu.append(f"vadd-{self.seq:06d}")
        for _ in range(self.cpu_per_step):
            self.seq += 1
            cpu.append(f"pause-{self.seq:06d}")
        for nm in gpu + cpu:
            self.t[nm] = {"wave": 0, "cpu": nm in cpu}
            self.done_events[nm] = asyncio.Event()
        tw = time.time()
        # the GPU pods are submitted first and the pause pods right after them (a client that
        # queues its accelerator work ahead of the rest of the batch)
        for group in (gpu, cpu):
            creates = []
            for nm in group:
                self.t[nm]["create"] = time.perf_counter()
                creates.append(self.lc.client.create(self.pod(nm) if nm in gpu else self.cpu_pod(nm), "default"))
            for obj in await asyncio.gather(*creates):
                POD_TRACE(m.uid_of(obj), "bench_create", tw)
                if group is gpu:
                    POD_TRACE(m.uid_of(obj), "bench_gpu_pod", tw)
        # the previous step's pause pods go once this step's pods are in (their deletes would
        # otherwise queue in the apiserver ahead of this step's creates)
        for nm in old:
            self.deleting.add(nm)
            asyncio.create_task(self._delete(nm))
        await asyncio.wait_for(asyncio.gather(*(self.done_events[nm].wait() for nm in gpu + cpu)), timeout)
        self.pending_cleanup = cpu
        self.step_devices.append(sorted({d for nm in gpu for d in self.t[nm].get("devices", [])}))
        return gpu + cpu

    async def run(self, steps: int):
        t0 = time.perf_counter()
        self.step_devices = []
        names = []
        for _ in range(steps):
            names += await (self.density_step() if self.mode == "density" else self.step())
        el = time.perf_counter() - t0
        cpu_recs = [self.t[n] for n in names if self.t[n].get("cpu")]
        names_all = names
        names = [n for n in names if not self.t[n].get("cpu")]
        recs = [self.t[n] for n in names]
        first = [r["started"] - r["create"] for r in recs if r["wave"] == 0]
        allstart = [r["started"] - r["create"] for r in recs]
        node = [r["started"] - r["bound"] for r in recs]
        sched = [r["bound"] - r["create"] for r in recs if r["wave"] == 0]
        life = [r["done"] - r["started"] for r in recs]
        ms = lambda v: None if v is None else round(v * 1000, 2)  # noqa: E731
        cpu_start = [r["started"] - r["create"] for r in cpu_recs]
        every = allstart + cpu_start
        return {"pods": len(names_all), "gpu_pods": len(names), "cpu_pods": len(cpu_recs), "elapsed_s": el,
                "pods_per_s": len(names_all) / el if el else 0.0, "gpu_pods_per_s": len(names) / el if el else 0.0,
                "p50_startup_all_pods_ms": ms(pct(every, 50)), "p90_startup_all_pods_ms": ms(pct(every, 90)),
                "p99_startup_all_pods_ms": ms(pct(every, 99)), "p50_cpu_pod_startup_ms": ms(pct(cpu_start, 50)),
                "failed": len(self.failed), "failures": self.failed[:5],
                "p50_startup_ms": ms(pct(first, 50)), "p90_startup_ms": ms(pct(first, 90)), "p99_startup_ms": ms(pct(first, 99)),
                "p50_startup_all_ms": ms(pct(allstart, 50)), "p50_node_startup_ms": ms(pct(node, 50)),
                "p99_node_startup_ms": ms(pct(node, 99)), "p50_schedule_ms": ms(pct(sched, 50)),
                "p50_pod_runtime_ms": ms(pct(life, 50)),
                "gpu_devices_per_step": [len(d) for d in self.step_devices],
                "gpu_devices_seen": sorted({d for ds in self.step_devices for d in ds})}

    # ------------------------------------------------------------ node density (density_test.go)
    async def _create_and_wait(self, names: list[str], gpu: set, interval: float = 0.0, timeout: float = 300.0):
        """Create pods (GPU pods for names in `gpu`, pause pods otherwise) `interval` apart; wait
        until each is Running (pause) or Succeeded (GPU). Returns (create→started lags, batch s)."""
        t0 = time.perf_counter()
        for nm in names:
            self.t[nm] = {"wave": 0, "cpu": nm not in gpu}
            self.done_events[nm] = asyncio.Event()
        creates = []
        for nm in names:
            self.t[nm]["create"] = time.perf_counter()
            creates.append(asyncio.ensure_future(self.lc.client.create(self.pod(nm) if nm in gpu else self.cpu_pod(nm),
                                                                       "default")))
            if interval:
                await asyncio.sleep(interval)
        await asyncio.gather(*creates)
        await asyncio.wait_for(asyncio.gather(*(self.done_events[nm].wait() for nm in names)), timeout)
        lags = [self.t[nm]["started"] - self.t[nm]["create"] for nm in names]
        return lags, time.perf_counter() - t0

    def _names(self, prefix: str, n: int) -> list[str]:
        out = []
        for _ in range(n):
            self.seq += 1
            out.append(f"{prefix}-{self.seq:06d}")
        return out

    async def _cleanup(self, names):
        for nm in names:
            if nm not in self.deleting:
                self.deleting.add(nm)
                await self._delete(nm)
        end = time.monotonic() + 60
        while time.monotonic() < end:
            left, _ = await self.lc.client.list("pods", "default", label_selector="app=podbench")
            if not left:
                return
            await asyncio.sleep(0.1)

    async def node_density(self, pids: dict[str, int], api=None) -> dict:
        """density_test.go's limit-checked tests, with pause pods (the reference's) and GPU pods."""
        api_mark = len(api.lat_samples) if api is not None else 0
        from . import apiresp
        try:
            await apiresp.reset_metrics(self.lc.client)      # metrics_util.go ResetMetrics
            api_reset = True
        except Exception as e:
            log.warning("DELETE /metrics failed: %r", e)
            api_reset = False
        sampler = ResourceSampler(pids)
        sampler.start()
        ms = lambda v: None if v is None else round(v * 1000, 2)  # noqa: E731
        lat = lambda xs: {"p50": ms(pct(xs, 50)), "p90": ms(pct(xs, 90)), "p99": ms(pct(xs, 99))}  # noqa: E731
        out = {}
        old, self.pending_cleanup = self.pending_cleanup, []
        await self._cleanup(old)
        # create a batch of 10 pods, 0 interval (density_test.go:72-92)
        names = self._names("batch", 10)
        lags, el = await self._create_and_wait(names, set())
        out["batch10_startup_ms"], out["batch10_batch_ms"] = lat(lags), ms(el)
        await self._cleanup(names)
        # the same batch as GPU pods (amd.com/gpu: 1 each; they queue for the node's GPUs)
        names = self._names("gbatch", 10)
        lags, el = await self._create_and_wait(names, set(names))
        out["batch10_gpu_startup_ms"], out["batch10_gpu_batch_ms"] = lat(lags), ms(el)
        await self._cleanup(names)
        # 10 pods in sequence beside 50 background pods (density_test.go:213-229), GPU pods
        bg = self._names("bg", 50)
        await self._create_and_wait(bg, set())
        lags = []
        for nm in self._names("seq", 10):
            lag, _ = await self._create_and_wait([nm], {nm})
            lags += lag
        out["seq10_bg50_startup_ms"] = lat(lags)
        # and with pause pods, as the reference runs it
        lags = []
        seqp = self._names("seqp", 10)
        for nm in seqp:
            lag, _ = await self._create_and_wait([nm], set())
            lags += lag
        out["seq10_bg50_pause_startup_ms"] = lat(lags)
        await self._cleanup(bg + seqp)
        res = await sampler.stop()
        for role in ("kubelet", "runtime"):
            r = res.get(role) or {}
            out[f"{role}_cpu_cores_p50"], out[f"{role}_cpu_cores_p95"] = r.get("cpu_cores_p50"), r.get("cpu_cores_p95")
            out[f"{role}_rss_mib"] = r.get("rss_mib_max")
        out["resource_windows"] = min((r.get("windows") or 0 for r in res.values()), default=0)
        if api_reset:
            # the reference's API-responsiveness check: quantiles of apiserver_request_latencies_summary
            summ = apiresp.summarize(await apiresp.read_latency_metrics(self.lc.client))
            out["api_p99_ms"], out["api_list_p99_ms"], out["api_worst"] = summ["api_p99_ms"], summ["api_list_p99_ms"], summ["worst"][:3]
            out["api_bad_calls"], out["api_source"] = summ["api_bad_calls"], summ["source"]
        if api is not None:
            # cross-check from the exact per-request samples
            exact = api.latency_summary(api_mark)
            out["api_p99_ms_exact"] = exact["api_p99_ms"]
            if not api_reset:
                out["api_p99_ms"], out["api_list_p99_ms"], out["api_worst"] = exact["api_p99_ms"], exact["api_list_p99_ms"], exact["worst"][:3]
        out["limits"] = DENSITY_LIMITS
        out["within_limits"] = _within(out)
        return out


def _within(r: dict) -> bool:
    """Every reported density value at or under its reference limit."""
    L = DENSITY_LIMITS
    checks = []
    for k in ("batch10_startup_ms", "seq10_bg50_startup_ms"):
        checks += [(r.get(k) or {}).get(q) is not None and r[k][q] <= L[k][q] for q in ("p50", "p90", "p99")]
    checks.append(r.get("batch10_batch_ms") is not None and r["batch10_batch_ms"] <= L["batch10_batch_ms"])
    for role in ("kubelet", "runtime"):
        lim = L[f"{role}_cpu_cores"]
        for q in ("p50", "p95"):
            v = r.get(f"{role}_cpu_cores_{q}")
            checks.append(v is not None and v <= lim[q])
        v = r.get(f"{role}_rss_mib")
        checks.append(v is not None and v <= L[f"{role}_rss_mib"])
    if r.get("api_p99_ms") is not None:
        checks.append(r["api_p99_ms"] <= L["api_p99_ms"])
    return all(checks)


async def serve(args):
    logging.basicConfig(level=logging.WARNING, stream=sys.stderr)
    if args.procs:
        from amdkube.benchmark.procnode import ProcessNode
        lc = ProcessNode(args.backend, args.gpus, relist_period=1.0, health_probe=args.health_probe,
                         isolation=args.isolation)
    else:
        lc = LocalCluster(gpus=args.backend, n_gpus=args.gpus, relist_period=1.0, with_controllers=False,
                          health_probe=args.health_probe, isolation=args.isolation)
    await lc.start()
    await lc.wait_gpus(args.gpus, 60)
    node = await lc.client.get("nodes", lc.node_name)
    devs = list(((node["status"].get("extendedResources") or {}).get("amd.com/gpu") or {}).get("resources") or {})
    pb = PodBench(lc, args.gpus, args.pods_per_gpu, args.image, args.args, args.mode)
    await pb.start()
    iso = getattr(lc, "isolation", None)
    if iso == "auto":
        from amdkube.runtime.rocshim import probe_isolation, resolve_isolation
        iso = resolve_isolation("auto", probe_isolation())
    print(json.dumps({"ready": True, "gpus": devs, "backend": lc.backend.name if lc.backend else "none", "isolation": iso}),
          flush=True)
    loop = asyncio.get_running_loop()
    reader = asyncio.StreamReader()
    await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), sys.stdin)
    try:
        while True:
            line = await reader.readline()
            if not line:
                break
            cmd = json.loads(line)
            if cmd.get("cmd") == "quit":
                break
            if cmd.get("cmd") == "run":
                cpu0 = lc.cpu_seconds() if hasattr(lc, "cpu_seconds") else {}
                res = await pb.run(int(cmd.get("steps", 1)))
                if cpu0:   # CPU seconds each node daemon spent on the steps
                    res["node_cpu_s"] = {k: round(v - cpu0.get(k, 0.0), 3) for k, v in lc.cpu_seconds().items()}
                res["scheduler"] = {"scheduled": lc.scheduler.scheduled, "bind_errors": lc.scheduler.bind_errors}
                print(json.dumps(res), flush=True)
            if cmd.get("cmd") == "node_density":
                pids = lc.daemon_pids() if hasattr(lc, "daemon_pids") else {"kubelet": os.getpid(), "runtime": os.getpid()}
                try:
                    res = await pb.node_density(pids, getattr(lc, "api", None))
                except Exception as e:          # reported, never fatal to the headline bench
                    res = {"error": repr(e)}
                print(json.dumps(res), flush=True)
            if cmd.get("cmd") == "schedperf":
                from amdkube.benchmark.schedperf import run_schedperf
                res = await run_schedperf(int(cmd.get("nodes", 100)), int(cmd.get("pods", 3000)), gpus_per_node=8,
                                          gpu_pods=cmd.get("gpu_pods", "mixed"))
                print(json.dumps(res), flush=True)
    finally:
        await lc.stop()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--pods-per-gpu", type=int, default=4, help="churn mode: GPU pods per GPU per step")
    ap.add_argument("--mode", default="density", choices=("density", "churn"))
    ap.add_argument("--procs", type=int, default=1, help="1: rocshim, device plugin and kubelet as separate processes")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--image", default="rocm/vector-add")
    ap.add_argument("--health-probe", default="none")
    ap.add_argument("--isolation", default=None, help="rocshim device isolation (default: auto on real GPUs, env on fake)")
    ap.add_argument("args", nargs="*", default=[])
    prof_path = os.environ.get("AMDKUBE_CPROFILE")      # the bench process itself (apiserver + client)
    if prof_path:
        import cProfile
        pr = cProfile.Profile()
        pr.enable()
        try:
            asyncio.run(serve(ap.parse_args()))
        finally:
            pr.disable()
            pr.dump_stats(f"{prof_path}.podbench.{os.getpid()}")
        return
    asyncio.run(serve(ap.parse_args()))


if __name__ == "__main__":
    main()
