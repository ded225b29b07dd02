"""bench.py's driver contract on CPU: torchrun with 2 ranks over gloo, rank 0 drives the node
(fake 8xMI355X backend, busybox pods instead of the gfx950 vector-add), every rank brackets the
timed steps with barriers, the elapsed time is MAX-reduced and rank 0 prints one JSON line."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", AMDKUBE_REQUIRE_NATIVE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "fake", "--no-sched-perf", "--density-nodes", "0", "--image", "busybox",
           "--pod-arg=-c", "--pod-arg=true"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["unit"] == "pods/s"
    assert d["metric"].startswith("p50 GPU-pod startup latency") and d["higher_is_better"] is True
    assert d["gpu_pods"] == 4 and d["failed_pods"] == 0, d
    assert d["cpu_pods"] == 2 * round(22 * 2 / 8)
    assert d["value"] > 0 and abs(d["value"] - (d["gpu_pods"] + d["cpu_pods"]) / (d["ms_per_step"] * d["steps"] / 1000)) < 0.05 * d["value"]


def test_bench_eight_ranks_gloo_fake_8gpu_node():
    """The driver's N=8 launch rehearsed on CPU: torchrun --nproc-per-node 8 over gloo, a fake
    8×MI355X node, busybox GPU pods. One JSON line, n_gpus 8, every step's 8 GPU pods on 8
    distinct device IDs, and the timed region MAX-reduced over the 8 ranks."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", AMDKUBE_REQUIRE_NATIVE="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1",
           "--backend", "fake", "--no-sched-perf", "--no-node-density", "--density-nodes", "0", "--image", "busybox",
           "--pod-arg=-c", "--pod-arg=true"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["steps"] == 2 and d["failed_pods"] == 0, d
    assert d["gpu_pods"] == 16 and d["cpu_pods"] == 2 * 22
    assert d["gpu_devices_per_step"] == [8, 8], d["gpu_devices_per_step"]
    assert len(d["gpu_devices_seen"]) == 8
    assert d["config"]["parallelism"] == "8 allocatable MI355X"


def test_bench_node_density_fields_single_rank():
    """The density_test.go fields (batch of 10, 10-in-sequence with 50 background, kubelet and
    runtime CPU/RSS, API p99) are reported beside their limits."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", AMDKUBE_REQUIRE_NATIVE="0")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--backend", "fake",
           "--no-sched-perf", "--density-nodes", "0", "--image", "busybox", "--pod-arg=-c", "--pod-arg=true"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    nd = d["node_density"]
    assert "error" not in nd, nd
    for k in ("batch10_startup_ms", "seq10_bg50_startup_ms"):
        assert set(d[k]) == {"p50", "p90", "p99"} and 0 < d[k]["p50"] <= d[k]["p99"]
    for k in ("kubelet_cpu_cores_p50", "kubelet_cpu_cores_p95", "runtime_cpu_cores_p50", "runtime_rss_mib",
              "kubelet_rss_mib", "api_p99_ms", "batch10_batch_ms"):
        assert d[k] is not None and d[k] >= 0, k
    assert nd["limits"]["api_p99_ms"] == 1000 and nd["limits"]["kubelet_rss_mib"] == 100
    assert isinstance(nd["within_limits"], bool)
