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
