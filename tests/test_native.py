"""Native layer on CPU: topology allocator C++ == Python reference, ASan/UBSan self-test,
pause semantics, nsexec device isolation (root only), hipcc cross-compile of the kernels."""
import os
import random
import signal
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "amdkube", "_native", "bin")
sys.path.insert(0, os.path.join(ROOT, "native"))


@pytest.fixture(scope="module", autouse=True)
def built():
    import build as nb
    nb.build(sanitize=True, cpu_only=True, jobs=4)


def test_topology_native_matches_python():
    from amdkube.ops import topology as t
    assert t.NATIVE
    rng = random.Random(3)
    for _ in range(200):
        n = rng.choice([4, 8, 8, 16])
        numa = [i // (n // 2) for i in range(n)]
        link = [[0 if i == j else (15 if numa[i] == numa[j] else 30) + rng.randint(0, 2) for j in range(n)] for i in range(n)]
        free = sorted(rng.sample(range(n), rng.randint(1, n)))
        k = rng.randint(1, len(free))
        a = t.select(free, k, link, numa, free)
        b = t.py_select(free, k, link, numa, free)
        assert a[0] == b[0] and abs(a[1] - b[1]) < 1e-9, (free, k, a, b)
        assert abs(t.score(free, k, link, numa, free) - t.py_score(free, k, link, numa, free)) < 1e-9
    assert t.select([0, 1], 3, [[0, 1], [1, 0]], [0, 0])[0] == []


def test_topology_asan_selftest():
    r = subprocess.run([os.path.join(BIN, "topo-selftest-asan")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("binary", ["sampler-selftest-tsan", "sampler-selftest-asan"])
def test_activity_sampler_sanitized_selftest(binary):
    """native/sampler_core.h under ThreadSanitizer and ASan/UBSan: readers racing the sampler
    thread and concurrent start/stop (TSan variant for the shim's sampler)."""
    r = subprocess.run([os.path.join(BIN, binary)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66"))
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr[-3000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr


@pytest.mark.parametrize("binary", ["pause", "pause-asan"])
def test_pause_reaps_and_exits_on_term(binary, tmp_path):
    pid_file = tmp_path / "pid"
    p = subprocess.Popen([os.path.join(BIN, binary), "--pidfile", str(pid_file)])
    for _ in range(100):
        if pid_file.exists() and pid_file.read_text().strip():
            break
        time.sleep(0.01)
    assert int(pid_file.read_text()) == p.pid
    p.send_signal(signal.SIGTERM)
    assert p.wait(5) == 0


@pytest.mark.parametrize("binary", ["amdkube-logpump", "amdkube-logpump-asan"])
def test_logpump_records_under_asan(binary, tmp_path):
    """native/logpump.cpp (and its ASan/UBSan build) on bursts of mixed-size lines from both
    streams: every byte comes back through the CRI decoder, per stream, in order."""
    from amdkube.kubelet.logs import LogOptions, read_logs_sync
    rng = random.Random(7)
    chunks = {1: [], 2: []}
    for _ in range(300):
        fd = rng.choice((1, 2))
        chunks[fd].append(b"y" * rng.choice((0, 1, 80, 4000, 20000, 40000)) + (b"\n" if rng.random() < 0.8 else b""))
    spec = tmp_path / "spec.py"
    spec.write_text("import itertools, os\n"
                    f"c1={chunks[1]!r}\nc2={chunks[2]!r}\n"
                    "for a, b in itertools.zip_longest(c1, c2):\n"
                    "    a and os.write(1, a)\n"
                    "    b and os.write(2, b)\n")
    script = f"exec(open({str(spec)!r}).read())"
    log = tmp_path / "0.log"
    ro, wo = os.pipe()
    re_, we = os.pipe()
    pump = subprocess.Popen([os.path.join(BIN, binary), "--log", str(log), "--stdout-fd", str(ro), "--stderr-fd", str(re_)],
                            pass_fds=(ro, re_), stderr=subprocess.PIPE)
    os.close(ro)
    os.close(re_)
    w = subprocess.Popen([sys.executable, "-c", script], stdout=wo, stderr=we)
    os.close(wo)
    os.close(we)
    assert w.wait(60) == 0
    _, err = pump.communicate(timeout=60)
    assert pump.returncode == 0, err.decode()[-2000:]
    out, errs = [], []
    read_logs_sync(str(log), LogOptions(), out.append, errs.append)
    assert b"".join(out) == b"".join(chunks[1]) and b"".join(errs) == b"".join(chunks[2])


@pytest.mark.skipif(os.geteuid() != 0, reason="mount namespaces need root")
def test_nsexec_hides_other_render_nodes(tmp_path):
    dev = tmp_path / "dev"
    (dev / "dri").mkdir(parents=True)
    for n in ("renderD128", "renderD129", "card1"):
        (dev / "dri" / n).write_text("x")
    (dev / "kfd").write_text("kfd")
    r = subprocess.run([os.path.join(BIN, "amdkube-nsexec"), "--dev-root", str(dev), "--keep", str(dev / "dri" / "renderD129"),
                        "--hide-kfd", "--", "sh", "-c", f"ls {dev}/dri; cat {dev}/kfd; echo end"],
                       capture_output=True, text=True, timeout=30)
    if r.returncode == 126 and "unshare" in r.stderr:
        pytest.skip("unshare not permitted in this container")
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["renderD129", "end"]
    assert sorted(os.listdir(dev / "dri")) == ["card1", "renderD128", "renderD129"]  # host view untouched


def test_hip_kernels_cross_compile_for_gfx950(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not installed")
    out = tmp_path / "vadd.o"
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-c", os.path.join(ROOT, "kernels", "vector_add.hip"), "-o", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    # the device code object must contain MFMA for the burn kernel and be built for gfx950
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", os.path.join(ROOT, "kernels", "gpu_burn.hip"),
                        "-o", str(tmp_path / "burn.s")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    asm = (tmp_path / "burn.s").read_text()
    assert "v_mfma_f32_32x32x16_bf16" in asm and "gfx950" in asm
