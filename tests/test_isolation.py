"""Kernel-enforced GPU device isolation (native/devguard.h, native/devview.c, rocshim modes).

Reference: the container's device list reaches runc through HostConfig.Resources.Devices
(pkg/kubelet/dockershim/docker_container.go:155-172, makeDevices in
pkg/kubelet/kuberuntime/kuberuntime_container.go:277), which the devices cgroup enforces. Here
a fake /dev tree of 8 MI355X render nodes + kfd stands in for the node; the checks are what the
GPU tier repeats on the real MI355X (tests/test_gpu.py::test_device_guard_on_mi355x).
"""
import asyncio
import json
import os
import subprocess
import sys
import tempfile

import pytest

from amdkube.grpcdesc.cri import CRI as C
from amdkube.kubelet.cri_client import CRIClient
from amdkube.runtime import RocShim
from amdkube.runtime.images import NATIVE_BIN
from amdkube.runtime.rocshim import DEVVIEW_LIB, container_caps, probe_isolation, resolve_isolation
from tests.conftest import run, log_text

NSEXEC = os.path.join(NATIVE_BIN, "amdkube-nsexec")
PROBE = probe_isolation(NSEXEC) if os.path.exists(NSEXEC) else {}
needs_landlock = pytest.mark.skipif(PROBE.get("landlock_abi", 0) < 1, reason="kernel without Landlock")

OPEN_ALL = r"""
import glob, json, os, sys
root = sys.argv[1]
res = {}
for p in sorted(glob.glob(root + '/dri/*')) + sorted(glob.glob(root + '/dri/by-path/*')) + [root + '/kfd']:
    try:
        os.close(os.open(p, os.O_RDWR)); res[os.path.basename(p)] = 'ok'
    except OSError as e:
        res[os.path.basename(p)] = e.strerror
# a same-uid process outside the container reaches the host's /dev through /proc/<pid>/root
try:
    os.close(os.open('/proc/%d/root%s/dri/renderD131' % (os.getppid(), root), os.O_RDWR)); res['proc_root'] = 'ok'
except OSError as e:
    res['proc_root'] = e.strerror
try:
    os.mknod(root + '/../mknod-226', 0o020600, os.makedev(226, 140)); res['mknod'] = 'ok'
except OSError as e:
    res['mknod'] = e.strerror
print(json.dumps(res))
"""


@pytest.fixture
def fake_dev():
    d = tempfile.mkdtemp(prefix="akdev", dir="/tmp")
    dev = os.path.join(d, "dev")
    os.makedirs(os.path.join(dev, "dri", "by-path"))
    for m in range(128, 136):   # 8 × MI355X
        open(os.path.join(dev, "dri", f"renderD{m}"), "w").close()
        open(os.path.join(dev, "dri", f"card{m - 128}"), "w").close()
    os.symlink("../renderD129", os.path.join(dev, "dri", "by-path", "pci-0000:15:00.0-render"))
    open(os.path.join(dev, "kfd"), "w").close()
    yield dev
    subprocess.run(["rm", "-rf", d])


def _run(args, env=None, dev=None):
    p = subprocess.run([NSEXEC, *args, "--", sys.executable, "-c", OPEN_ALL, dev], capture_output=True, text=True,
                       timeout=30, env=env)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


@needs_landlock
def test_landlock_gpu_container_sees_exactly_its_render_node(fake_dev):
    keep = f"{fake_dev}/dri/renderD130"
    r = _run(["--no-namespaces", "--landlock", "--dev-root", fake_dev, "--keep", keep], dev=fake_dev)
    assert r["renderD130"] == "ok" and r["kfd"] == "ok"
    others = {k: v for k, v in r.items() if k.startswith(("renderD", "card")) and k != "renderD130"}
    assert len(others) == 15 and set(others.values()) == {"Permission denied"}, r
    assert r["pci-0000:15:00.0-render"] == "Permission denied"    # a link resolves to the denied node
    assert r["proc_root"] == "Permission denied"                   # /proc/<pid>/root is the same inode
    assert r["mknod"] == "Permission denied"


@needs_landlock
def test_landlock_non_gpu_container_has_no_kfd(fake_dev):
    r = _run(["--no-namespaces", "--landlock", "--dev-root", fake_dev, "--hide-kfd"], dev=fake_dev)
    assert r["kfd"] == "Permission denied"
    assert {v for k, v in r.items() if k.startswith("renderD")} == {"Permission denied"}


@needs_landlock
def test_devview_preload_makes_foreign_nodes_absent(fake_dev):
    """ROCr skips an absent render node (ENOENT) but fails hsa_init on a refused one (EACCES,
    measured on MI355X): the rocm handler's preload shows the container exactly its devices."""
    assert os.path.exists(DEVVIEW_LIB)
    keep = f"{fake_dev}/dri/renderD133"
    env = dict(os.environ, AMDKUBE_DEVVIEW_LIB=DEVVIEW_LIB, AMDKUBE_DEVVIEW_ROOT=fake_dev,
               AMDKUBE_DEVVIEW_ALLOW=f"{keep},{fake_dev}/kfd")
    r = _run(["--no-namespaces", "--landlock", "--dev-root", fake_dev, "--keep", keep], env=env, dev=fake_dev)
    assert r["renderD133"] == "ok" and r["kfd"] == "ok"
    # the foreign nodes are not even listed (the directory walk is filtered too) ...
    assert not [k for k in r if k.startswith(("renderD", "card")) and k != "renderD133"], r
    # ... and a link to one resolves to nothing
    assert r["pci-0000:15:00.0-render"] == "No such file or directory"
    # without the preload (or a process that bypasses it) the kernel still refuses
    r = _run(["--no-namespaces", "--landlock", "--dev-root", fake_dev, "--keep", keep], dev=fake_dev)
    assert r["renderD128"] == "Permission denied"


def test_unguarded_launch_sees_everything(fake_dev):
    """Control: without --landlock every node opens (the fixture really is reachable)."""
    r = _run(["--no-namespaces"], dev=fake_dev)
    assert r["renderD128"] == "ok" and r["kfd"] == "ok" and r["proc_root"] == "ok"


def test_isolation_resolution_order():
    full = {"root": True, "cgroup2_writable": True, "userns": True, "landlock_abi": 7}
    assert resolve_isolation("auto", full) == "namespaces"
    assert resolve_isolation("auto", {"root": False, "userns": True, "landlock_abi": 7}) == "userns"
    # the MI355X gpurun box: unprivileged, user.max_user_namespaces=0, Landlock ABI 7
    assert resolve_isolation("auto", {"root": False, "userns": False, "landlock_abi": 7}) == "landlock"
    assert resolve_isolation("auto", {"root": False, "userns": False, "landlock_abi": 0}) == "env"
    assert resolve_isolation("env", full) == "env"
    with pytest.raises(ValueError):
        resolve_isolation("bogus", full)


def test_container_capabilities_from_security_context():
    sc = C.LinuxContainerSecurityContext(capabilities=C.Capability(add_capabilities=["SYS_PTRACE"],
                                                                   drop_capabilities=["MKNOD", "NET_RAW"]))
    caps = container_caps(sc).split(",")
    assert "SYS_PTRACE" in caps and "MKNOD" not in caps and "NET_RAW" not in caps and "CHOWN" in caps
    assert "SYS_ADMIN" not in container_caps(C.LinuxContainerSecurityContext()).split(",")
    assert container_caps(C.LinuxContainerSecurityContext(privileged=True)) == "all"
    assert container_caps(C.LinuxContainerSecurityContext(capabilities=C.Capability(drop_capabilities=["ALL"]))) == "none"


@needs_landlock
def test_rocshim_landlock_mode_end_to_end(fake_dev):
    """rocshim isolation=landlock: the rocm-handler GPU container opens only its render node even
    with every *_VISIBLE_DEVICES unset; the non-GPU container opens neither kfd nor any node."""
    async def go():
        base = tempfile.mkdtemp(prefix="rsll", dir="/tmp")
        shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks"),
                             isolation="landlock", dev_root=fake_dev).start()
        cri = await CRIClient(os.path.join(base, "s.sock")).connect()
        try:
            assert shim.isolation == "landlock"
            sc = C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name="p", uid="u1", namespace="default"))
            sid = await cri.run_pod_sandbox(sc)
            script = ("import os; [os.environ.pop(k, None) for k in list(os.environ) if k.endswith('_VISIBLE_DEVICES')]; "
                      "exec(open(%r).read())")
            prog = os.path.join(base, "open_all.py")
            with open(prog, "w") as f:
                f.write(OPEN_ALL)
            out = {}
            for name, devs in (("gpu", [f"{fake_dev}/kfd", f"{fake_dev}/dri/renderD134"]), ("cpu", [])):
                cfg = C.ContainerConfig(metadata=C.ContainerMetadata(name=name), image=C.ImageSpec(image="busybox"),
                                        command=[sys.executable, "-c", script % prog, fake_dev],
                                        envs=[C.KeyValue(key="ROCR_VISIBLE_DEVICES", value="6")] if devs else [],
                                        devices=[C.Device(container_path=d, host_path=d, permissions="rw") for d in devs])
                cid = await cri.create_container(sid, cfg, sc)
                await cri.start_container(cid)
                for _ in range(500):
                    st, info = await cri.container_status(cid, verbose=True)
                    if st.state == C.CONTAINER_EXITED:
                        break
                    await asyncio.sleep(0.01)
                assert st.exit_code == 0, log_text(st.log_path)
                out[name] = (json.loads(log_text(st.log_path).strip().splitlines()[-1]), info["handler"])
            gpu, handler = out["gpu"]
            assert handler == "rocm"
            assert [k for k, v in gpu.items() if v == "ok"] == ["renderD134", "kfd"]
            assert gpu["mknod"] == "Permission denied"
            cpu, handler = out["cpu"]
            assert handler == "default"
            assert "ok" not in cpu.values(), cpu
        finally:
            await cri.close()
            await shim.stop(kill_pods=True)
            subprocess.run(["rm", "-rf", base])
    run(go())


@needs_landlock
def test_exec_runs_inside_the_container_guard(fake_dev):
    """CRI ExecSync (and the streaming exec, same argv) starts the process under the container's
    own guard, the way docker exec enters the container: a GPU container's exec opens only its
    render node, a non-GPU container's exec reaches neither kfd nor any node."""
    async def go():
        base = tempfile.mkdtemp(prefix="rsex", dir="/tmp")
        shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks"),
                             isolation="landlock", dev_root=fake_dev).start()
        cri = await CRIClient(os.path.join(base, "s.sock")).connect()
        try:
            sc = C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name="p", uid="u2", namespace="default"))
            sid = await cri.run_pod_sandbox(sc)
            prog = os.path.join(base, "open_all.py")
            with open(prog, "w") as f:
                f.write(OPEN_ALL)
            seen = {}
            for name, devs in (("gpu", [f"{fake_dev}/kfd", f"{fake_dev}/dri/renderD131"]), ("cpu", [])):
                cfg = C.ContainerConfig(metadata=C.ContainerMetadata(name=name), image=C.ImageSpec(image="busybox"),
                                        command=["sleep", "30"],
                                        devices=[C.Device(container_path=d, host_path=d, permissions="rw") for d in devs])
                cid = await cri.create_container(sid, cfg, sc)
                await cri.start_container(cid)
                out, err, rc = await cri.exec_sync(cid, [sys.executable, prog, fake_dev], 20)
                assert rc == 0, err
                seen[name] = json.loads(out.decode().strip().splitlines()[-1])
            assert [k for k, v in seen["gpu"].items() if v == "ok"] == ["renderD131", "kfd"], seen["gpu"]
            assert "ok" not in seen["cpu"].values(), seen["cpu"]
        finally:
            await cri.close()
            await shim.stop(kill_pods=True)
            subprocess.run(["rm", "-rf", base])
    run(go())


@needs_landlock
def test_nsexec_under_asan_ubsan(fake_dev):
    """The launcher built with AddressSanitizer + UBSan (host code only) enforces the same view
    and reports no memory or undefined-behaviour error on the guard, mknod and seccomp paths."""
    asan = os.path.join(os.path.dirname(NSEXEC), "amdkube-nsexec-asan")
    if not os.path.exists(asan):
        pytest.skip("sanitizer build absent (python native/build.py --sanitize)")
    keep = f"{fake_dev}/dri/renderD130"
    prof = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amdkube", "runtime", "seccomp_default.json")
    p = subprocess.run([asan, "--no-namespaces", "--landlock", "--dev-root", fake_dev, "--keep", keep, "--seccomp", prof,
                        "--caps", "default", "--", sys.executable, "-c", OPEN_ALL, fake_dev],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1"))
    assert p.returncode == 0, p.stderr[-2000:]
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert [k for k, v in r.items() if v == "ok"] == ["renderD130", "kfd"]
    # a malformed profile is refused cleanly (parser under ASan)
    bad = os.path.join(fake_dev, "..", "bad.json")
    with open(bad, "w") as f:
        f.write('{"defaultAction": "SCMP_ACT_ERRNO", "syscalls": [{"names": ["read"], "action": 7}]')
    p = subprocess.run([asan, "--no-namespaces", "--seccomp", bad, "--", "true"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 126 and "AddressSanitizer" not in p.stderr, p.stderr[-2000:]


@needs_landlock
def test_devview_libdrm_style_enumeration_sees_only_its_own_node(fake_dev, tmp_path):
    """An 8-render-node node under --landlock with the devview preload: a libdrm/ROCr-style walk
    (readdir/scandir/glob of <root>/dri, then stat64/lstat/statx/fstatat/faccessat/fopen/open/
    openat on every node) lists only the container's render node and meets ENOENT — never
    EACCES — on the other seven (round-3 review: the guard's foreign nodes on an 8-GPU box)."""
    exe = str(tmp_path / "drm_enum")
    subprocess.run(["gcc", "-O1", "-o", exe, os.path.join(os.path.dirname(__file__), "fixtures", "drm_enum.c")],
                   check=True, timeout=60)
    keep = f"{fake_dev}/dri/renderD133"
    env = dict(os.environ, LD_PRELOAD=DEVVIEW_LIB, AMDKUBE_DEVVIEW_ROOT=fake_dev,
               AMDKUBE_DEVVIEW_ALLOW=f"{keep},{fake_dev}/kfd")
    p = subprocess.run([NSEXEC, "--no-namespaces", "--landlock", "--dev-root", fake_dev, "--keep", keep, "--", exe, fake_dev],
                       capture_output=True, text=True, timeout=30, env=env)
    assert p.returncode == 0, p.stderr
    r = json.loads(p.stdout)
    assert r["readdir"] == ["by-path", "renderD133"], r["readdir"]
    assert r["scandir"] == ["by-path", "renderD133"], r["scandir"]
    assert r["glob"] == ["renderD133"], r["glob"]
    for minor in range(128, 136):
        probes = r["probe"][f"renderD{minor}"]
        want = "ok" if minor == 133 else "No such file or directory"
        assert set(probes.values()) == {want}, (minor, probes)
    # the same walk without the preload: the kernel's refusal shows (what ROCr would fail on)
    p = subprocess.run([NSEXEC, "--no-namespaces", "--landlock", "--dev-root", fake_dev, "--keep", keep, "--", exe, fake_dev],
                       capture_output=True, text=True, timeout=30)
    r = json.loads(p.stdout)
    assert r["probe"]["renderD128"]["open"] == "Permission denied"
    assert len(r["readdir"]) == 17
