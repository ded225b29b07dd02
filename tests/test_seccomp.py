"""Seccomp profiles compiled to BPF by amdkube's native applier (SURVEY §2.3 libseccomp row;
reference annotations seccomp.security.alpha.kubernetes.io/pod and
container.seccomp.security.alpha.kubernetes.io/<name>, pkg/kubelet/kuberuntime/helpers.go
getSeccompProfileFromAnnotations; dockershim applies them through Docker)."""
from __future__ import annotations

import asyncio
import json
import os
import subprocess

import pytest

from amdkube.kubelet.kuberuntime import seccomp_profile
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.runtime.images import NATIVE_BIN

CHECK = os.path.join(NATIVE_BIN, "seccomp-check")
NSEXEC = os.path.join(NATIVE_BIN, "amdkube-nsexec")
ALLOW, KILL_PROCESS, TRAP = 0x7FFF0000, 0x80000000, 0x00030000


def errno(e):
    return 0x00050000 | e


def evaluate(profile_path, call, *args, arch=None):
    argv = [CHECK, str(profile_path), call]
    if arch is not None:
        argv += ["--arch", hex(arch)]
    r = subprocess.run(argv + [str(a) for a in args], capture_output=True, text=True, check=True)
    return int(r.stdout, 16)


def write(tmp_path, prof, name="p.json"):
    p = tmp_path / name
    p.write_text(json.dumps(prof))
    return p


@pytest.mark.parametrize("op,value,cases", [
    ("SCMP_CMP_EQ", 1 << 32, [(1 << 32, True), ((1 << 32) + 1, False), (0, False)]),
    ("SCMP_CMP_NE", 7, [(7, False), (8, True), ((1 << 32) + 7, True)]),
    ("SCMP_CMP_GE", 1 << 32, [((1 << 32) - 1, False), (1 << 32, True), ((1 << 33), True), (5, False)]),
    ("SCMP_CMP_GT", (1 << 32) + 5, [((1 << 32) + 5, False), ((1 << 32) + 6, True), (1 << 40, True), (6, False)]),
    ("SCMP_CMP_LT", (1 << 32) + 5, [((1 << 32) + 4, True), ((1 << 32) + 5, False), (1 << 33, False), (9, True)]),
    ("SCMP_CMP_LE", (1 << 32) + 5, [((1 << 32) + 5, True), ((1 << 32) + 6, False), (0, True), (1 << 34, False)]),
])
def test_argument_comparisons_64bit(tmp_path, op, value, cases):
    p = write(tmp_path, {"defaultAction": "SCMP_ACT_ALLOW",
                         "syscalls": [{"names": ["dup3"], "action": "SCMP_ACT_ERRNO", "errnoRet": 22,
                                       "args": [{"index": 2, "value": value, "op": op}]}]})
    for arg, hit in cases:
        assert evaluate(p, "dup3", 0, 0, arg) == (errno(22) if hit else ALLOW), (op, value, arg)


def test_masked_eq_order_arch_guard_and_actions(tmp_path):
    p = write(tmp_path, {"defaultAction": "SCMP_ACT_ERRNO", "syscalls": [
        {"names": ["ioctl"], "action": "SCMP_ACT_TRAP", "args": [{"index": 1, "value": 0xFF, "valueTwo": 0x54, "op": "SCMP_CMP_MASKED_EQ"}]},
        {"names": ["ioctl", "read", "write", "bogus_syscall_name"], "action": "SCMP_ACT_ALLOW"},
        {"names": ["read"], "action": "SCMP_ACT_KILL_PROCESS"}]})
    assert evaluate(p, "ioctl", 3, 0x1254) == TRAP
    assert evaluate(p, "ioctl", 3, 0x5401) == ALLOW
    assert evaluate(p, "read") == ALLOW                    # first matching rule wins
    assert evaluate(p, "mkdir") == errno(1)                # default action, EPERM
    assert evaluate(p, "read", arch=0x40000003) == KILL_PROCESS   # i386 entry point
    assert evaluate(p, "1073741824") == KILL_PROCESS       # x32 syscall bit
    bad = write(tmp_path, {"defaultAction": "SCMP_ACT_NOPE"}, "bad.json")
    assert subprocess.run([CHECK, str(bad), "read"], capture_output=True).returncode == 1


def test_default_profile_keeps_rocm_syscalls():
    p = os.path.join(os.path.dirname(NSEXEC), "..", "..", "runtime", "seccomp_default.json")
    for call in ("ioctl", "mmap", "mbind", "set_mempolicy", "move_pages", "sched_setaffinity", "clone", "futex"):
        assert evaluate(p, call) == ALLOW, call
    for call in ("mount", "ptrace", "kexec_load", "bpf", "perf_event_open", "unshare", "keyctl"):
        assert evaluate(p, call) == errno(1), call
    assert evaluate(p, "personality", 8) == ALLOW and evaluate(p, "personality", 0x0040000) == errno(1)


def test_nsexec_enforces_profile(tmp_path):
    p = write(tmp_path, {"defaultAction": "SCMP_ACT_ALLOW", "syscalls": [{"names": ["mkdir", "mkdirat"], "action": "SCMP_ACT_ERRNO"}]})
    r = subprocess.run([NSEXEC, "--no-namespaces", "--seccomp", str(p), "--", "sh", "-c", f"mkdir {tmp_path}/x; echo rc=$?"],
                       capture_output=True, text=True)
    assert "rc=1" in r.stdout and "not permitted" in r.stderr and not (tmp_path / "x").exists()
    r = subprocess.run([NSEXEC, "--no-namespaces", "--seccomp", str(tmp_path / "missing.json"), "--", "true"], capture_output=True)
    assert r.returncode == 126


def test_annotation_resolution():
    pod = {"metadata": {"annotations": {"seccomp.security.alpha.kubernetes.io/pod": "docker/default",
                                        "container.seccomp.security.alpha.kubernetes.io/b": "localhost/gpu.json",
                                        "container.seccomp.security.alpha.kubernetes.io/c": "unconfined"}}}
    assert seccomp_profile(pod, "a", "/r") == "runtime/default"
    assert seccomp_profile(pod, "b", "/r") == "localhost//r/gpu.json"
    assert seccomp_profile(pod, "c", "/r") == ""
    assert seccomp_profile({"metadata": {}}, "a") == ""


async def test_pod_with_seccomp_annotations(tmp_path):
    prof = write(tmp_path, {"defaultAction": "SCMP_ACT_ALLOW", "syscalls": [{"names": ["mkdir", "mkdirat"], "action": "SCMP_ACT_ERRNO"}]})
    script = f"mkdir {tmp_path}/d-$HOSTNAME && echo made || echo denied"
    async with LocalCluster(gpus="none", relist_period=0.2) as lc:
        c = lc.client
        for name, ann in (("confined", {"container.seccomp.security.alpha.kubernetes.io/c": f"localhost/{prof}"}),
                          ("free", {}),
                          ("default", {"seccomp.security.alpha.kubernetes.io/pod": "runtime/default"})):
            cmd = script if name != "default" else "unshare -U true && echo unshared || echo denied"
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "annotations": ann},
                            "spec": {"restartPolicy": "Never",
                                     "containers": [{"name": "c", "image": "busybox", "args": ["-c", cmd]}]}}, "default")
        out = {}
        for name in ("confined", "free", "default"):
            await wait_pod(c, "default", name, ("Succeeded", "Failed"), 20)
            out[name] = (await c.logs("default", name)).strip()
        # stdout and stderr are separate streams in the CRI log (their relative order is not kept)
    lines = {k: v.splitlines() for k, v in out.items()}
    assert "denied" in lines["confined"] and lines["free"][-1:] == ["made"] and "denied" in lines["default"], out


def test_seccomp_compiler_under_asan_matches(tmp_path):
    """The profile compiler + BPF evaluator built with ASan/UBSan gives the same verdicts as the
    production build over the default profile (host code under sanitizers)."""
    asan = CHECK + "-asan"
    if not os.path.exists(asan):
        pytest.skip("sanitizer build absent (python native/build.py --sanitize)")
    prof = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amdkube", "runtime",
                        "seccomp_default.json")
    for call, args in (("read", ()), ("ioctl", (3, 0xC0184B01)), ("mount", ()), ("personality", (0,)),
                       ("personality", (0xFFFFFFFF,)), ("clone", (0x10000000,)), ("kexec_load", ())):
        outs = []
        for binary in (CHECK, asan):
            r = subprocess.run([binary, prof, call] + [str(a) for a in args], capture_output=True, text=True,
                               env=dict(os.environ, ASAN_OPTIONS="abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1"))
            assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr
            outs.append(r.stdout.strip())
        assert outs[0] == outs[1], (call, outs)
