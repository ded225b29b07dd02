"""Build every native artefact in-tree (so it travels to the GPU box with the snapshot).

  python native/build.py            # CPU-side pybind modules + pause (g++), HIP targets (hipcc, gfx950)
  python native/build.py --cpu-only # just the g++ targets (used by the CPU test tier)
  python native/build.py --sanitize # also the ASan/UBSan host builds (pause, topo self-test, sampler)
                                    # and the ThreadSanitizer build of the activity sampler

Outputs: amdkube/_native/{_amdsmi,_topo,_kproto,_quantile,_hipops}.<ext> and amdkube/_native/bin/{pause,
amdkube-nsexec,amdkube-logpump,rocm-vector-add,hsa-vector-add,hbm-probe,gpu-burn,xgmi-probe[,topo-selftest-asan,pause-asan,
amdkube-nsexec-asan,amdkube-logpump-asan,
seccomp-check-asan,sampler-selftest-{asan,tsan}]}.
Targets are rebuilt only when a source/header is newer than the output.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "amdkube", "_native")
BIN = os.path.join(OUT, "bin")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes():
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _hipcc():
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else shutil.which("hipcc")


def targets(sanitize=False, cpu_only=False):
    py = _py_includes()
    rocm_inc = [f"-I{ROCM}/include"]
    rpath = [f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib"]
    n = lambda *p: os.path.join(ROOT, *p)  # noqa: E731
    t = [
        (n(OUT, "_topo" + EXT), [n("native/topo_alloc.cpp"), n("native/topo_core.h")],
         ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", *py, n("native/topo_alloc.cpp"), "-o", "{out}"]),
        # the apiserver's JSON <-> protobuf transcoder (plain CPython API)
        (n(OUT, "_kproto" + EXT), [n("native/kproto.cpp")],
         ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-fno-strict-aliasing",
          f"-I{sysconfig.get_paths()['include']}", n("native/kproto.cpp"), "-o", "{out}"]),
        # Prometheus Summary quantile streams (kubelet / device manager / apiserver latencies)
        (n(OUT, "_quantile" + EXT), [n("native/quantile.cpp"), n("native/quantile_core.h")],
         ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", *py, n("native/quantile.cpp"), "-o", "{out}"]),
        (n(OUT, "_amdsmi" + EXT), [n("native/amdsmi_shim.cpp"), n("native/sampler_core.h")],
         ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", *py, *rocm_inc, n("native/amdsmi_shim.cpp"), *rpath,
          "-lamd_smi", "-o", "{out}"]),
        (n(OUT, "lib", "libamdkube-devview.so"), [n("native/devview.c")],
         ["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-fno-delete-null-pointer-checks", n("native/devview.c"), "-o",
          "{out}", "-ldl"]),
        (n(OUT, "lib", "libamdkube-rootview.so"), [n("native/rootview.c")],
         ["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-Wno-nonnull-compare", "-Wno-format-truncation",
          "-fno-delete-null-pointer-checks", n("native/rootview.c"), "-o", "{out}", "-ldl"]),
        (n(BIN, "pause"), [n("native/pause.cpp")],
         ["g++", "-O2", "-std=c++17", n("native/pause.cpp"), "-o", "{out}"]),
        (n(BIN, "amdkube-nsexec"), [n("native/nsexec.cpp"), n("native/seccomp_bpf.h"), n("native/devguard.h"), SYSCALL_TABLE],
         ["g++", "-O2", "-std=c++17", n("native/nsexec.cpp"), "-o", "{out}"]),
        (n(BIN, "seccomp-check"), [n("native/seccomp_check.cpp"), n("native/seccomp_bpf.h"), SYSCALL_TABLE],
         ["g++", "-O2", "-std=c++17", n("native/seccomp_check.cpp"), "-o", "{out}"]),
        (n(BIN, "amdkube-logpump"), [n("native/logpump.cpp")],
         ["g++", "-O2", "-std=c++17", "-Wall", n("native/logpump.cpp"), "-o", "{out}"]),
        (n(BIN, "cni", "amdkube-cni"), [n("native/cni_ipam.cpp")],
         ["g++", "-O2", "-std=c++17", n("native/cni_ipam.cpp"), "-o", "{out}"]),
        (n(BIN, "cni", "amdkube-bridge"), [n("native/cni_bridge.cpp")],
         ["g++", "-O2", "-std=c++17", "-Wall", n("native/cni_bridge.cpp"), "-o", "{out}"]),
    ]
    if sanitize:
        san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
        t += [
            (n(BIN, "topo-selftest-asan"), [n("native/topo_selftest.cpp"), n("native/topo_core.h")],
             ["g++", "-O1", "-std=c++17", *san, n("native/topo_selftest.cpp"), "-o", "{out}"]),
            (n(BIN, "quantile-selftest-asan"), [n("native/quantile_selftest.cpp"), n("native/quantile_core.h")],
             ["g++", "-O1", "-std=c++17", *san, n("native/quantile_selftest.cpp"), "-o", "{out}"]),
            (n(BIN, "pause-asan"), [n("native/pause.cpp")],
             ["g++", "-O1", "-std=c++17", *san, n("native/pause.cpp"), "-o", "{out}"]),
            (n(BIN, "sampler-selftest-asan"), [n("native/sampler_selftest.cpp"), n("native/sampler_core.h")],
             ["g++", "-O1", "-std=c++17", *san, n("native/sampler_selftest.cpp"), "-pthread", "-o", "{out}"]),
            # the container launcher and the seccomp compiler: host code that parses untrusted input
            # (profiles, mountinfo, flags) and changes privileges
            (n(BIN, "amdkube-nsexec-asan"), [n("native/nsexec.cpp"), n("native/seccomp_bpf.h"), n("native/devguard.h"),
                                             SYSCALL_TABLE],
             ["g++", "-O1", "-std=c++17", *san, n("native/nsexec.cpp"), "-o", "{out}"]),
            (n(BIN, "amdkube-logpump-asan"), [n("native/logpump.cpp")],
             ["g++", "-O1", "-std=c++17", *san, n("native/logpump.cpp"), "-o", "{out}"]),
            (n(BIN, "seccomp-check-asan"), [n("native/seccomp_check.cpp"), n("native/seccomp_bpf.h"), SYSCALL_TABLE],
             ["g++", "-O1", "-std=c++17", *san, n("native/seccomp_check.cpp"), "-o", "{out}"]),
            (n(BIN, "sampler-selftest-tsan"), [n("native/sampler_selftest.cpp"), n("native/sampler_core.h")],
             ["g++", "-O1", "-std=c++17", "-fsanitize=thread", "-fno-omit-frame-pointer", "-g",
              n("native/sampler_selftest.cpp"), "-pthread", "-o", "{out}"]),
        ]
    if not cpu_only:
        hip = _hipcc()
        if hip is None:
            raise SystemExit("hipcc not found: cannot build gfx950 targets")
        ho = [hip, f"--offload-arch={ARCH}", "-O3", "-std=c++17"]
        hdr = n("kernels/gpu_common.h")
        t += [
            (n(OUT, "_hipops" + EXT), [n("native/hipops.hip"), hdr],
             [*ho, "-shared", "-fPIC", *py, n("native/hipops.hip"), "-o", "{out}"]),
            (n(BIN, "rocm-vector-add"), [n("kernels/vector_add.hip"), hdr], [*ho, n("kernels/vector_add.hip"), "-o", "{out}"]),
            # the HIP-free pod workload: a bare gfx950 code object, then the HSA host embedding it
            (n(BIN, "hsa-vector-add"), [n("kernels/hsa_vector_add.cpp"), n("kernels/vadd_kernel.hip")],
             ["sh", "-c", f'"$0" --offload-arch={ARCH} -O3 --offload-device-only --no-gpu-bundle-output -c '
              f'{n("kernels/vadd_kernel.hip")} -o {n(OUT, "lib", "vadd_" + ARCH + ".co")} && '
              f'g++ -O2 -std=c++17 -Wall -DVADD_CO_PATH=\\"{n(OUT, "lib", "vadd_" + ARCH + ".co")}\\" '
              f'-I{ROCM}/include {n("kernels/hsa_vector_add.cpp")} -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lhsa-runtime64 -o "$1"',
              hip, "{out}"]),
            (n(BIN, "hbm-probe"), [n("kernels/hbm_probe.hip"), hdr], [*ho, n("kernels/hbm_probe.hip"), "-o", "{out}"]),
            (n(BIN, "gpu-burn"), [n("kernels/gpu_burn.hip"), hdr], [*ho, n("kernels/gpu_burn.hip"), "-o", "{out}"]),
            (n(BIN, "xgmi-probe"), [n("kernels/xgmi_probe.cpp")],
             [*ho, "-x", "hip", n("kernels/xgmi_probe.cpp"), *rocm_inc, *rpath, "-lrccl", "-o", "{out}"]),
        ]
    return t


SYSCALL_TABLE = os.path.join(ROOT, "native", "syscall_table_gen.h")
UNISTD = "/usr/include/x86_64-linux-gnu/asm/unistd_64.h"


def gen_syscall_table():
    """name → number table for the seccomp compiler, from the kernel UAPI header (x86_64)."""
    import re
    src = UNISTD if os.path.exists(UNISTD) else "/usr/include/asm/unistd_64.h"
    if os.path.exists(SYSCALL_TABLE) and os.path.getmtime(SYSCALL_TABLE) >= os.path.getmtime(src) \
            and os.path.getmtime(SYSCALL_TABLE) >= os.path.getmtime(__file__):
        return
    rows = sorted((m.group(1), int(m.group(2))) for m in re.finditer(r"#define __NR_(\w+)\s+(\d+)", open(src).read()))
    body = ",\n".join(f'    {{"{n}", {v}}}' for n, v in rows)
    with open(SYSCALL_TABLE + ".tmp", "w") as f:
        f.write(f"// generated by native/build.py from {src}; do not edit\n#pragma once\n#include <cstring>\n\n"
                "namespace amdkube_seccomp {\nstruct SyscallName { const char* name; int nr; };\n"
                f"static const SyscallName kSyscalls[] = {{\n{body}\n}};\n"
                "inline int syscall_number(const char* name) {\n"
                "  size_t lo = 0, hi = sizeof(kSyscalls) / sizeof(kSyscalls[0]);\n"
                "  while (lo < hi) {\n    size_t mid = (lo + hi) / 2;\n    int c = std::strcmp(kSyscalls[mid].name, name);\n"
                "    if (c == 0) return kSyscalls[mid].nr;\n    if (c < 0) lo = mid + 1; else hi = mid;\n  }\n  return -1;\n}\n"
                "}  // namespace amdkube_seccomp\n")
    os.replace(SYSCALL_TABLE + ".tmp", SYSCALL_TABLE)


def stale(out, deps):
    if not os.path.exists(out):
        return True
    mt = os.path.getmtime(out)
    return any(os.path.getmtime(d) > mt for d in deps)


def build(sanitize=False, cpu_only=False, force=False, jobs=4, verbose=False):
    os.makedirs(os.path.join(BIN, "cni"), exist_ok=True)
    os.makedirs(os.path.join(OUT, "lib"), exist_ok=True)
    gen_syscall_table()
    init = os.path.join(OUT, "__init__.py")
    if not os.path.exists(init):
        open(init, "w").write('"""Built native artefacts (see native/build.py)."""\n')
    todo = [(o, d, c) for o, d, c in targets(sanitize, cpu_only) if force or stale(o, d)]

    def one(item):
        out, _, cmd = item
        cmd = [c.replace("{out}", out + ".tmp") for c in cmd]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"build of {os.path.basename(out)} failed:\n{r.stderr[-4000:]}")
        os.replace(out + ".tmp", out)
        return os.path.basename(out)

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        built = list(ex.map(one, todo))
    return built


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sanitize", action="store_true")
    ap.add_argument("--cpu-only", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=4)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    built = build(a.sanitize, a.cpu_only, a.force, a.j, a.v)
    print("built:", ", ".join(built) if built else "(up to date)")


if __name__ == "__main__":
    sys.exit(main())
