"""Run an image's program without a mount namespace (the unprivileged MI355X node has no user
namespaces and no CAP_SYS_ADMIN, so it cannot pivot_root into the image).

The program, its interpreter (`#!` line or the ELF PT_INTERP dynamic loader) and its shared
libraries all come from the image's root filesystem: a dynamic executable is started as
`<rootfs>/<PT_INTERP> --library-path <rootfs library dirs> <rootfs>/<program> args…`, so the
image's own loader and libc run it, as they would under a chroot. The paths the program opens
at run time are moved under the image by the rootview preload (native/rootview.c, armed by
`rootview_env`): /etc/… is the image's, volumes appear at their mount paths, /tmp is the
container's own, /dev, /proc and /sys stay the host's, and programs the workload execs run
through the image's loader too. Images without a glibc loader (musl, static) cannot take a
glibc preload and keep the host view. Namespace-capable nodes (isolation=namespaces|userns)
pivot_root into the image instead (native/nsexec.cpp --rootfs).
"""
from __future__ import annotations

import os
import struct

ROOTVIEW_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native", "lib",
                            "libamdkube-rootview.so")
GLIBC_LOADERS = ("/lib64/ld-linux-x86-64.so.2", "/lib/x86_64-linux-gnu/ld-linux-x86-64.so.2",
                 "/usr/lib64/ld-linux-x86-64.so.2", "/usr/lib/x86_64-linux-gnu/ld-linux-x86-64.so.2")
LIB_DIRS = ("lib/x86_64-linux-gnu", "usr/lib/x86_64-linux-gnu", "lib64", "usr/lib64", "lib", "usr/lib",
            "usr/local/lib")
PT_INTERP = 3


class RootfsExecError(OSError):
    pass


def _inside(root: str, p: str) -> str:
    """Host path of container path `p` (absolute inside the image); symlinks are resolved
    inside the image (an absolute link target is relative to the image root)."""
    root = os.path.realpath(root)
    parts = [x for x in p.split("/") if x and x != "."]
    cur = root
    hops = 0
    while parts:
        part = parts.pop(0)
        if part == "..":
            cur = os.path.dirname(cur) if cur != root else root
            continue
        nxt = os.path.join(cur, part)
        if os.path.islink(nxt):
            hops += 1
            if hops > 40:
                raise RootfsExecError(f"too many symlinks resolving {p}")
            tgt = os.readlink(nxt)
            parts = [x for x in tgt.split("/") if x and x != "."] + parts
            cur = root if tgt.startswith("/") else cur
            continue
        cur = nxt
    return cur


def elf_interp(path: str) -> str | None:
    """PT_INTERP of an ELF64 executable (None for a static binary); ValueError if not ELF."""
    with open(path, "rb") as f:
        head = f.read(64)
        if head[:4] != b"\x7fELF":
            raise ValueError("not an ELF file")
        if head[4] != 2:
            raise ValueError("only ELF64 images are supported")
        end = "<" if head[5] == 1 else ">"
        phoff, = struct.unpack(end + "Q", head[32:40])
        phentsize, phnum = struct.unpack(end + "HH", head[54:58])
        for i in range(phnum):
            f.seek(phoff + i * phentsize)
            ph = f.read(phentsize)
            ptype, = struct.unpack(end + "I", ph[:4])
            if ptype == PT_INTERP:
                off, = struct.unpack(end + "Q", ph[8:16])
                size, = struct.unpack(end + "Q", ph[32:40])
                f.seek(off)
                return f.read(size).rstrip(b"\x00").decode()
    return None


def library_dirs(root: str) -> list[str]:
    out = []
    for d in LIB_DIRS:
        p = _inside(root, "/" + d)
        if os.path.isdir(p) and p not in out:
            out.append(p)
    conf = _inside(root, "/etc/ld.so.conf.d")
    if os.path.isdir(conf):
        for fn in sorted(os.listdir(conf)):
            try:
                with open(os.path.join(conf, fn)) as f:
                    for line in f:
                        line = line.split("#", 1)[0].strip()
                        if line.startswith("/") and os.path.isdir(_inside(root, line)):
                            p = _inside(root, line)
                            if p not in out:
                                out.append(p)
            except OSError:
                pass
    return out


def resolve_program(root: str, prog: str, path_env: str, workdir: str = "/") -> str:
    if "/" in prog:
        host = _inside(root, prog if prog.startswith("/") else os.path.join(workdir, prog))
        if os.path.isfile(host):
            return host
        raise RootfsExecError(f"{prog}: not found in the image")
    for d in (path_env or "").split(":"):
        if d.startswith("/"):
            host = _inside(root, os.path.join(d, prog))
            if os.path.isfile(host) and os.access(host, os.X_OK):
                return host
    raise RootfsExecError(f"{prog}: executable file not found in the image's $PATH")


def rootfs_argv(root: str, argv: list[str], path_env: str, workdir: str = "/", depth: int = 0) -> list[str]:
    """Host argv that runs container argv `argv` from image root `root`."""
    if not argv:
        raise RootfsExecError("no command")
    if depth > 4:
        raise RootfsExecError("interpreter chain too deep")
    prog = resolve_program(root, argv[0], path_env, workdir)
    with open(prog, "rb") as f:
        head = f.read(256)
    if head.startswith(b"#!"):
        line = head[2:].split(b"\n", 1)[0].decode().strip().split(None, 1)
        interp = [line[0]] + ([line[1]] if len(line) > 1 else [])
        # the interpreter is the image's; the script it reads is passed by its host path
        return rootfs_argv(root, interp + [prog] + list(argv[1:]), path_env, workdir, depth + 1)
    interp = elf_interp(prog)
    if interp is None:
        return [prog] + list(argv[1:])
    ld = _inside(root, interp)
    if not os.path.isfile(ld):
        raise RootfsExecError(f"{argv[0]}: the image has no dynamic loader {interp}")
    return [ld, "--library-path", ":".join(library_dirs(root)), prog] + list(argv[1:])



def rootview_env(root: str, mounts: list[dict], scratch: str, passthrough: tuple[str, ...] = (),
                 env: dict | None = None, workdir: str = "/") -> dict:
    """Environment that arms the rootview preload for a container of image root `root`:
    `mounts` ({container_path, host_path}) keep their paths, `passthrough` host paths (the rocm
    handler's /opt/rocm) stay visible at the same path, /tmp is `scratch`/tmp, and writes to the
    image's files land in `scratch`/upper (copied up first), so the shared image stays as pulled.
    {} when the image has no glibc loader or the preload is not built."""
    if not os.path.exists(ROOTVIEW_LIB) or not any(os.path.isfile(_inside(root, ld)) for ld in GLIBC_LOADERS):
        return {}
    tmp, upper = os.path.join(scratch, "tmp"), os.path.join(scratch, "upper")
    os.makedirs(tmp, exist_ok=True)
    os.chmod(tmp, 0o1777)
    os.makedirs(upper, exist_ok=True)
    taken = {m["container_path"].rstrip("/") or "/" for m in mounts}
    table = [f"{m['container_path']}={m['host_path']}" for m in mounts
             if m["container_path"].startswith("/") and "\n" not in m["container_path"] + m["host_path"]]
    table += [f"{h}={h}" for h in passthrough if os.path.exists(h) and h not in taken]
    if "/tmp" not in taken:
        table.append(f"/tmp={tmp}")
    pre = (env or {}).get("LD_PRELOAD", "")
    return {"AMDKUBE_ROOTVIEW": os.path.realpath(root), "AMDKUBE_ROOTVIEW_UPPER": os.path.realpath(upper),
            "AMDKUBE_ROOTVIEW_MOUNTS": "\n".join(table),
            "AMDKUBE_ROOTVIEW_LIBPATH": ":".join(library_dirs(root)),
            "LD_PRELOAD": ROOTVIEW_LIB + (":" + pre if pre else ""),
            "PWD": workdir or "/"}          # shells trust $PWD for their logical cwd
