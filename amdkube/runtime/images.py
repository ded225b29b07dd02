"""Local image store for rocshim (CRI ImageService backend).

There is no registry access on the target machines, so an "image" is a named, versioned
entrypoint: a native binary, a script, or a directory with a `run` file. Built-in images
map the e2e workloads to amdkube's gfx950 binaries (the reference's cuda-vector-add image,
test/images/cuda-vector-add, becomes `rocm/vector-add`). Extra images are registered from
`images.json` in the runtime's state dir or via PullImage of a local path (`file:///...`).
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys

NATIVE_BIN = os.path.join(os.path.dirname(os.path.dirname(__file__)), "_native", "bin")


def _b(name):
    return os.path.join(NATIVE_BIN, name)


def builtin_images() -> dict[str, dict]:
    py = sys.executable
    sh = shutil.which("sh") or "/bin/sh"
    return {
        "amdkube/pause:3.1": {"entrypoint": [_b("pause")]},
        "rocm/vector-add:latest": {"entrypoint": [_b("rocm-vector-add")]},
        "amdkube/rocm-vector-add:latest": {"entrypoint": [_b("rocm-vector-add")]},
        "amdkube/hbm-probe:latest": {"entrypoint": [_b("hbm-probe")]},
        "amdkube/gpu-burn:latest": {"entrypoint": [_b("gpu-burn")]},
        "amdkube/xgmi-probe:latest": {"entrypoint": [_b("xgmi-probe")]},
        "busybox:latest": {"entrypoint": [sh]},
        "python:3": {"entrypoint": [py]},
        "amdkube/amdkube:latest": {"entrypoint": [py, "-m", "amdkube"]},
        "nginx:latest": {"entrypoint": [py, "-m", "http.server", "--bind", "127.0.0.1"], "cmd": ["8080"]},
        "k8s.gcr.io/pause:3.1": {"entrypoint": [_b("pause")]},
    }


def normalize(ref: str) -> str:
    ref = ref.strip()
    if ref.startswith("docker.io/"):
        ref = ref[len("docker.io/"):]
    if ref.startswith("library/"):
        ref = ref[len("library/"):]
    if "@" in ref:
        return ref
    last = ref.rsplit("/", 1)[-1]
    return ref if ":" in last else ref + ":latest"


class ImageStore:
    def __init__(self, state_dir: str):
        self.path = os.path.join(state_dir, "images.json")
        self.images = builtin_images()
        if os.path.exists(self.path):
            with open(self.path) as f:
                self.images.update(json.load(f))

    def _save(self):
        extra = {k: v for k, v in self.images.items() if k not in builtin_images()}
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(extra, f)
        os.replace(tmp, self.path)

    def resolve(self, ref: str) -> tuple[str, dict] | None:
        n = normalize(ref)
        if n in self.images:
            return n, self.images[n]
        return None

    def image_id(self, name: str) -> str:
        return "sha256:" + hashlib.sha256(json.dumps(self.images[name], sort_keys=True).encode()).hexdigest()

    def pull(self, ref: str) -> str:
        if self.resolve(ref):
            return self.image_id(self.resolve(ref)[0])
        path = ref[len("file://"):] if ref.startswith("file://") else ref
        if os.path.isabs(path) and os.path.exists(path):
            entry = os.path.join(path, "run") if os.path.isdir(path) else path
            self.images[normalize(ref)] = {"entrypoint": [entry], "workdir": path if os.path.isdir(path) else ""}
            self._save()
            return self.image_id(normalize(ref))
        raise KeyError(f"image {ref!r} not found (no registry access; register it in images.json or pull a local path)")

    def remove(self, ref: str):
        n = normalize(ref)
        if n in self.images and n not in builtin_images():
            del self.images[n]
            self._save()

    def list(self):
        return [(n, self.image_id(n), spec) for n, spec in self.images.items()]
