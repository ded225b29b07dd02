"""Local image store for rocshim (CRI ImageService backend).

Two kinds of image:
  * rootfs — a real container image: a docker-archive (`docker save`) or OCI image layout,
    pulled from a local path (`file:///…/image.tar` or an OCI directory). Its layers are
    unpacked with whiteouts into a root filesystem and its config (Entrypoint, Cmd, Env,
    WorkingDir, User) builds the container (runtime/oci.py; reference
    pkg/kubelet/dockershim/docker_image.go:73, docker_container.go:88-172);
  * scratch — a named, versioned entrypoint on the host: a native binary, a script, or a
    directory with a `run` file (no registry access on the target machines). Built-in images
map the e2e workloads to amdkube's gfx950 binaries (the reference's cuda-vector-add image,
test/images/cuda-vector-add, becomes `rocm/vector-add`, the HSA build; `rocm/vector-add-hip` is the HIP one). Extra images are registered from
`images.json` in the runtime's state dir or via PullImage of a local path (`file:///...`).

Registry pulls: a reference naming a registry host (`registry.local:5000/rocm/app:1`,
`host.domain/repo@sha256:…`) is pulled over the Docker Registry HTTP API v2 (runtime/registry.py:
token/basic auth with the CRI AuthConfig, manifest lists, digest-verified blobs) and unpacked
like an archive import.

A registry directory (`rocshim --registry-dir`) stands in for remote registries:
`<dir>/<host[:port]>/<repository>/<tag>/` holds an image tree (entrypoint `run`), and an
optional `<dir>/<host[:port]>/auth.json` {"users": {"<name>": "<sha256 hex of password>"}}
makes the registry private: PullImage then needs matching CRI AuthConfig credentials
(username/password or `auth` = base64 "user:password"), which the kubelet takes from the
pod's imagePullSecrets or the node's docker config (kubelet/credentialprovider.py).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
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
        # the GPU-pod workload runs on the bare ROCr runtime (kernels/hsa_vector_add.cpp: 250 ms
        # per pod on MI355X against 320 ms for the HIP build); the HIP build stays available
        "rocm/vector-add:latest": {"entrypoint": [_b("hsa-vector-add")]},
        "amdkube/hsa-vector-add:latest": {"entrypoint": [_b("hsa-vector-add")]},
        "rocm/vector-add-hip:latest": {"entrypoint": [_b("rocm-vector-add")]},
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


def _tree_size(path: str) -> int:
    if os.path.isfile(path):
        return os.path.getsize(path)
    tot = 0
    for dp, _dn, fns in os.walk(path):
        for fn in fns:
            try:
                tot += os.path.getsize(os.path.join(dp, fn))
            except OSError:
                pass
    return tot


class ImageStore:
    """Images pulled from a local path are copied into `<state>/images/<digest>/` (the
    runtime's image filesystem), so they occupy space there, report their size and free it
    when removed (kubelet image GC); built-in images are preloaded and cannot be removed."""

    def __init__(self, state_dir: str, registry_dir: str | None = None, registry_client=None):
        self.registry_dir = registry_dir
        # Docker Registry HTTP API v2 pulls of `host[:port]/repo[:tag|@digest]` (runtime/registry.py)
        if registry_client is None:
            from .registry import RegistryClient
            registry_client = RegistryClient()
        self.registry = registry_client
        self.path = os.path.join(state_dir, "images.json")
        self.blob_root = os.path.join(state_dir, "images")
        os.makedirs(self.blob_root, exist_ok=True)
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
        spec = self.images[name]
        if spec.get("kind") == "rootfs":
            return spec["id"]          # the config digest, as docker reports it
        return "sha256:" + hashlib.sha256(json.dumps(spec, sort_keys=True).encode()).hexdigest()

    @staticmethod
    def is_archive(path: str) -> bool:
        if os.path.isdir(path):
            return any(os.path.exists(os.path.join(path, f)) for f in ("index.json", "manifest.json")) and \
                not os.path.exists(os.path.join(path, "run"))
        import tarfile
        try:
            return os.path.isfile(path) and tarfile.is_tarfile(path)
        except OSError:
            return False

    def _import(self, ref: str, path: str) -> str:
        from .oci import import_image
        rec = import_image(path, self.blob_root)
        rec["size"] = _tree_size(rec["blob"])
        names = [normalize(ref)] + [normalize(t) for t in rec.get("repo_tags") or []]
        for n in names:
            self.images[n] = rec
        self._save()
        return rec["id"]

    def _registry_image(self, ref: str) -> tuple[str, str] | None:
        """(image tree, registry root) of `ref` in the registry directory, or None."""
        if not self.registry_dir or ref.startswith(("file://", "/")):
            return None
        from ..kubelet.credentialprovider import split_image
        host, port, repo = split_image(ref)
        last = ref.split("@", 1)[0].rsplit("/", 1)[-1]
        tag = last.split(":", 1)[1] if ":" in last else "latest"
        reg = os.path.join(self.registry_dir, host + (f":{port}" if port else ""))
        tree = os.path.join(reg, repo, tag)
        return (tree, reg) if os.path.isdir(tree) else None

    @staticmethod
    def _authorized(reg: str, auth: dict | None) -> bool:
        f = os.path.join(reg, "auth.json")
        if not os.path.exists(f):
            return True                                  # public registry
        users = (json.load(open(f)).get("users") or {})
        auth = auth or {}
        user, pw = auth.get("username", ""), auth.get("password", "")
        if not user and auth.get("auth"):
            try:
                user, _, pw = base64.b64decode(auth["auth"]).decode().partition(":")
            except Exception:
                return False
        want = users.get(user)
        return bool(user) and want is not None and hmac.compare_digest(hashlib.sha256(pw.encode()).hexdigest(), want)

    def pull(self, ref: str, auth: dict | None = None) -> str:
        reg = self._registry_image(ref)
        if reg is None and self.registry_dir and not ref.startswith(("file://", "/")):
            from ..kubelet.credentialprovider import split_image
            host, port, _ = split_image(ref)
            if os.path.isdir(os.path.join(self.registry_dir, host + (f":{port}" if port else ""))):
                # a registry the directory stands in for: what it lacks does not exist
                raise KeyError(f"image {ref!r} not found in registry {host}")
        if reg is not None:
            tree, root = reg
            if not self._authorized(root, auth):
                raise PermissionError(f"pull access denied for {ref}: unauthorized: authentication required")
            if self.resolve(ref) is None:
                self._store(normalize(ref), tree)
            return self.image_id(normalize(ref))
        from .registry import is_remote
        if is_remote(ref) and self.registry is not None:
            return self._pull_remote(ref, auth)
        if self.resolve(ref):
            return self.image_id(self.resolve(ref)[0])
        path = ref[len("file://"):] if ref.startswith("file://") else ref
        if os.path.isabs(path) and os.path.exists(path) and self.is_archive(path):
            return self._import(ref, path)
        if os.path.isabs(path) and os.path.exists(path):
            digest = hashlib.sha256(normalize(ref).encode()).hexdigest()[:32]
            blob = os.path.join(self.blob_root, digest)
            shutil.rmtree(blob, ignore_errors=True)
            if os.path.isdir(path):
                shutil.copytree(path, blob, symlinks=True)
                entry, workdir = os.path.join(blob, "run"), blob
            else:
                os.makedirs(blob)
                entry = os.path.join(blob, os.path.basename(path))
                shutil.copy2(path, entry)
                workdir = ""
            self.images[normalize(ref)] = {"entrypoint": [entry], "workdir": workdir, "blob": blob, "size": _tree_size(blob)}
            self._save()
            return self.image_id(normalize(ref))
        raise KeyError(f"image {ref!r} not found (no registry access; register it in images.json or pull a local path)")

    def _pull_remote(self, ref: str, auth: dict | None) -> str:
        """A registry pull. A tag already held is re-checked against the registry's manifest
        digest (dockerd's pull of an existing tag): unchanged, nothing is downloaded."""
        from .registry import parse_reference, pull_image
        name = normalize(ref)
        have = self.images.get(name)
        if have is not None and have.get("repo_digests"):
            host, repo, tag = parse_reference(ref)
            _, digest = self.registry.manifest(host, repo, tag, auth)
            if f"{host}/{repo}@{digest}" in have["repo_digests"]:
                return have["id"]
        rec = pull_image(ref, self.blob_root, auth, self.registry)
        rec["size"] = _tree_size(rec["blob"])
        for n in {name, normalize(rec["repo_digests"][0])}:
            self.images[n] = rec
        self._save()
        return rec["id"]

    def _store(self, name: str, tree: str):
        digest = hashlib.sha256(name.encode()).hexdigest()[:32]
        blob = os.path.join(self.blob_root, digest)
        shutil.rmtree(blob, ignore_errors=True)
        shutil.copytree(tree, blob, symlinks=True)
        self.images[name] = {"entrypoint": [os.path.join(blob, "run")], "workdir": blob, "blob": blob, "size": _tree_size(blob)}
        self._save()

    def remove(self, ref: str):
        n = normalize(ref) if not ref.startswith("sha256:") else next(
            (k for k in self.images if self.image_id(k) == ref), ref)
        if n in self.images and n not in builtin_images():
            spec = self.images[n]
            blob = spec.get("blob")
            # a rootfs image is removed under every tag it was stored as (docker rmi by id)
            for k in [k for k, v in self.images.items() if v is spec or (blob and v.get("blob") == blob)]:
                del self.images[k]
            self._save()
            if blob and blob.startswith(self.blob_root + os.sep):
                shutil.rmtree(blob, ignore_errors=True)
            self._gc_layers()

    def _gc_layers(self):
        """Drop unpacked layer blobs no remaining image references (image GC frees layers)."""
        d = os.path.join(self.blob_root, "layers")
        if not os.path.isdir(d):
            return
        live = {lid.split(":", 1)[-1] for v in self.images.values() for lid in v.get("layers") or ()}
        for f in os.listdir(d):
            if f.endswith(".tar") and f[:-4] not in live:
                try:
                    os.unlink(os.path.join(d, f))
                except OSError:
                    pass

    def layers(self, name: str) -> list[str]:
        return list((self.images.get(name) or {}).get("layers") or [])

    def removable(self, name: str) -> bool:
        return name not in builtin_images()

    def size(self, name: str) -> int:
        spec = self.images.get(name) or {}
        if "size" in spec:
            return int(spec["size"])
        ep = (spec.get("entrypoint") or [""])[0]
        return _tree_size(ep) if ep.startswith(NATIVE_BIN) and os.path.exists(ep) else 0

    def used_bytes(self) -> int:
        return _tree_size(self.blob_root)

    def list(self):
        return [(n, self.image_id(n), spec) for n, spec in self.images.items()]
