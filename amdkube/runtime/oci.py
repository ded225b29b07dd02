"""Container images with real root filesystems: import of docker-archive (`docker save`) and
OCI image-layout archives, layer unpack with whiteouts, and the image config.

Reference: dockerService.PullImage (pkg/kubelet/dockershim/docker_image.go:73) hands the pull to
dockerd, and CreateContainer inspects the image and builds the container from it
(docker_container.go:88-172): the image's Entrypoint/Cmd/Env/WorkingDir/User apply unless the
container overrides them (kuberuntime_container.go generateContainerConfig). There is no
registry access on an MI355X node here, so images arrive as local archives (`file://…`).

Layout on disk (rocshim state dir):

  images/layers/<diff id>/            one unpacked layer (kept for accounting and re-use)
  images/<image id>/rootfs/            the merged root filesystem (layers applied in order)
  images/<image id>/config.json        the image config

Whiteouts (OCI image spec, "Representing Changes"): `.wh.<name>` deletes <name> from the layers
below; `.wh..wh..opq` in a directory hides everything the lower layers put there. A layer is
applied by first processing its whiteouts against the lower content, then extracting its other
entries. Extraction refuses any entry whose resolved path leaves the root (tarfile's "tar"
filter, with symlinked parents followed) and skips device nodes (the runtime supplies /dev).
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import re
import shutil
import tarfile
import tempfile

WHITEOUT = ".wh."
OPAQUE = ".wh..wh..opq"


class ImageFormatError(ValueError):
    pass


_DIGEST_LEN = {"sha256": 64, "sha512": 128}    # the OCI image-spec's registered digest algorithms


def _hash_file(path: str, algo: str) -> str:
    h = hashlib.new(algo)
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def _sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def _diff_id(layer: str) -> str:
    with open(layer, "rb") as f:
        gz = f.read(2) == b"\x1f\x8b"
    if not gz:
        return _sha256_file(layer)
    import gzip
    h = hashlib.sha256()
    with gzip.open(layer, "rb") as g:
        for chunk in iter(lambda: g.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def _norm(name: str) -> str:
    """Entry name inside the root: no leading ./ or /, no '..' (refused by the caller)."""
    n = os.path.normpath(name.lstrip("/"))
    return "" if n == "." else n


def _remove(path: str):
    if os.path.islink(path) or not os.path.isdir(path):
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
    else:
        shutil.rmtree(path, ignore_errors=True)


def _inside(root: str, path: str) -> bool:
    real = os.path.realpath(path)
    return real == root or real.startswith(root + os.sep)


def apply_layer(tar_path: str, root: str) -> dict:
    """Apply one layer tar (plain or gzip) onto `root`. Returns counts for the record."""
    root = os.path.realpath(root)
    os.makedirs(root, exist_ok=True)
    stats = {"files": 0, "whiteouts": 0, "opaque": 0, "skipped": 0}
    with tarfile.open(tar_path, "r:*") as tf:
        members = tf.getmembers()
        keep = []
        for mb in members:
            name = _norm(mb.name)
            if not name or name.startswith("..") or "/../" in f"/{name}/":
                raise ImageFormatError(f"layer entry {mb.name!r} leaves the root")
            base, parent = os.path.basename(name), os.path.dirname(name)
            if base == OPAQUE:
                d = os.path.realpath(os.path.join(root, parent))
                if _inside(root, d) and os.path.isdir(d):
                    for child in os.listdir(d):
                        _remove(os.path.join(d, child))
                stats["opaque"] += 1
                continue
            if base.startswith(WHITEOUT):
                hidden = base[len(WHITEOUT):]
                if hidden in ("", ".", ".."):
                    raise ImageFormatError(f"layer entry {mb.name!r}: whiteout of {hidden!r}")
                victim = os.path.join(root, parent, hidden)
                # the directory must resolve inside the root; the victim itself is removed as a
                # name (a symlink victim is unlinked, never followed)
                if _inside(root, os.path.dirname(victim)):
                    _remove(os.path.join(os.path.realpath(os.path.dirname(victim)), hidden))
                stats["whiteouts"] += 1
                continue
            if mb.ischr() or mb.isblk():
                stats["skipped"] += 1
                continue
            if mb.islnk():     # a hard link must name a file of this image, never one outside it
                src = _norm(mb.linkname)
                if not src or src.startswith("..") or not _inside(root, os.path.join(root, src)):
                    raise ImageFormatError(f"layer entry {mb.name!r}: hard link to {mb.linkname!r} leaves the root")
                mb.linkname = src
            mb.name = name
            keep.append(mb)
        for mb in keep:
            # run the filter first: it refuses an entry whose symlinked parents resolve outside
            # the root, before anything on disk is touched for it
            try:
                _layer_filter(mb, root)
            except tarfile.FilterError as e:
                raise ImageFormatError(f"layer entry {mb.name!r}: {e}") from e
            # a later layer may replace a directory with a file or a link with a directory: the
            # old entry is removed by its final name under its parent resolved inside the root
            parent = os.path.realpath(os.path.join(root, os.path.dirname(mb.name)))
            if not _inside(root, parent):
                raise ImageFormatError(f"layer entry {mb.name!r}: parent resolves outside the root")
            target = os.path.join(parent, os.path.basename(mb.name))
            if os.path.lexists(target) and not (mb.isdir() and os.path.isdir(target) and not os.path.islink(target)):
                _remove(target)
            try:
                tf.extract(mb, root, set_attrs=True, filter=_layer_filter)
            except tarfile.FilterError as e:
                raise ImageFormatError(f"layer entry {mb.name!r}: {e}") from e
            stats["files"] += 1
    return stats


def _layer_filter(member: tarfile.TarInfo, dest: str) -> tarfile.TarInfo:
    """tarfile's "tar" filter (no absolute names, nothing resolved outside dest — symlinked
    parents included), keeping the permission bits images rely on except set-id bits."""
    return tarfile.tar_filter(member, dest)


def _read_json(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def read_archive(path: str, work: str) -> tuple[dict, list[str], list[str]]:
    """(image config, [layer tar paths in order], [repo tags]) of a docker-archive or an OCI
    image layout — a directory or a tar of one. Archives are unpacked into `work`."""
    if os.path.isdir(path):
        src = path
    else:
        src = os.path.join(work, "archive")
        os.makedirs(src)
        with tarfile.open(path, "r:*") as tf:
            tf.extractall(src, filter="data")
    src = os.path.realpath(src)

    def member(rel) -> str:
        """A file named by the archive's own metadata: it must resolve inside the archive."""
        p = os.path.join(src, str(rel))
        if os.path.isabs(str(rel)) or not _inside(src, p):
            raise ImageFormatError(f"archive path {rel!r} leaves the archive")
        return p
    if os.path.exists(os.path.join(src, "manifest.json")):          # docker save
        man = _read_json(os.path.join(src, "manifest.json"))
        if not isinstance(man, list) or not man:
            raise ImageFormatError("manifest.json: expected a non-empty list")
        m0 = man[0]
        cfg = _read_json(member(m0["Config"]))
        layers = [member(lp) for lp in m0.get("Layers") or []]
        tags = list(m0.get("RepoTags") or [])
    elif os.path.exists(os.path.join(src, "index.json")):           # OCI image layout
        idx = _read_json(os.path.join(src, "index.json"))
        mans = idx.get("manifests") or []
        if not mans:
            raise ImageFormatError("index.json lists no manifest")

        def blob(digest):
            algo, _, hexd = str(digest).partition(":")
            if algo not in _DIGEST_LEN or not re.fullmatch(f"[0-9a-f]{{{_DIGEST_LEN[algo]}}}", hexd):
                raise ImageFormatError(f"unsupported or malformed digest {digest!r}")
            p = member(os.path.join("blobs", algo, hexd))
            if not os.path.exists(p):
                raise ImageFormatError(f"missing blob {digest}")
            if _hash_file(p, algo) != hexd:
                raise ImageFormatError(f"blob {digest} does not match its digest")
            return p
        m = _read_json(blob(mans[0]["digest"]))
        if m.get("manifests"):        # an index nested in the index: take its first manifest
            m = _read_json(blob(m["manifests"][0]["digest"]))
        cfg = _read_json(blob(m["config"]["digest"]))
        layers = [blob(layer["digest"]) for layer in m.get("layers") or []]
        ann = mans[0].get("annotations") or {}
        tags = [ann["org.opencontainers.image.ref.name"]] if ann.get("org.opencontainers.image.ref.name") else []
    else:
        raise ImageFormatError("neither a docker archive (manifest.json) nor an OCI layout (index.json)")
    for lp in layers:
        if not os.path.exists(lp):
            raise ImageFormatError(f"missing layer {lp}")
    return cfg, layers, tags


def image_spec(cfg: dict) -> dict:
    """The parts of an image config a container is built from (docker_container.go:88-172)."""
    c = cfg.get("config") or cfg.get("Config") or {}
    env = {}
    for kv in c.get("Env") or []:
        k, _, v = kv.partition("=")
        env[k] = v
    return {"entrypoint": list(c.get("Entrypoint") or []), "cmd": list(c.get("Cmd") or []), "env": env,
            "workdir": c.get("WorkingDir") or "/", "user": c.get("User") or "",
            "diff_ids": list((cfg.get("rootfs") or {}).get("diff_ids") or [])}


def import_image(path: str, store_root: str) -> dict:
    """Unpack an archive into `<store_root>/<id>/rootfs`; returns the image record."""
    os.makedirs(store_root, exist_ok=True)
    with tempfile.TemporaryDirectory(dir=store_root, prefix=".import-") as work:
        cfg, layers, tags = read_archive(path, work)
        return import_layers(cfg, layers, tags, store_root)


def import_layers(cfg: dict, layers: list[str], tags: list[str], store_root: str) -> dict:
    """Apply layer files (plain or gzip tars, in order) into `<store_root>/<id>/rootfs`, checking
    each against the config's rootfs.diff_ids; returns the image record. Shared by archive
    imports and registry pulls (runtime/registry.py)."""
    os.makedirs(store_root, exist_ok=True)
    layers_root = os.path.join(store_root, "layers")
    os.makedirs(layers_root, exist_ok=True)
    spec = image_spec(cfg)
    cfg_bytes = json.dumps(cfg, sort_keys=True).encode()
    iid = hashlib.sha256(cfg_bytes).hexdigest()
    dest = os.path.join(store_root, iid)
    shutil.rmtree(dest, ignore_errors=True)
    rootfs = os.path.join(dest, "rootfs")
    os.makedirs(rootfs)
    diff_ids, sizes = [], []
    for i, lp in enumerate(layers):
        did = "sha256:" + _diff_id(lp)    # digest of the uncompressed layer
        if spec["diff_ids"] and i < len(spec["diff_ids"]) and spec["diff_ids"][i] != did:
            raise ImageFormatError(f"layer {i}: diff id {did} does not match the config's {spec['diff_ids'][i]}")
        apply_layer(lp, rootfs)
        diff_ids.append(did)
        sizes.append(os.path.getsize(lp))
        # keep the layer blob by diff id (shared by images built on it)
        keep = os.path.join(layers_root, did.split(":", 1)[1] + ".tar")
        if not os.path.exists(keep):
            shutil.copyfile(lp, keep)
    if spec["diff_ids"] and len(spec["diff_ids"]) != len(layers):
        raise ImageFormatError(f"the config lists {len(spec['diff_ids'])} layers, the manifest {len(layers)}")
    with open(os.path.join(dest, "config.json"), "wb") as f:
        f.write(cfg_bytes)
    return {"kind": "rootfs", "id": "sha256:" + iid, "rootfs": rootfs, "blob": dest, "layers": diff_ids,
            "layer_sizes": sizes, "repo_tags": tags, "entrypoint": spec["entrypoint"], "cmd": spec["cmd"],
            "env": spec["env"], "workdir": spec["workdir"], "user": spec["user"]}


# ------------------------------------------------------------------------- archive writer
def _tar_bytes(entries: list[tuple[str, bytes | None, int, str | None]]) -> bytes:
    """entries: (name, data or None for a directory, mode, symlink target or None)."""
    bio = io.BytesIO()
    with tarfile.open(fileobj=bio, mode="w") as tf:
        for name, data, mode, link in entries:
            ti = tarfile.TarInfo(name)
            ti.mode = mode
            if link is not None:
                ti.type, ti.linkname = tarfile.SYMTYPE, link
                tf.addfile(ti)
            elif data is None:
                ti.type = tarfile.DIRTYPE
                tf.addfile(ti)
            else:
                ti.size = len(data)
                tf.addfile(ti, io.BytesIO(data))
    return bio.getvalue()


def write_docker_archive(path: str, layers: list[list[tuple]], config: dict, tags: list[str]):
    """Build a `docker save`-format archive from in-memory layers (tests and image tooling)."""
    with tarfile.open(path, "w") as out:
        names, diff_ids = [], []
        for i, entries in enumerate(layers):
            data = _tar_bytes(entries)
            did = hashlib.sha256(data).hexdigest()
            diff_ids.append("sha256:" + did)
            name = f"{did}/layer.tar"
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            out.addfile(ti, io.BytesIO(data))
            names.append(name)
        cfg = {"architecture": "amd64", "os": "linux", "config": config, "rootfs": {"type": "layers", "diff_ids": diff_ids}}
        cb = json.dumps(cfg).encode()
        cname = hashlib.sha256(cb).hexdigest() + ".json"
        for n, b in ((cname, cb), ("manifest.json", json.dumps([{"Config": cname, "RepoTags": tags, "Layers": names}]).encode())):
            ti = tarfile.TarInfo(n)
            ti.size = len(b)
            out.addfile(ti, io.BytesIO(b))


def layer_from_tree(root: str, prefix: str = "") -> list[tuple]:
    """Entries for a layer holding the files under `root` (placed at `prefix` in the image)."""
    out = []
    for dp, dns, fns in os.walk(root):
        rel = os.path.relpath(dp, root)
        base = os.path.join(prefix, rel) if rel != "." else prefix
        if base:
            out.append((base, None, 0o755, None))
        for fn in sorted(fns):
            p = os.path.join(dp, fn)
            name = os.path.join(base, fn) if base else fn
            if os.path.islink(p):
                out.append((name, b"", 0o777, os.readlink(p)))
            else:
                with open(p, "rb") as f:
                    out.append((name, f.read(), os.stat(p).st_mode & 0o7777, None))
    return out
