"""Real container images: docker-archive / OCI-layout import, layer whiteouts, image config
precedence, image GC of layers, and running an image (path-rooted on an unprivileged node,
pivot_root into an overlay in namespace modes).

Reference: dockershim PullImage (pkg/kubelet/dockershim/docker_image.go:73) and CreateContainer
(docker_container.go:88-172) through dockerd; OCI image spec layer changesets (whiteouts)."""
import asyncio
import gzip
import hashlib
import io
import json
import os
import shutil
import subprocess
import tarfile
import tempfile

import pytest

from amdkube.grpcdesc.cri import CRI as C
from amdkube.kubelet.cri_client import CRIClient
from amdkube.runtime import RocShim
from amdkube.runtime.images import NATIVE_BIN
from amdkube.runtime.oci import ImageFormatError, apply_layer, import_image, write_docker_archive
from amdkube.runtime.rootless import elf_interp, rootfs_argv
from tests.conftest import run, log_text


def host_closure(*progs) -> list[tuple]:
    """Layer entries holding `progs` and their shared-library closure (ldd), at host paths."""
    files = set()
    for p in progs:
        files.add(p)
        out = subprocess.run(["ldd", p], capture_output=True, text=True).stdout
        for line in out.splitlines():
            parts = line.split()
            for tok in parts:
                if tok.startswith("/") and os.path.exists(tok):
                    files.add(tok)
    entries, dirs = [], set()
    for f in sorted(files):
        rel = f.lstrip("/")
        d = os.path.dirname(rel)
        while d and d not in dirs:
            dirs.add(d)
            d = os.path.dirname(d)
        with open(os.path.realpath(f), "rb") as fh:
            entries.append((rel, fh.read(), 0o755, None))
    return [(d, None, 0o755, None) for d in sorted(dirs)] + entries


def test_layer_whiteouts_opaque_and_replacement(tmp_path):
    base = [("a", None, 0o755, None), ("a/x", b"x", 0o644, None), ("a/y", b"y", 0o644, None),
            ("b", None, 0o755, None), ("b/old1", b"1", 0o644, None), ("b/sub", None, 0o755, None),
            ("b/sub/old2", b"2", 0o644, None), ("c", b"file", 0o644, None), ("etc", None, 0o755, None),
            ("etc/conf", b"v1", 0o644, None), ("lnk", b"", 0o777, "/etc/conf")]
    top = [("a/.wh.x", b"", 0o644, None),            # delete a/x
           ("b/.wh..wh..opq", b"", 0o644, None),     # hide everything lower layers put in b/
           ("b/new", b"n", 0o644, None),
           ("c", None, 0o755, None), ("c/inside", b"i", 0o644, None),   # file → directory
           ("etc/conf", b"v2", 0o644, None)]
    arch = tmp_path / "img.tar"
    write_docker_archive(str(arch), [base, top], {"Entrypoint": ["/bin/true"]}, ["amdkube/test:1"])
    rec = import_image(str(arch), str(tmp_path / "store"))
    r = rec["rootfs"]
    listing = sorted(os.path.relpath(os.path.join(dp, f), r) for dp, dn, fn in os.walk(r) for f in fn + dn)
    assert listing == ["a", "a/y", "b", "b/new", "c", "c/inside", "etc", "etc/conf", "lnk"], listing
    assert open(os.path.join(r, "etc/conf")).read() == "v2"
    assert os.readlink(os.path.join(r, "lnk")) == "/etc/conf"      # absolute links stay (image-relative)
    assert len(rec["layers"]) == 2 and all(x.startswith("sha256:") for x in rec["layers"])
    assert rec["repo_tags"] == ["amdkube/test:1"] and rec["entrypoint"] == ["/bin/true"]


@pytest.mark.parametrize("evil", [
    [("../escape", b"x", 0o644, None)],
    [("link", b"", 0o777, "/tmp"), ("link/pwned", b"x", 0o644, None)],     # write through a symlinked parent
    [(".wh..", b"", 0o644, None)],                                         # whiteout of the root's parent
    [("sub/x", b"x", 0o644, None), ("sub/.wh..", b"", 0o644, None)],
])
def test_layer_cannot_write_outside_the_root(tmp_path, evil):
    data = io.BytesIO()
    with tarfile.open(fileobj=data, mode="w") as tf:
        for name, body, mode, link in evil:
            ti = tarfile.TarInfo(name)
            ti.mode = mode
            if link:
                ti.type, ti.linkname = tarfile.SYMTYPE, link
                tf.addfile(ti)
            else:
                ti.size = len(body)
                tf.addfile(ti, io.BytesIO(body))
    lp = tmp_path / "layer.tar"
    lp.write_bytes(data.getvalue())
    with pytest.raises(ImageFormatError):
        apply_layer(str(lp), str(tmp_path / "root"))
    assert not os.path.exists("/tmp/pwned") and not (tmp_path / "escape").exists()
    assert lp.exists()     # nothing beside the root was whited out


@pytest.mark.parametrize("victim_is_dir", [False, True])
def test_layer_symlinked_parent_cannot_delete_host_files(tmp_path, victim_is_dir):
    """A layer holding `x -> <host dir>` and then `x/victim` must be refused BEFORE the existing
    `<host dir>/victim` is removed to make room for the new entry."""
    host = tmp_path / "host"
    host.mkdir()
    if victim_is_dir:
        (host / "victim").mkdir()
        (host / "victim" / "keep").write_text("precious")
    else:
        (host / "victim").write_text("precious")
    data = io.BytesIO()
    with tarfile.open(fileobj=data, mode="w") as tf:
        ti = tarfile.TarInfo("x")
        ti.type, ti.linkname = tarfile.SYMTYPE, str(host)
        tf.addfile(ti)
        ti = tarfile.TarInfo("x/victim")
        ti.size = 4
        tf.addfile(ti, io.BytesIO(b"evil"))
    lp = tmp_path / "layer.tar"
    lp.write_bytes(data.getvalue())
    with pytest.raises(ImageFormatError):
        apply_layer(str(lp), str(tmp_path / "root"))
    keep = host / "victim" / "keep" if victim_is_dir else host / "victim"
    assert keep.read_text() == "precious"


def _oci_layout(dirpath, layers, config):
    """Write an OCI image layout (gzip layers) to `dirpath`."""
    os.makedirs(os.path.join(dirpath, "blobs", "sha256"))

    def put(b):
        d = hashlib.sha256(b).hexdigest()
        with open(os.path.join(dirpath, "blobs", "sha256", d), "wb") as f:
            f.write(b)
        return "sha256:" + d, len(b)
    from amdkube.runtime.oci import _tar_bytes
    descs, diffs = [], []
    for entries in layers:
        raw = _tar_bytes(entries)
        diffs.append("sha256:" + hashlib.sha256(raw).hexdigest())
        dg, n = put(gzip.compress(raw))
        descs.append({"mediaType": "application/vnd.oci.image.layer.v1.tar+gzip", "digest": dg, "size": n})
    cdg, cn = put(json.dumps({"architecture": "amd64", "os": "linux", "config": config,
                              "rootfs": {"type": "layers", "diff_ids": diffs}}).encode())
    mdg, mn = put(json.dumps({"schemaVersion": 2, "config": {"mediaType": "application/vnd.oci.image.config.v1+json",
                                                             "digest": cdg, "size": cn}, "layers": descs}).encode())
    with open(os.path.join(dirpath, "index.json"), "w") as f:
        json.dump({"schemaVersion": 2, "manifests": [{"mediaType": "application/vnd.oci.image.manifest.v1+json",
                                                      "digest": mdg, "size": mn,
                                                      "annotations": {"org.opencontainers.image.ref.name": "oci/demo:2"}}]}, f)
    with open(os.path.join(dirpath, "oci-layout"), "w") as f:
        json.dump({"imageLayoutVersion": "1.0.0"}, f)


def test_oci_layout_import_checks_digests(tmp_path):
    lay = tmp_path / "oci"
    _oci_layout(str(lay), [[("hello.txt", b"hi", 0o644, None)]], {"Cmd": ["cat", "/hello.txt"], "WorkingDir": "/w"})
    rec = import_image(str(lay), str(tmp_path / "store"))
    assert open(os.path.join(rec["rootfs"], "hello.txt")).read() == "hi"
    assert rec["cmd"] == ["cat", "/hello.txt"] and rec["workdir"] == "/w" and rec["repo_tags"] == ["oci/demo:2"]
    # a tampered blob fails the digest check
    blobs = lay / "blobs" / "sha256"
    layer = max(blobs.iterdir(), key=lambda p: p.stat().st_size if p.read_bytes()[:2] == b"\x1f\x8b" else -1)
    layer.write_bytes(gzip.compress(b"tampered"))
    with pytest.raises(ImageFormatError):
        import_image(str(lay), str(tmp_path / "store2"))


def test_archive_metadata_cannot_name_files_outside_the_archive(tmp_path):
    """manifest.json Config/Layers and index.json digests are archive-relative: a '../' path or a
    digest that is not hex of its algorithm's length is refused, not read from the host."""
    secret = tmp_path / "host-secret.json"
    secret.write_text("{}")
    dock = tmp_path / "dock"
    dock.mkdir()
    (dock / "manifest.json").write_text(json.dumps([{"Config": "../host-secret.json", "Layers": []}]))
    with pytest.raises(ImageFormatError, match="leaves the archive"):
        import_image(str(dock), str(tmp_path / "s1"))
    (dock / "manifest.json").write_text(json.dumps([{"Config": str(secret), "Layers": []}]))
    with pytest.raises(ImageFormatError, match="leaves the archive"):
        import_image(str(dock), str(tmp_path / "s2"))
    lay = tmp_path / "oci"
    _oci_layout(str(lay), [[("a", b"a", 0o644, None)]], {})
    for bad in ("sha512:../../host-secret.json", "md5:" + "0" * 32, "sha256:" + "0" * 63):
        (lay / "index.json").write_text(json.dumps({"schemaVersion": 2, "manifests": [{"digest": bad}]}))
        with pytest.raises(ImageFormatError, match="digest"):
            import_image(str(lay), str(tmp_path / "s3"))


def test_rootfs_argv_runs_the_images_own_loader(tmp_path):
    arch = tmp_path / "sh.tar"
    write_docker_archive(str(arch), [host_closure("/bin/sh", "/bin/cat")], {"Entrypoint": ["/bin/sh", "-c"]}, [])
    rec = import_image(str(arch), str(tmp_path / "store"))
    assert elf_interp(os.path.join(rec["rootfs"], "bin/sh")).endswith("ld-linux-x86-64.so.2")
    argv = rootfs_argv(rec["rootfs"], ["sh", "-c", "echo from-image"], "/usr/bin:/bin")
    assert argv[0].startswith(rec["rootfs"]) and argv[1] == "--library-path"
    assert subprocess.run(argv, capture_output=True, text=True).stdout.strip() == "from-image"


def test_image_config_precedence_and_gc_through_cri(tmp_path):
    arch = tmp_path / "app.tar"
    layer = host_closure("/bin/sh") + [("srv", None, 0o755, None)]
    write_docker_archive(str(arch), [layer], {"Entrypoint": ["/bin/sh", "-c"], "Cmd": ["echo CMD $GREETING; pwd"],
                                              "Env": ["GREETING=from-image", "PATH=/usr/bin:/bin"], "WorkingDir": "/srv"},
                         ["amdkube/app:1"])

    async def go():
        base = tempfile.mkdtemp(prefix="rsimg", dir="/tmp")
        shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks")).start()
        cri = await CRIClient(os.path.join(base, "s.sock")).connect()
        try:
            ref = await cri.pull_image(f"file://{arch}")
            assert ref.startswith("sha256:")
            before = (await cri.image_fs_info())[0].used_bytes.value
            assert before > 0
            assert os.listdir(os.path.join(base, "state", "images", "layers"))
            sc = C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name="p", uid="u1", namespace="default"))
            sid = await cri.run_pod_sandbox(sc)
            logs = {}
            for name, cmd, args, envs in (("default", [], [], {}),                                   # Entrypoint + Cmd
                                          ("args", [], ["echo ARGS $GREETING"], {"GREETING": "from-pod"}),  # Entrypoint + args
                                          ("cmd", ["/bin/sh", "-c"], ["echo OWN"], {})):             # command replaces both
                cfg = C.ContainerConfig(metadata=C.ContainerMetadata(name=name), image=C.ImageSpec(image="amdkube/app:1"),
                                        command=cmd, args=args, envs=[C.KeyValue(key=k, value=v) for k, v in envs.items()])
                cid = await cri.create_container(sid, cfg, sc)
                await cri.start_container(cid)
                for _ in range(300):
                    st, _ = await cri.container_status(cid)
                    if st.state == C.CONTAINER_EXITED:
                        break
                    await asyncio.sleep(0.01)
                assert st.exit_code == 0, log_text(st.log_path)
                logs[name] = log_text(st.log_path).split()
            assert logs["default"][:2] == ["CMD", "from-image"] and logs["default"][2] == "/srv"   # rootview: image paths
            assert logs["args"][:2] == ["ARGS", "from-pod"]
            assert logs["cmd"] == ["OWN"]
            await cri.stop_pod_sandbox(sid)
            await cri.remove_pod_sandbox(sid)
            await cri.remove_image(ref)
            assert os.listdir(os.path.join(base, "state", "images", "layers")) == []   # layers freed
            assert (await cri.image_fs_info())[0].used_bytes.value < before
        finally:
            await cri.close()
            await shim.stop(kill_pods=True)
            shutil.rmtree(base, ignore_errors=True)
    run(go())


@pytest.mark.skipif(os.geteuid() != 0, reason="pivot_root into an overlay needs root (or a user namespace)")
def test_nsexec_pivots_into_the_image(tmp_path):
    arch = tmp_path / "img.tar"
    layer = host_closure("/bin/sh", "/bin/cat", "/bin/ls") + [("etc", None, 0o755, None), ("etc/marker", b"in-image", 0o644, None)]
    write_docker_archive(str(arch), [layer], {}, [])
    rec = import_image(str(arch), str(tmp_path / "store"))
    vol = tmp_path / "vol"
    vol.mkdir()
    (vol / "data").write_text("volume-data")
    upper = tmp_path / "ctr"
    script = "cat /etc/marker; echo; cat /data/data; echo; for f in /dev/*; do printf '%s ' ${f#/dev/}; done; echo; echo w > /written; pwd"
    p = subprocess.run([os.path.join(NATIVE_BIN, "amdkube-nsexec"), "--dev-root", "/dev", "--rootfs", rec["rootfs"],
                        "--rootfs-upper", str(upper), "--workdir", "/etc", "--bind", f"{vol}:/data:ro", "--hide-kfd",
                        "--", "/bin/sh", "-c", script], capture_output=True, text=True, timeout=30,
                       env={"PATH": "/usr/bin:/bin"})
    if p.returncode == 126 and "overlay" in p.stderr:
        pytest.skip(f"no overlayfs here: {p.stderr.strip()}")
    assert p.returncode == 0, p.stderr
    out = p.stdout.splitlines()
    assert out[0] == "in-image" and out[1] == "volume-data"
    assert set(out[2].split()) >= {"null", "zero", "urandom", "shm"} and "kfd" not in out[2].split()
    assert out[3] == "/etc"
    # the write landed in the container's layer, not in the image
    assert (upper / "upper" / "written").exists() and not os.path.exists(os.path.join(rec["rootfs"], "written"))


def test_rootview_makes_the_image_root_the_containers_root(tmp_path):
    """No mount namespace (isolation=env, as on the unprivileged MI355X node): the rootview
    preload (native/rootview.c) moves a workload's own file-system calls under the image. /etc
    is the image's (an absolute symlink in the image resolves inside it), the host's files are
    gone, volumes sit at their mount paths, /tmp is the container's own, cwd reads as a
    container path, and programs the workload execs — a `#!` script too — come from the image."""
    arch = tmp_path / "view.tar"
    layer = host_closure("/bin/sh", "/bin/cat", "/bin/ls") + [
        ("etc", None, 0o755, None), ("etc/marker", b"in-image\n", 0o644, None),
        ("etc/abs-link", None, 0o777, "/etc/marker"), ("srv", None, 0o755, None),
        ("usr", None, 0o755, None), ("usr/local", None, 0o755, None), ("usr/local/bin", None, 0o755, None),
        ("usr/local/bin/hello.sh", b"#!/bin/sh\necho hello-from-image-script\n", 0o755, None)]
    write_docker_archive(str(arch), [layer], {"Entrypoint": ["/bin/sh", "-c"], "Env": ["PATH=/usr/local/bin:/usr/bin:/bin"],
                                              "WorkingDir": "/srv"}, ["amdkube/view:1"])
    vol = tmp_path / "vol"
    vol.mkdir()
    (vol / "f").write_text("from-volume\n")
    script = ("cat /etc/marker; cat /etc/abs-link; cat /etc/hostname 2>/dev/null || echo no-host-etc; pwd; "
              "echo scratch > /tmp/rv-probe; cat /tmp/rv-probe; cat /data/f; hello.sh; echo $(ls /); "
              "echo changed > /etc/marker; cat /etc/marker; echo new > /etc/added; echo $(ls /etc)")

    async def go():
        base = tempfile.mkdtemp(prefix="rsview", dir="/tmp")
        shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks")).start()
        cri = await CRIClient(os.path.join(base, "s.sock")).connect()
        try:
            await cri.pull_image(f"file://{arch}")
            sc = C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name="p", uid="u2", namespace="default"))
            sid = await cri.run_pod_sandbox(sc)
            cfg = C.ContainerConfig(metadata=C.ContainerMetadata(name="v"), image=C.ImageSpec(image="amdkube/view:1"),
                                    args=[script], mounts=[C.Mount(container_path="/data", host_path=str(vol))])
            cid = await cri.create_container(sid, cfg, sc)
            await cri.start_container(cid)
            for _ in range(500):
                st, _ = await cri.container_status(cid)
                if st.state == C.CONTAINER_EXITED:
                    break
                await asyncio.sleep(0.01)
            out = log_text(st.log_path)
            assert st.exit_code == 0, out
            lines = out.split("\n")
            assert lines[:8] == ["in-image", "in-image", "no-host-etc", "/srv", "scratch", "from-volume",
                                 "hello-from-image-script", lines[7]], lines
            listing = set(lines[7].split())
            # the image's directories, not the host's (mount points are not listed: no mount table)
            assert {"bin", "etc", "srv", "usr"} <= listing and not listing & {"root", "home", "opt", "var"}, listing
            # writes land in the container's own layer: the view sees them, the image does not change
            assert lines[8] == "changed" and sorted(lines[9].split()) == ["abs-link", "added", "marker"], lines[8:10]
            rootfs = os.path.join(base, "state", "images")
            marker = [os.path.join(dp, f) for dp, _, fs in os.walk(rootfs) for f in fs if f == "marker"]
            assert marker and all(open(x).read() == "in-image\n" for x in marker), marker
            assert not [f for _, _, fs in os.walk(rootfs) for f in fs if f == "added"]
            assert not os.path.exists("/tmp/rv-probe")                 # the container's /tmp, not the host's
            await cri.stop_pod_sandbox(sid)
            await cri.remove_pod_sandbox(sid)
        finally:
            await cri.close()
            await shim.stop(kill_pods=True)
            shutil.rmtree(base, ignore_errors=True)
    run(go())
