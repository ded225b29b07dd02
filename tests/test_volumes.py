"""Volume plugins, the kubelet volume manager and the attach/detach controller
(pkg/volume/*/..._test.go with the fake mounter/exec, flexvolume driver-call and
attacher/mounter tests against a scripted driver, csi_attacher/csi_mounter tests against a fake
CSI driver, kubelet volumemanager reconciler tests, attachdetach controller tests)."""
import asyncio
import json
import os
import stat
import textwrap

import grpc

from amdkube.api import meta as m
from amdkube.grpcdesc.csi import CSI
from amdkube.kubelet.volumemanager import VolumeManager, subpath
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.volume import FakeExec, FakeMounter, MountError, PluginMgr, Spec, VolumeError, VolumeHost, default_plugins
from amdkube.volume.csi import ExternalAttacher, attachment_name
from amdkube.volume.flex import probe
from tests.conftest import run


class FakeClient:
    def __init__(self, objs=None):
        self.objs = objs or {}

    async def get_or_none(self, res, name, ns=""):
        return self.objs.get((res, ns, name))


def _host(tmp_path, mounter=None, executor=None, client=None):
    h = VolumeHost(str(tmp_path / "kubelet"), "node-a", client or FakeClient(), mounter or FakeMounter(), executor or FakeExec())
    h.dev_root = str(tmp_path / "root")
    h.sys_root = str(tmp_path / "sys")
    h.attach_poll = 0.01
    return h


def _pod(uid="u1", volumes=(), ns="default", **spec):
    return {"metadata": {"name": "p", "namespace": ns, "uid": uid}, "spec": {"volumes": list(volumes), "containers": [], **spec}}


def test_plugin_manager_matching_and_unique_names(tmp_path):
    mgr = PluginMgr(default_plugins(), _host(tmp_path))
    names = {p.name for p in mgr.plugins.values()}
    assert {"kubernetes.io/empty-dir", "kubernetes.io/host-path", "kubernetes.io/nfs", "kubernetes.io/iscsi", "kubernetes.io/rbd",
            "kubernetes.io/fc", "kubernetes.io/csi", "kubernetes.io/cephfs", "kubernetes.io/glusterfs", "kubernetes.io/secret",
            "kubernetes.io/local-volume", "kubernetes.io/aws-ebs"} <= names
    ed = Spec(volume={"name": "scratch", "emptyDir": {}})
    p = mgr.find_by_spec(ed)
    assert p.name == "kubernetes.io/empty-dir" and p.unique_name(ed, "uid1") == "kubernetes.io/empty-dir/uid1-scratch"
    iscsi = Spec(pv={"metadata": {"name": "pv1"}, "spec": {"iscsi": {"targetPortal": "10.0.0.1", "iqn": "iqn.x:t", "lun": 3}}})
    ip = mgr.find_by_spec(iscsi)
    assert ip.attachable and ip.unique_name(iscsi, "any") == "kubernetes.io/iscsi/10.0.0.1:3260:iqn.x:t:3"
    # local is PV-only; csi is PV-only; unknown sources match nothing
    try:
        mgr.find_by_spec(Spec(volume={"name": "x", "local": {"path": "/"}}))
        raise AssertionError("inline local volume must not match")
    except VolumeError:
        pass
    try:
        mgr.find_by_spec(Spec(volume={"name": "x", "fancyVolume": {}}))
        raise AssertionError("expected no match")
    except VolumeError as e:
        assert "no volume plugin matched" in str(e)


def test_empty_dir_media_and_teardown(tmp_path):
    async def go():
        fm = FakeMounter()
        mgr = PluginMgr(default_plugins(), _host(tmp_path, fm))
        ed = mgr.find_by_name("kubernetes.io/empty-dir")
        base = tmp_path / "kubelet" / "pods" / "u1" / "volumes" / "kubernetes.io~empty-dir"
        d = str(base / "disk")
        assert await ed.set_up(Spec(volume={"name": "disk", "emptyDir": {}}), _pod(), d) == d
        assert stat.S_IMODE(os.stat(d).st_mode) == 0o777 and not fm.log
        open(os.path.join(d, "f"), "w").write("x")
        mem = str(base / "mem")
        await ed.set_up(Spec(volume={"name": "mem", "emptyDir": {"medium": "Memory", "sizeLimit": "64Mi"}}), _pod(), mem)
        assert fm.log[-1] == ("mount", mem, "tmpfs", "tmpfs", [f"size={64 << 20}"])
        huge = str(base / "huge")
        pod = _pod(containers=[{"name": "c", "resources": {"limits": {"hugepages-2Mi": "4Mi", "memory": "1Gi"}}}])
        await ed.set_up(Spec(volume={"name": "huge", "emptyDir": {"medium": "HugePages"}}), pod, huge)
        assert fm.log[-1] == ("mount", huge, "nodev", "hugetlbfs", ["pagesize=2Mi"])
        for x in (d, mem, huge):
            await ed.tear_down(x)
            assert not os.path.exists(x)
        assert [a[1] for a in fm.actions("unmount")] == [mem, huge]
        assert not [e for e in os.listdir(base) if ".deleting~" in e]
    run(go(), 10)


def test_network_filesystems(tmp_path):
    async def go():
        fm = FakeMounter()
        client = FakeClient({("secrets", "default", "ceph"): {"data": {"key": "QVFCc2VjcmV0"}},
                             ("endpoints", "default", "gluster"): {"subsets": [{"addresses": [{"ip": "10.1.0.1"}, {"ip": "10.1.0.2"}]}]}})
        mgr = PluginMgr(default_plugins(), _host(tmp_path, fm, client=client))
        pv = {"metadata": {"name": "share"}, "spec": {"nfs": {"server": "nas", "path": "/export/ds"},
                                                      "mountOptions": ["vers=4.1", "hard"]}}
        nfs = Spec(pv=pv, read_only=True)
        d = str(tmp_path / "nfs")
        await mgr.find_by_spec(nfs).set_up(nfs, _pod(), d)
        assert fm.log[-1] == ("mount", d, "nas:/export/ds", "nfs", ["ro", "vers=4.1", "hard"])
        ceph = Spec(volume={"name": "c", "cephfs": {"monitors": ["m1:6789", "m2:6789"], "path": "/data", "user": "k8s",
                                                    "secretRef": {"name": "ceph"}}})
        d2 = str(tmp_path / "ceph")
        await mgr.find_by_spec(ceph).set_up(ceph, _pod(), d2)
        assert fm.log[-1] == ("mount", d2, "m1:6789,m2:6789:/data", "ceph", ["name=k8s", "secret=AQBsecret"])
        gl = Spec(volume={"name": "g", "glusterfs": {"endpoints": "gluster", "path": "vol0"}})
        d3 = str(tmp_path / "gl")
        await mgr.find_by_spec(gl).set_up(gl, _pod(), d3)
        act = fm.log[-1]
        assert act[2] == "10.1.0.1:vol0" and act[3] == "glusterfs" and "backup-volfile-servers=10.1.0.2" in act[4]
        assert any(o.startswith("log-file=") and o.endswith("u1-glusterfs.log") for o in act[4])
        # a failing mount leaves no directory behind
        fm.fail[str(tmp_path / "bad")] = "mount.nfs: Connection timed out"
        try:
            await mgr.find_by_spec(nfs).set_up(nfs, _pod(), str(tmp_path / "bad"))
            raise AssertionError("expected failure")
        except VolumeError as e:
            assert "Connection timed out" in str(e)
        assert not os.path.exists(tmp_path / "bad")
        for x in (d, d2, d3):
            await mgr.find_by_spec(nfs).tear_down(x)
        assert len(fm.actions("unmount")) == 3 and not fm.mounts
        # a vendor volume whose backend is unreachable fails with a precise reason
        pwx = Spec(volume={"name": "e", "portworxVolume": {"volumeID": "vol-1"}})
        try:
            await mgr.find_by_spec(pwx).set_up(pwx, _pod(), str(tmp_path / "e"))
            raise AssertionError("expected failure")
        except VolumeError as e:
            assert "storage backend at http://127.0.0.1:9001/v1/osd-volumes/vol-1 is unreachable" in str(e)
        # an EBS disk is a real attachable plugin, served through the AWS cloud provider
        ebs = Spec(volume={"name": "e", "awsElasticBlockStore": {"volumeID": "vol-1"}})
        assert mgr.find_by_spec(ebs).attachable and mgr.find_by_spec(ebs).name == "kubernetes.io/aws-ebs"
    run(go(), 10)


class FirstMountFails(FakeMounter):
    def mount(self, source, target, fstype="", options=None):
        if source.startswith(("/dev/", "/")) and fstype == "ext4" and not getattr(self, "_failed", False):
            self._failed = True
            raise MountError("wrong fs type, bad option, bad superblock")
        super().mount(source, target, fstype, options)


def test_iscsi_login_format_mount_bind_and_logout(tmp_path):
    async def go():
        fm = FirstMountFails()
        ex = FakeExec({("blkid",): (2, ""), ("iscsiadm", "-m", "node"): (0, "")})
        h = _host(tmp_path, fm, ex, FakeClient({("secrets", "default", "chap"): {"data": {
            "node.session.auth.username": "dXNlcg==", "node.session.auth.password": "cGFzcw=="}}}))
        mgr = PluginMgr(default_plugins(), h)
        spec = Spec(pv={"metadata": {"name": "lun0"}, "spec": {"iscsi": {
            "targetPortal": "10.0.0.9:3260", "iqn": "iqn.2018-01.io.amd:store", "lun": 0, "fsType": "ext4",
            "chapAuthSession": True, "secretRef": {"name": "chap"}}}})
        p = mgr.find_by_spec(spec)
        dev = tmp_path / "root" / "dev" / "disk" / "by-path" / "ip-10.0.0.9:3260-iscsi-iqn.2018-01.io.amd:store-lun-0"

        async def appear():
            await asyncio.sleep(0.05)        # udev creates the link after login
            dev.parent.mkdir(parents=True)
            dev.write_text("")
        t = asyncio.create_task(appear())
        device = await p.wait_for_attach(spec, "", _pod(), 5)
        await t
        assert device == str(dev)
        cmds = [" ".join(c) for c in ex.calls]
        assert any("--discover" in c for c in cmds) and any(c.endswith("--login") for c in cmds)
        assert any("node.session.auth.username -v user" in c for c in cmds)
        gpath = p.device_mount_path(spec)
        assert gpath.endswith("kubernetes.io~iscsi/iface-default/10.0.0.9:3260-iqn.2018-01.io.amd:store-lun-0")
        await p.mount_device(spec, device, gpath)
        assert any(c[0] == "mkfs.ext4" and c[-1] == device for c in ex.calls)     # blank device formatted once
        assert fm.mounts[-1].path == os.path.realpath(gpath) and fm.mounts[-1].type == "ext4"
        d = str(tmp_path / "pod-vol")
        assert await p.set_up(spec, _pod(), d, gpath) == d
        assert fm.log[-1][0] == "mount" and fm.log[-1][4] == ["bind"] and fm.get_mount_refs(gpath) == [os.path.realpath(d)]
        await p.tear_down(d)
        await p.unmount_device(gpath)
        cmds = [" ".join(c) for c in ex.calls]
        assert any(c.endswith("--logout") for c in cmds) and not fm.mounts
    run(go(), 10)


def test_rbd_map_and_unmap(tmp_path):
    async def go():
        fm = FakeMounter()
        ex = FakeExec({("rbd", "map"): (0, "/dev/rbd3\n")})
        mgr = PluginMgr(default_plugins(), _host(tmp_path, fm, ex))
        spec = Spec(volume={"name": "r", "rbd": {"monitors": ["10.0.0.1:6789"], "image": "ds", "pool": "kube",
                                                   "keyring": "/etc/ceph/k", "fsType": "xfs"}})
        p = mgr.find_by_spec(spec)
        dev = await p.wait_for_attach(spec, "", _pod(), 5)
        assert dev == "/dev/rbd3" and ex.calls[0][:3] == ["rbd", "map", "kube/ds"] and "--keyring=/etc/ceph/k" in ex.calls[0]
        g = p.device_mount_path(spec)
        await p.mount_device(spec, dev, g)
        assert fm.log[-1] == ("mount", g, "/dev/rbd3", "xfs", [])
        await p.unmount_device(g)
        assert ex.calls[-1] == ["rbd", "unmap", "/dev/rbd3"]
    run(go(), 10)


FLEX = textwrap.dedent("""\
    #!/bin/sh
    echo "$@" >> "$(dirname "$0")/calls.log"
    case "$1" in
      init) echo '{"status": "Success", "capabilities": {"attach": ATTACH}}' ;;
      attach) echo '{"status": "Success", "device": "/dev/flex0"}' ;;
      waitforattach) echo "{\\"status\\": \\"Success\\", \\"device\\": \\"$2\\"}" ;;
      mountdevice) echo '{"status": "Not supported"}' ;;
      mount) mkdir -p "$2"; echo '{"status": "Success"}' ;;
      unmount) rmdir "$2"; echo '{"status": "Success"}' ;;
      detach) echo '{"status": "Success"}' ;;
      *) echo '{"status": "Not supported"}' ;;
    esac
    """)


def _driver(d, vendor, name, attach):
    dd = d / f"{vendor}~{name}"
    dd.mkdir(parents=True)
    exe = dd / name
    exe.write_text(FLEX.replace("ATTACH", "true" if attach else "false"))
    exe.chmod(0o755)
    return dd / "calls.log"


def test_flexvolume_driver_calls(tmp_path):
    async def go():
        plug = tmp_path / "volumeplugins"
        log_a = _driver(plug, "amd", "blk", True)
        log_b = _driver(plug, "amd", "nas", False)
        (plug / "amd~broken").mkdir()              # no executable: skipped by the prober
        fm = FakeMounter()
        h = _host(tmp_path, fm, client=FakeClient({("secrets", "ns1", "cred"): {"data": {"token": "czNj"}}}))
        h.flex_dir = str(plug)
        found = {p.name: p for p in probe(str(plug))}
        assert set(found) == {"flexvolume-amd/blk", "flexvolume-amd/nas"}
        assert found["flexvolume-amd/blk"].attachable and not found["flexvolume-amd/nas"].attachable
        mgr = PluginMgr(default_plugins(), h)
        spec = Spec(volume={"name": "v", "flexVolume": {"driver": "amd/blk", "fsType": "ext4", "secretRef": {"name": "cred"},
                                                        "options": {"size": "10G"}}})
        p = mgr.find_by_spec(spec)            # discovered on demand
        assert p.name == "flexvolume-amd/blk"
        dev = await p.attach(spec, "node-a")
        dev = await p.wait_for_attach(spec, dev, None, 5)
        assert dev == "/dev/flex0"
        g = p.device_mount_path(spec)
        await p.mount_device(spec, dev, g)          # "Not supported" → format+mount the device
        assert "mountdevice" in p.unsupported and fm.log[-1][:4] == ("mount", g, "/dev/flex0", "ext4")
        pod = {"metadata": {"name": "web", "namespace": "ns1", "uid": "u9"}, "spec": {"serviceAccountName": "sa"}}
        d = str(tmp_path / "pods" / "u9" / "v")
        await p.set_up(spec, pod, d, g, fs_group=2000)
        await p.tear_down(d)
        await p.detach("v", "node-a")
        calls = [c for c in log_a.read_text().splitlines() if c != "init"]      # probed twice: by the test, by the manager
        assert [c.split()[0] for c in calls] == ["attach", "waitforattach", "mountdevice", "mount", "unmount", "detach"]
        opts = json.loads(calls[3].split(" ", 2)[2])
        assert opts["kubernetes.io/pod.name"] == "web" and opts["kubernetes.io/pod.namespace"] == "ns1"
        assert opts["kubernetes.io/serviceAccount.name"] == "sa" and opts["kubernetes.io/fsGroup"] == "2000"
        assert opts["kubernetes.io/secret/token"] == "czNj" and opts["size"] == "10G" and opts["kubernetes.io/readwrite"] == "rw"
        assert calls[0].split()[-1] == "node-a" and not os.path.exists(d)
        assert set(log_b.read_text().split()) == {"init"}     # the non-attaching driver was only probed
    run(go(), 20)


# ------------------------------------------------------------------------ CSI
class FakeCSIDriver:
    def __init__(self, sock):
        self.sock = sock
        self.calls = []
        self.fail_publish = None

    async def GetSupportedVersions(self, req, ctx):
        return CSI.GetSupportedVersionsResponse(supported_versions=[CSI.Version(major=0, minor=1, patch=0)])

    async def GetPluginInfo(self, req, ctx):
        return CSI.GetPluginInfoResponse(name="csi.amd.com", vendor_version="0.1")

    async def ControllerPublishVolume(self, req, ctx):
        self.calls.append(("ControllerPublish", req.volume_id, req.node_id, req.volume_capability.access_mode.mode))
        return CSI.ControllerPublishVolumeResponse(publish_volume_info={"lun": "7"})

    async def ControllerUnpublishVolume(self, req, ctx):
        self.calls.append(("ControllerUnpublish", req.volume_id, req.node_id))
        return CSI.ControllerUnpublishVolumeResponse()

    async def NodeProbe(self, req, ctx):
        return CSI.NodeProbeResponse()

    async def NodePublishVolume(self, req, ctx):
        if self.fail_publish:
            await ctx.abort(grpc.StatusCode.INTERNAL, self.fail_publish)
        self.calls.append(("NodePublish", req.volume_id, req.target_path, dict(req.publish_volume_info),
                           req.volume_capability.mount.fs_type, dict(req.volume_attributes), req.readonly))
        return CSI.NodePublishVolumeResponse()

    async def NodeUnpublishVolume(self, req, ctx):
        self.calls.append(("NodeUnpublish", req.volume_id, req.target_path))
        return CSI.NodeUnpublishVolumeResponse()

    async def start(self):
        os.makedirs(os.path.dirname(self.sock), exist_ok=True)
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((CSI.Identity.handler(self), CSI.Controller.handler(self), CSI.Node.handler(self)))
        self.server.add_insecure_port("unix://" + self.sock)
        await self.server.start()
        return self

    async def stop(self):
        await self.server.stop(0)


async def _until(fn, timeout=20.0):
    end = asyncio.get_running_loop().time() + timeout
    while True:
        v = await fn()
        if v:
            return v
        if asyncio.get_running_loop().time() > end:
            raise AssertionError("condition not met")
        await asyncio.sleep(0.05)


def test_csi_attach_publish_unpublish_detach_end_to_end():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, node_status_update_frequency=0.5,
                                kubelet_kw={"volume_mounter": "fake", "volume_reconcile_period": 0.2}) as lc:
            c = lc.client
            drv = await FakeCSIDriver(os.path.join(lc.kubelet.cfg.root_dir, "plugins", "csi.amd.com", "csi.sock")).start()
            att = ExternalAttacher(c, "csi.amd.com", drv.sock, resync=0.1).start()
            try:
                await c.create({"apiVersion": "v1", "kind": "PersistentVolume", "metadata": {
                    "name": "ds-pv", "annotations": {"csi.volume.kubernetes.io/volume-attributes": '{"tier": "hbm"}'}},
                    "spec": {"capacity": {"storage": "10Gi"}, "accessModes": ["ReadWriteOnce"],
                             "csi": {"driver": "csi.amd.com", "volumeHandle": "vol-42"},
                             "claimRef": {"namespace": "default", "name": "ds"}}})
                await c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "ds"},
                                "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}},
                                         "volumeName": "ds-pv"}}, "default")
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "train"}, "spec": {
                    "volumes": [{"name": "data", "persistentVolumeClaim": {"claimName": "ds"}}],
                    "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"],
                                    "volumeMounts": [{"name": "data", "mountPath": "/data", "subPath": "shard0"}]}]}},
                               "default")
                pod = await wait_pod(c, "default", "train", timeout=30)
                uid = m.uid_of(pod)
                target = os.path.join(lc.kubelet.cfg.root_dir, "pods", uid, "volumes", "kubernetes.io~csi", "ds-pv", "mount")
                pubs = [x for x in drv.calls if x[0] == "NodePublish"]
                assert pubs == [("NodePublish", "vol-42", target, {"lun": "7"}, "ext4", {"tier": "hbm"}, False)]
                assert ("ControllerPublish", "vol-42", lc.node_name, CSI.SINGLE_NODE_WRITER) in drv.calls
                va = await c.get("volumeattachments", attachment_name("vol-42", "csi.amd.com", lc.node_name))
                assert va["status"]["attached"] and va["spec"]["attacher"] == "csi.amd.com"
                node = await c.get("nodes", lc.node_name)
                assert [a["name"] for a in node["status"]["volumesAttached"]] == ["kubernetes.io/csi/csi.amd.com^vol-42"]

                async def in_use():
                    n = await c.get("nodes", lc.node_name)
                    return n["status"].get("volumesInUse") == ["kubernetes.io/csi/csi.amd.com^vol-42"]
                await _until(in_use)
                assert os.path.isdir(os.path.join(target, "shard0"))          # subPath created inside the volume
                # pod gone → NodeUnpublish, then (volumesInUse cleared) detach → ControllerUnpublish
                await c.delete("pods", "train", "default", grace=0)

                async def detached():
                    return any(x[0] == "ControllerUnpublish" for x in drv.calls) and \
                        await c.get_or_none("volumeattachments", va["metadata"]["name"]) is None
                await _until(detached, 30)
                assert ("NodeUnpublish", "vol-42", target) in drv.calls
                i_unpub = next(i for i, x in enumerate(drv.calls) if x[0] == "NodeUnpublish")
                i_detach = next(i for i, x in enumerate(drv.calls) if x[0] == "ControllerUnpublish")
                assert i_unpub < i_detach            # safe detach: never while the node still uses it
                node = await c.get("nodes", lc.node_name)
                assert not node["status"].get("volumesAttached")
            finally:
                await att.stop()
                await drv.stop()
    run(go(), 90)


def test_failed_mount_event_and_subpath_escape(tmp_path):
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"volume_mount_timeout": 0.5, "volume_reconcile_period": 0.2}) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "nfs-pod"}, "spec": {
                "volumes": [{"name": "d", "nfs": {"server": "nas.invalid", "path": "/x"}}],
                "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "5"],
                                "volumeMounts": [{"name": "d", "mountPath": "/d"}]}]}}, "default")

            async def failed_mount():
                evs, _ = await c.list("events", "default")
                return [e for e in evs if e.get("reason") == "FailedMount" and "nfs-pod" in str(e.get("involvedObject"))]
            evs = await _until(failed_mount)
            assert "needs a privileged kubelet" in evs[0]["message"]
            p = await c.get("pods", "nfs-pod", "default")
            assert p["status"].get("phase", "Pending") == "Pending"
    run(go(), 60)
    d = tmp_path / "vol"
    d.mkdir()
    (d / "link").symlink_to("/etc")
    assert subpath(str(d), "a/b", "m").endswith("a/b") and os.path.isdir(d / "a" / "b")
    for bad in ("../x", "/abs", "link"):
        try:
            subpath(str(d), bad, "m")
            raise AssertionError(bad)
        except VolumeError:
            pass


def test_reconstruct_and_teardown_orphaned_volumes(tmp_path):
    async def go():
        fm = FakeMounter()
        h = _host(tmp_path, fm)
        vm_dir = tmp_path / "kubelet" / "pods" / "dead" / "volumes" / "kubernetes.io~empty-dir" / "cache"
        vm_dir.mkdir(parents=True)
        fm.mount("tmpfs", str(vm_dir), "tmpfs", [])

        class K:
            node_name, node, client, recorder = "node-a", {}, FakeClient(), None
        vm = VolumeManager(K(), PluginMgr(default_plugins(), h), period=0.05)
        vm.reconstruct()
        assert vm.has_mounts("dead")
        await vm.reconcile()
        assert not vm.has_mounts("dead") and not vm_dir.exists() and fm.actions("unmount")
    run(go(), 10)


def test_pod_dir_gc_keeps_directories_with_volumes(tmp_path):
    from amdkube.kubelet.kuberuntime import RuntimeManager

    class CRI:
        async def list_containers(self, *a, **k):
            return []

        async def list_pod_sandbox(self, *a, **k):
            return []
    rm = RuntimeManager.__new__(RuntimeManager)
    rm.cri, rm.root, rm.sandbox_ips = CRI(), str(tmp_path), {}
    for uid in ("a", "b"):
        (tmp_path / "pods" / uid).mkdir(parents=True)

    async def go():
        return await rm.garbage_collect(lambda uid: False, sources_ready=True, has_volumes=lambda uid: uid == "b")
    res = run(go(), 10)
    assert res["pod_dirs"] == 1 and not (tmp_path / "pods" / "a").exists() and (tmp_path / "pods" / "b").exists()


def _can_mount_tmpfs(tmp_path) -> bool:
    import subprocess
    if os.geteuid() != 0:
        return False
    d = tmp_path / "probe"
    d.mkdir()
    if subprocess.run(["mount", "-t", "tmpfs", "tmpfs", str(d)], capture_output=True).returncode != 0:
        return False
    subprocess.run(["umount", str(d)], capture_output=True)
    return True


def test_real_tmpfs_mounts_for_secret_and_memory_volumes(tmp_path):
    """With a privileged kubelet (system mounter) secret content lives on tmpfs, never on disk,
    and memory-medium emptyDirs are tmpfs; both are unmounted when the pod goes."""
    import pytest
    if not _can_mount_tmpfs(tmp_path):
        pytest.skip("needs root and mount(2)")
    from amdkube.volume.mount import SysMounter

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"volume_mounter": "system", "volume_reconcile_period": 0.2}) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "tok"}, "data": {"t": "czNjcjN0"}}, "default")
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sec"}, "spec": {
                "volumes": [{"name": "s", "secret": {"secretName": "tok"}}, {"name": "shm", "emptyDir": {"medium": "Memory"}}],
                "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"],
                                "volumeMounts": [{"name": "s", "mountPath": "/s"}, {"name": "shm", "mountPath": "/dev/shm"}]}]}},
                           "default")
            pod = await wait_pod(c, "default", "sec", timeout=30)
            vols = os.path.join(lc.kubelet.cfg.root_dir, "pods", m.uid_of(pod), "volumes")
            s_dir = os.path.join(vols, "kubernetes.io~secret", "s")
            shm = os.path.join(vols, "kubernetes.io~empty-dir", "shm")
            sm = SysMounter()
            table = {mp.path: mp.type for mp in sm.list()}
            assert table.get(os.path.realpath(s_dir)) == "tmpfs" and table.get(os.path.realpath(shm)) == "tmpfs"
            assert open(os.path.join(s_dir, "t")).read() == "s3cr3t"
            await c.delete("pods", "sec", "default", grace=0)

            async def unmounted():
                paths = {mp.path for mp in sm.list()}
                return os.path.realpath(s_dir) not in paths and os.path.realpath(shm) not in paths
            await _until(unmounted, 20)
    run(go(), 60)
