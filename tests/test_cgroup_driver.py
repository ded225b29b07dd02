"""--cgroup-driver=systemd: cgroup names, the D-Bus client, the kubelet's manager and rocshim scopes.

Reference: pkg/kubelet/cm/cgroup_manager_linux_test.go (TestLibcontainerAdapterAdaptToSystemd,
TestLibcontainerAdapterAdaptToSystemdAsCgroupFs — both tables transcribed),
cgroup_manager_linux.go (RevertFromSystemdToCgroupStyleName, the "systemd cgroup manager not
available" refusal), dockershim/docker_service.go:237-253 (kubelet and runtime must agree on the
driver). systemd itself is absent here and on the GPU box (and the box is unprivileged), so a
fake systemd speaking the D-Bus wire protocol over a unix socket stands in: it creates the slice
and scope directories under a temporary cgroup root and moves the scope's PIDs there. Parity
against a real systemd is unpinned.
"""
from __future__ import annotations

import asyncio
import os
import socket
import struct
import tempfile
import threading

import pytest

from amdkube.kubelet import cgroups as CG
from amdkube.utils import dbus as D
from tests.conftest import run, log_text


# ------------------------------------------------------------------ names (reference tables)
@pytest.mark.parametrize("inp,expected", [
    ("/", "-.slice"), ("/system.slice", "system.slice"), ("/system.slice/Burstable", "system-Burstable.slice"),
    ("/Burstable.slice/Burstable-pod_123.slice", "Burstable-pod_123.slice"),
    ("/test.slice/test-a.slice/test-a-b.slice", "test-a-b.slice"),
    ("/test.slice/test-a.slice/test-a-b.slice/Burstable", "test-a-b-Burstable.slice"),
    ("/Burstable", "Burstable.slice"), ("/Burstable/pod_123", "Burstable-pod_123.slice"),
    ("/BestEffort/pod_6c1a4e95-6bb6-11e6-bc26-28d2444e470d", "BestEffort-pod_6c1a4e95_6bb6_11e6_bc26_28d2444e470d.slice"),
])
def test_adapt_to_systemd(inp, expected):
    assert CG.CgroupManager(CG.SYSTEMD, units=object()).name(inp) == CG.expand_slice(expected)
    assert CG.to_systemd(inp) == expected


@pytest.mark.parametrize("inp,expected", [
    ("/", "/"), ("/Burstable", "Burstable.slice/"), ("/Burstable/pod_123", "Burstable.slice/Burstable-pod_123.slice/"),
    ("/BestEffort/pod_6c1a4e95-6bb6-11e6-bc26-28d2444e470d",
     "BestEffort.slice/BestEffort-pod_6c1a4e95_6bb6_11e6_bc26_28d2444e470d.slice/"),
])
def test_adapt_to_systemd_as_cgroupfs(inp, expected):
    assert CG.to_systemd(inp, True) == expected


@pytest.mark.parametrize("bad", ["", ".slice-", "a/b.slice", "test--a.slice", "-test.slice", "test.scope"])
def test_expand_slice_rejects_invalid_names(bad):
    with pytest.raises(CG.CgroupError):
        CG.expand_slice(bad)


def test_revert_and_cgroupfs_driver_identity():
    literal = CG.to_systemd("/kubepods/burstable/pod1234-5678", True)
    assert literal == "kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod1234_5678.slice/"
    assert CG.cgroupfs_to_systemd(literal) == "kubepods-burstable-pod1234_5678.slice"
    assert CG.revert_from_systemd(literal) == "kubepods/burstable/pod1234-5678"
    fs = CG.CgroupManager(CG.CGROUPFS)
    assert fs.name("/kubepods/pod1") == "/kubepods/pod1" and fs.cgroup_name("/kubepods/pod1") == "/kubepods/pod1"
    with pytest.raises(CG.CgroupError):
        CG.CgroupManager("upstart")


def test_pod_cgroup_parent_per_driver():
    from amdkube.kubelet.qos import cgroup_parent
    g = {"metadata": {"uid": "ab-cd"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "1", "memory": "1Gi"}, "limits": {"cpu": "1", "memory": "1Gi"}}}]}}
    b = {"metadata": {"uid": "ab-cd"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "1"}}}]}}
    be = {"metadata": {"uid": "ab-cd"}, "spec": {"containers": [{}]}}
    assert [cgroup_parent(p) for p in (g, b, be)] == ["kubepods/podab-cd", "kubepods/burstable/podab-cd",
                                                    "kubepods/besteffort/podab-cd"]
    assert [cgroup_parent(p, "systemd") for p in (g, b, be)] == [
        "kubepods.slice/kubepods-podab_cd.slice/",
        "kubepods.slice/kubepods-burstable.slice/kubepods-burstable-podab_cd.slice/",
        "kubepods.slice/kubepods-besteffort.slice/kubepods-besteffort-podab_cd.slice/"]


# ------------------------------------------------------------------ D-Bus wire format
def test_marshal_alignment_matches_the_specification():
    # y, then an array of (sv): length at 4, first struct 8-aligned, variant's signature, u 4-aligned
    got = D.marshal_body("ya(sv)", [1, [("a", ("u", 5))]])
    want = bytes([1, 0, 0, 0]) + struct.pack("<I", 16) + struct.pack("<I", 1) + b"a\0" + b"\x01u\0" + b"\0" * 3 + \
        struct.pack("<I", 5)
    assert got == want
    assert D.marshal_body("s", ["foo"]) == b"\x03\0\0\0foo\0"
    assert D.marshal_body("at", [[]]) == b"\0\0\0\0" + b"\0" * 4        # padding to 8 is not counted in the length


def test_message_round_trip_with_systemd_signatures():
    props = [("Description", ("s", "x")), ("PIDs", ("au", [1, 2])), ("Delegate", ("b", True)), ("MemoryMax", ("t", 1 << 40)),
             ("Slice", ("s", "kubepods.slice"))]
    msg = D.encode_message(D.METHOD_CALL, 7, {D.F_PATH: CG.SYSTEMD_PATH, D.F_INTERFACE: CG.SYSTEMD_MANAGER,
                                              D.F_MEMBER: "StartTransientUnit", D.F_DESTINATION: CG.SYSTEMD_DEST},
                           "ssa(sv)a(sa(sv))", ["a.scope", "replace", props, [("b.slice", [("X", ("s", "y"))])]])
    assert len(msg) == D.message_length(msg[:16])
    mtype, _flags, serial, fields, body = D.decode_message(msg)
    assert (mtype, serial, fields[D.F_MEMBER], fields[D.F_SIGNATURE]) == (D.METHOD_CALL, 7, "StartTransientUnit",
                                                                         "ssa(sv)a(sa(sv))")
    assert body == ["a.scope", "replace", [tuple(p) for p in props], [("b.slice", [("X", ("s", "y"))])]]
    assert D.split_signature("sa{sv}(ii)aay") == ["s", "a{sv}", "(ii)", "aay"]
    assert D.unmarshal_body("a{sv}", D.marshal_body("a{sv}", [{"k": ("i", -3)}])) == [{"k": ("i", -3)}]


# ------------------------------------------------------------------ a fake systemd on a unix socket
class FakeSystemd:
    """Peer-to-peer (private socket) or bus mode; StartTransientUnit creates the unit's cgroup
    under `root` (slices at their expanded path, scopes inside their Slice=) and moves PIDs."""

    def __init__(self, root: str, bus: bool = True, fail_scopes: bool = False):
        self.root, self.bus, self.fail_scopes = root, bus, fail_scopes
        self.path = os.path.join(tempfile.mkdtemp(prefix="sd", dir="/tmp"), "bus")
        self.calls: list[tuple[str, list]] = []
        self.units: dict[str, str] = {}
        self.srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.srv.bind(self.path)
        self.srv.listen(8)
        self.serial = 100
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        while True:
            try:
                conn, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn):
        buf = b""
        while b"BEGIN\r\n" not in buf:
            chunk = conn.recv(4096)
            if not chunk:
                return
            buf += chunk
            if b"AUTH EXTERNAL " in buf and b"OK" not in buf and buf.endswith(b"\r\n") and b"BEGIN" not in buf:
                hexuid = buf.split(b"AUTH EXTERNAL ")[1].split(b"\r\n")[0]
                assert bytes.fromhex(hexuid.decode()).decode() == str(os.getuid())
                conn.sendall(b"OK 0123456789abcdef0123456789abcdef\r\n")
        buf = buf.split(b"BEGIN\r\n", 1)[1]
        while True:
            while len(buf) < 16:
                chunk = conn.recv(65536)
                if not chunk:
                    return
                buf += chunk
            n = D.message_length(buf[:16])
            while len(buf) < n:
                buf += conn.recv(65536)
            msg, buf = buf[:n], buf[n:]
            _t, _f, serial, fields, body = D.decode_message(msg)
            member = fields.get(D.F_MEMBER)
            self.calls.append((member, body))
            try:
                sig, out = self._handle(member, body)
                self.serial += 1
                conn.sendall(D.encode_message(D.METHOD_RETURN, self.serial, {D.F_REPLY_SERIAL: serial}, sig, out))
            except D.DBusError as e:
                self.serial += 1
                conn.sendall(D.encode_message(D.ERROR, self.serial, {D.F_REPLY_SERIAL: serial, D.F_ERROR_NAME: e.name},
                                              "s", [e.message]))

    def _unit_dir(self, unit: str, props: dict) -> str:
        if unit.endswith(".slice"):
            return os.path.join(self.root, CG.expand_slice(unit).strip("/"))
        parent = props.get("Slice", ("s", "system.slice"))[1]
        return os.path.join(self.root, CG.expand_slice(parent).strip("/"), unit)

    def _handle(self, member, body):
        if member == "Hello":
            assert self.bus
            return "s", [":1.42"]
        if member == "StartTransientUnit":
            unit, mode, props, _aux = body
            props = dict(props)
            assert mode == "replace"
            if unit in self.units:
                raise D.DBusError("org.freedesktop.systemd1.UnitExists", f"Unit {unit} already exists.")
            if unit.endswith(".scope") and self.fail_scopes:
                raise D.DBusError("org.freedesktop.DBus.Error.AccessDenied", "Permission denied")
            d = self._unit_dir(unit, props)
            os.makedirs(d, exist_ok=True)
            for f in ("cgroup.procs", "memory.max", "cpu.max", "cpu.weight", "memory.events"):   # the kernel's files
                open(os.path.join(d, f), "a").close()
            if "PIDs" in props:
                with open(os.path.join(d, "cgroup.procs"), "a") as f:
                    f.write("".join(f"{p}\n" for p in props["PIDs"][1]))
            self.units[unit] = d
            return "o", [f"/org/freedesktop/systemd1/job/{len(self.calls)}"]
        if member == "StopUnit":
            unit, _mode = body
            d = self.units.pop(unit, None)
            if d is None:
                raise D.DBusError("org.freedesktop.systemd1.NoSuchUnit", f"Unit {unit} not loaded.")
            for f in os.listdir(d):
                os.unlink(os.path.join(d, f))
            os.rmdir(d)
            return "o", ["/org/freedesktop/systemd1/job/9"]
        if member == "SetUnitProperties":
            return "", []
        raise D.DBusError("org.freedesktop.DBus.Error.UnknownMethod", f"Unknown method {member}")

    def connect(self):
        return D.Connection(self.path, bus=self.bus).connect()

    def close(self):
        self.srv.close()


@pytest.fixture
def systemd(tmp_path):
    sd = FakeSystemd(str(tmp_path / "cg"))
    yield sd
    sd.close()


def test_connection_errors_and_peer_mode(tmp_path):
    sd = FakeSystemd(str(tmp_path / "cg"), bus=False)
    try:
        conn = D.Connection(sd.path, bus=False).connect()
        assert conn.unique_name == ""                                  # no Hello on a peer socket
        with pytest.raises(D.DBusError) as e:
            conn.call(CG.SYSTEMD_DEST, CG.SYSTEMD_PATH, CG.SYSTEMD_MANAGER, "Reboot")
        assert e.value.name == "org.freedesktop.DBus.Error.UnknownMethod"
        conn.close()
    finally:
        sd.close()


def test_systemd_manager_creates_updates_and_destroys_slices(systemd):
    mgr = CG.CgroupManager(CG.SYSTEMD, systemd.root, units=CG.SystemdUnits(systemd.connect))
    mgr.create("/kubepods", {"memory": 8 << 30, "cpu_quota": 400000, "cpu_period": 100000})
    start = [b for m, b in systemd.calls if m == "StartTransientUnit"][-1]
    assert start[0] == "kubepods.slice"
    props = dict(start[2])
    assert props["MemoryMax"] == ("t", 8 << 30) and props["CPUQuotaPerSecUSec"] == ("t", 4_000_000)
    path = os.path.join(systemd.root, "kubepods.slice")
    assert mgr.exists("/kubepods") and open(os.path.join(path, "memory.max")).read() == str(8 << 30)
    assert open(os.path.join(path, "cpu.max")).read() == "400000 100000"
    mgr.create("/kubepods", {"memory": 4 << 30})                         # exists: properties updated instead
    assert systemd.calls[-1][0] == "SetUnitProperties" and dict(systemd.calls[-1][1][2])["MemoryMax"] == ("t", 4 << 30)
    mgr.create("/kubepods/burstable/pod1-2", {})
    assert os.path.isdir(os.path.join(systemd.root, "kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod1_2.slice"))
    mgr.update("/kubepods/burstable/pod1-2", {"cpu_weight": 50})
    assert systemd.calls[-1] == ("SetUnitProperties", ["kubepods-burstable-pod1_2.slice", True, [("CPUWeight", ("t", 50))]])
    mgr.destroy("/kubepods/burstable/pod1-2")
    assert systemd.calls[-1] == ("StopUnit", ["kubepods-burstable-pod1_2.slice", "replace"])
    assert not mgr.exists("/kubepods/burstable/pod1-2")


def test_enforce_node_allocatable_through_the_systemd_driver(systemd):
    from amdkube.kubelet.cm import enforce_pods_cgroup
    mgr = CG.CgroupManager(CG.SYSTEMD, systemd.root, units=CG.SystemdUnits(systemd.connect))
    assert enforce_pods_cgroup(systemd.root, {"cpu": "1500m", "memory": "2Gi"}, manager=mgr)
    assert open(os.path.join(systemd.root, "kubepods.slice", "cpu.max")).read() == "150000 100000"
    assert dict([b for m, b in systemd.calls if m == "StartTransientUnit"][0][2])["MemoryMax"] == ("t", 2 << 30)
    # cgroupfs keeps its directory layout
    fs_root = os.path.join(systemd.root, "fs")
    assert enforce_pods_cgroup(fs_root, {"memory": "1Gi"})
    assert open(os.path.join(fs_root, "kubepods", "memory.max")).read() == str(1 << 30)


def test_kubelet_refuses_systemd_without_systemd(monkeypatch):
    from amdkube.cmd.components import kubelet
    monkeypatch.delenv("AMDKUBE_SYSTEMD_BUS", raising=False)
    monkeypatch.setattr(CG, "use_systemd", lambda run_dir="/run/systemd/system": False)
    with pytest.raises(SystemExit, match="systemd cgroup manager not available"):
        kubelet(["--cgroup-driver", "systemd", "--node-name", "n"])


# ------------------------------------------------------------------ rocshim: scopes, driver agreement
def _sandbox(uid, parent):
    from amdkube.grpcdesc.cri import CRI as C
    return C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name="p", uid=uid, namespace="default"),
                              labels={"io.kubernetes.pod.uid": uid}, linux=C.LinuxPodSandboxConfig(cgroup_parent=parent))


def _ctr(name, cmd, mem=0):
    from amdkube.grpcdesc.cri import CRI as C
    return C.ContainerConfig(metadata=C.ContainerMetadata(name=name), image=C.ImageSpec(image="busybox"), command=cmd,
                             linux=C.LinuxContainerConfig(resources=C.LinuxContainerResources(memory_limit_in_bytes=mem)))


async def _wait_exit(shim, cid):
    from amdkube.grpcdesc.cri import CRI as C
    for _ in range(500):
        if shim.containers[cid].state == C.CONTAINER_EXITED:
            return shim.containers[cid]
        await asyncio.sleep(0.01)
    raise AssertionError("container did not exit")


@pytest.mark.skipif(os.geteuid() != 0, reason="namespaces isolation needs root")
def test_rocshim_places_containers_in_systemd_scopes(tmp_path):
    from amdkube.runtime import RocShim
    from amdkube.kubelet.qos import cgroup_parent
    sd = FakeSystemd(str(tmp_path / "cg"))

    async def go():
        base = tempfile.mkdtemp(prefix="rsd", dir="/tmp")
        shim = RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks"),
                       isolation="namespaces", cgroup_root=sd.root, cgroup_driver="systemd",
                       systemd_units=CG.SystemdUnits(sd.connect))
        try:
            pod = {"metadata": {"uid": "aa-bb"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "1"}}}]}}
            parent = cgroup_parent(pod, "systemd")
            sc = _sandbox("aa-bb", parent)
            sid = await shim.run_sandbox(sc)
            cid = await shim.create_container(sid, _ctr("c", ["sh", "-c", "echo in-scope"], mem=64 << 20), sc)
            await shim.start_container(cid)
            c = await _wait_exit(shim, cid)
            if c.exit_code == 126 and "unshare" in log_text(c.log_path):
                pytest.skip("unshare not permitted in this container")
            assert c.exit_code == 0, log_text(c.log_path)
            assert log_text(c.log_path).strip() == "in-scope"
            starts = [b for m, b in sd.calls if m == "StartTransientUnit"]
            assert [s[0] for s in starts] == ["kubepods-burstable-podaa_bb.slice", f"amdkube-{cid}.scope"]
            props = dict(starts[1][2])
            assert props["Slice"] == ("s", "kubepods-burstable-podaa_bb.slice") and props["Delegate"] == ("b", True)
            assert props["PIDs"] == ("au", [c.pid]) and props["MemoryMax"] == ("t", 64 << 20)
            leaf = os.path.join(sd.root, "kubepods.slice/kubepods-burstable.slice/kubepods-burstable-podaa_bb.slice",
                                f"amdkube-{cid}.scope")
            assert shim._cgroup_of(c) == leaf
            assert open(os.path.join(leaf, "memory.max")).read() == str(64 << 20)    # nsexec wrote the v2 file too
            await shim.remove_container(cid)
            assert ("StopUnit", [f"amdkube-{cid}.scope", "replace"]) in sd.calls
            await shim.remove_sandbox(sid)
            assert sd.calls[-1] == ("StopUnit", ["kubepods-burstable-podaa_bb.slice", "replace"])
            # systemd refuses the scope: the launcher gets EOF and never runs the workload
            sd.fail_scopes = True
            sid = await shim.run_sandbox(sc)
            cid = await shim.create_container(sid, _ctr("d", ["sh", "-c", "echo must-not-run"]), sc)
            with pytest.raises(RuntimeError, match="Permission denied"):
                await shim.start_container(cid)
            assert "must-not-run" not in log_text(shim.containers[cid].log_path)
            # a non-slice parent is refused under the systemd driver
            with pytest.raises(CG.CgroupError):
                shim._cgroup_parent("kubepods/burstable/podx")
        finally:
            await shim.stop(kill_pods=True)
            sd.close()
    run(go(), 60)


def test_kubelet_checks_the_runtime_cgroup_driver():
    from types import SimpleNamespace
    from amdkube.kubelet.kubelet import Kubelet

    class Cri:
        def __init__(self, driver):
            self.driver = driver

        async def status(self):
            return SimpleNamespace(info={"cgroupDriver": self.driver} if self.driver else {})

    async def go():
        for kubelet_driver, runtime_driver, ok in (("cgroupfs", "cgroupfs", True), ("systemd", "systemd", True),
                                                   ("systemd", "cgroupfs", False), ("cgroupfs", "", True)):
            k = Kubelet.__new__(Kubelet)
            k.cri, k.cfg = Cri(runtime_driver), SimpleNamespace(cgroup_driver=kubelet_driver)
            if ok:
                await k._check_cgroup_driver()
            else:
                with pytest.raises(RuntimeError, match="misconfiguration: kubelet cgroup driver: 'systemd' is different"):
                    await k._check_cgroup_driver()
    run(go())


def test_rocshim_reports_its_cgroup_driver(tmp_path):
    from amdkube.kubelet.cri_client import CRIClient
    from amdkube.runtime import RocShim

    async def go():
        base = tempfile.mkdtemp(prefix="rsd", dir="/tmp")
        shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks"),
                             cgroup_driver="systemd", systemd_units=CG.SystemdUnits(lambda: None)).start()
        cri = await CRIClient(os.path.join(base, "s.sock")).connect()
        try:
            assert dict((await cri.status()).info)["cgroupDriver"] == "systemd"
        finally:
            await cri.close()
            await shim.stop()
    run(go())
    with pytest.raises(CG.CgroupError):
        RocShim(str(tmp_path / "x.sock"), str(tmp_path / "st"), cgroup_driver="openrc")


def test_concurrent_scope_starts_share_one_connection(tmp_path):
    """Many containers starting at once (rocshim's asyncio.to_thread calls) share one systemd
    connection: every call gets its own reply and every scope is created exactly once."""
    from concurrent.futures import ThreadPoolExecutor
    sd = FakeSystemd(str(tmp_path / "cg"))
    units = CG.SystemdUnits(connect=lambda: D.Connection(sd.path, timeout=3).connect())
    try:
        names = [f"cri-containerd-{i:02d}.scope" for i in range(24)]
        with ThreadPoolExecutor(max_workers=12) as ex:
            jobs = list(ex.map(lambda n: units.start_transient(n, [("Slice", ("s", "kubepods.slice")),
                                                                     ("PIDs", ("au", [os.getpid()]))]), names))
        assert len(jobs) == len(names) and all(j.startswith("/org/freedesktop/systemd1/job/") for j in jobs)
        assert sorted(sd.units) == sorted(names)
        assert [m for m, _ in sd.calls].count("StartTransientUnit") == len(names)    # no resend after a lost reply
    finally:
        units.close()
        sd.close()


def test_systemd_cgroup_root_is_the_cgroup2_mount(tmp_path):
    mi = tmp_path / "mountinfo"
    mi.write_text("22 1 0:21 / /sys rw,nosuid - sysfs sysfs rw\n"
                  "30 22 0:26 / /sys/fs/cgroup rw,nosuid,nodev - cgroup2 cgroup2 rw,nsdelegate\n"
                  "40 1 0:40 / /mnt/cg\\040two rw - cgroup2 none rw\n")
    assert CG.cgroup2_mount_of("/sys/fs/cgroup/amdkube/x", str(mi)) == "/sys/fs/cgroup"
    assert CG.cgroup2_mount_of("/mnt/cg two/a", str(mi)) == "/mnt/cg two"
    assert CG.cgroup2_mount_of("/sys/fs/cgroupx", str(mi)) is None
    assert CG.systemd_cgroup_root("/sys/fs/cgroup", str(mi)) == "/sys/fs/cgroup"
    assert CG.systemd_cgroup_root(CG.RUNTIME_DEFAULT_ROOT, str(mi)) == "/sys/fs/cgroup"     # rocshim's default, remapped
    assert CG.systemd_cgroup_root(str(tmp_path), str(mi)) == str(tmp_path)                  # no cgroup2 fs: a test tree
    with pytest.raises(CG.CgroupError, match="is not the cgroup2 mount /sys/fs/cgroup"):
        CG.systemd_cgroup_root("/sys/fs/cgroup/kubelet", str(mi))


def test_kubelet_enforces_the_pods_cgroup_off_its_event_loop():
    """A slow pods-cgroup create (systemd answering late, its directory appearing late) runs in a
    worker thread: the kubelet's loop keeps turning, a second status update does not start a
    second create, and a failed create is retried on a later update."""
    import time
    from types import SimpleNamespace
    from amdkube.kubelet.kubelet import Kubelet

    class SlowManager:
        def __init__(self):
            self.creates, self.fail = 0, True

        def path(self, internal):
            return "/x" + internal

        def create(self, internal, res):
            self.creates += 1
            time.sleep(0.3)
            if self.fail:
                self.fail = False
                raise CG.CgroupError("systemd did not create the slice")

    async def go():
        k = Kubelet.__new__(Kubelet)
        k.cfg = SimpleNamespace(cgroup_root="/cg", enforce_node_allocatable="pods", cgroup_driver="systemd")
        k._pods_cgroup_enforced, k._cgroup_task, k._cgroup_manager = None, None, SlowManager()
        alloc = {"cpu": "3", "memory": "1Gi"}
        ticks = 0

        async def ticker():
            nonlocal ticks
            while True:
                ticks += 1
                await asyncio.sleep(0.01)
        t = asyncio.get_running_loop().create_task(ticker())
        task = k._enforce_pods_cgroup(alloc)
        assert task is not None and k._enforce_pods_cgroup(alloc) is None      # one at a time
        await task
        assert ticks >= 10 and k._pods_cgroup_enforced is None                  # the loop ran; the create failed
        await k._enforce_pods_cgroup(alloc)                                     # retried on the next update
        assert k._pods_cgroup_enforced == ("3", "1Gi") and k._cgroup_manager.creates == 2
        assert k._enforce_pods_cgroup(alloc) is None                            # nothing changed: nothing to do
        t.cancel()
    run(go())


def test_launcher_gone_before_its_scope_is_joined(tmp_path):
    """nsexec exits before the kubelet's go-ahead: the write end of the wait pipe is closed, the
    launcher reaped, the scope made for it stopped, and the start fails."""
    from types import SimpleNamespace
    from amdkube.runtime import RocShim

    async def go():
        base = tempfile.mkdtemp(prefix="rsd", dir="/tmp")
        shim = RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks"),
                       cgroup_driver="systemd", systemd_units=CG.SystemdUnits(lambda: None))
        stopped, waited, fds = [], [], []

        class Proc:
            pid = 4242

            async def wait(self):
                waited.append(True)
                return 1

        async def launch(argv, **kw):
            fds.append(int(argv[argv.index("--cgroup-wait-fd") + 1]))
            return Proc()
        shim._launch = launch
        shim._place_in_scope = lambda c, pid: None
        shim.systemd.stop = lambda unit: stopped.append(unit)
        before = set(os.listdir("/proc/self/fd"))
        c = SimpleNamespace(id="c1", env={}, cwd="/", log_path=os.path.join(base, "log"))
        with pytest.raises(RuntimeError, match="launcher exited before joining its scope"):
            await shim._launch_in_scope(c, ["nsexec", "--", "true"])
        assert waited and stopped == ["amdkube-c1.scope"]
        assert set(os.listdir("/proc/self/fd")) <= before          # neither pipe end leaks
    run(go())
