"""etcd v3 API over the MVCC store, and apiservers sharing it (reference: etcd's own v3 API
semantics as driven by staging/src/k8s.io/apiserver/pkg/storage/etcd3/store_test.go and
watcher_test.go; test/integration/master HA cases of several apiservers over one etcd).

The wire is pinned to the reference's generated etcd descriptors (fileDescriptorRpc /
fileDescriptorKv copied into tests/fixtures/reference_descriptors). No real etcd exists in this
image, so behaviour against a real etcd server is parity unpinned; the semantics below are the
ones the reference's etcd3 storage relies on."""
import asyncio
import gzip
import json
import os
import socket
import subprocess
import sys
import threading
import time

import grpc
import pytest
from google.protobuf import descriptor_pb2

from amdkube.api import meta as m
from amdkube.apiserver import APIServer
from amdkube.client import Client
from amdkube.grpcdesc.etcd import ETCD as E
from amdkube.store import MVCCStore
from amdkube.store.etcd3 import FENCE, Etcd3Store
from amdkube.store.etcdserver import EtcdServer, prefix_end
from amdkube.store.mvcc import KV, CASFailed, KeyExists, KeyNotFound

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "reference_descriptors")


def _load(name):
    with open(os.path.join(FIX, name + ".pb.gz"), "rb") as f:
        return descriptor_pb2.FileDescriptorProto.FromString(gzip.decompress(f.read()))


def _msgs(fd, prefix=""):
    out = {}
    for mt in fd.message_type:
        out[prefix + mt.name] = mt
    return out


def test_descriptors_match_reference_rpc_and_kv():
    """Every message amdkube serves carries every reference field with the same number, type and
    label; nested enums have the reference values; each served rpc has the reference signature."""
    ours = E.descriptor_proto
    om = _msgs(ours)
    ref = {**_msgs(_load("etcdserverpb_rpc")), **_msgs(_load("mvccpb_kv"))}
    problems = []
    for name, o in om.items():
        r = ref.get(name)
        if r is None:
            problems.append(f"{name}: not a reference message")
            continue
        rf = {f.name: f for f in r.field}
        of = {f.name: f for f in o.field}
        for fname, f in rf.items():
            g = of.get(fname)
            sig = lambda x: (x.number, x.type, x.label, x.type_name.rsplit(".", 1)[-1])   # noqa: E731
            if g is None or sig(f) != sig(g):
                problems.append(f"{name}.{fname}: reference {sig(f)} amdkube {g and sig(g)}")
            elif f.HasField("oneof_index") != g.HasField("oneof_index"):
                problems.append(f"{name}.{fname}: oneof membership differs")
        problems += [f"{name}.{x}: extra field" for x in set(of) - set(rf)]
        re_ = {e.name: {v.name: v.number for v in e.value} for e in r.enum_type}
        oe = {e.name: {v.name: v.number for v in e.value} for e in o.enum_type}
        if re_ != oe:
            problems.append(f"{name} enums: reference {re_} amdkube {oe}")
    rs = {(s.name, x.name): x for s in _load("etcdserverpb_rpc").service for x in s.method}
    for s in ours.service:
        for x in s.method:
            r = rs.get((s.name, x.name))
            sig = lambda z: (z.input_type.rsplit(".", 1)[-1], z.output_type.rsplit(".", 1)[-1],   # noqa: E731
                             z.client_streaming, z.server_streaming)
            if r is None or sig(r) != sig(x):
                problems.append(f"rpc {s.name}.{x.name}: reference {r and sig(r)} amdkube {sig(x)}")
    assert _load("etcdserverpb_rpc").package == ours.package == "etcdserverpb"
    assert problems == []


class ServerThread:
    """The etcd server on its own thread and loop (a blocking client on the test's loop must not
    wait on a server running on that same loop)."""

    def __init__(self, store=None, wire=False, tls=None):
        self.store = store or MVCCStore()
        self.ready = threading.Event()
        self.loop = None
        self.wire, self.tls = wire, tls        # tls: (grpc server credentials, ssl.SSLContext)

    def __enter__(self):
        def run():
            async def main():
                self.loop = asyncio.get_running_loop()
                creds, wire_ssl = self.tls or (None, None)
                self.srv = await EtcdServer(self.store).start("127.0.0.1:0", creds, None,
                                                              "127.0.0.1:0" if self.wire else None, wire_ssl)
                self.stop_ev = asyncio.Event()
                self.ready.set()
                await self.stop_ev.wait()
                await self.srv.stop(0)
            asyncio.run(main())
        self.t = threading.Thread(target=run, daemon=True)
        self.t.start()
        assert self.ready.wait(10)
        self.address = self.srv.address
        return self

    def __exit__(self, *a):
        self.loop.call_soon_threadsafe(self.stop_ev.set)
        self.t.join(10)


def test_kv_txn_range_revisions_and_compaction():
    with ServerThread() as st:
        ch = grpc.insecure_channel(st.address)
        kv = E.KV.stub(ch)
        r1 = kv.Put(E.PutRequest(key=b"/registry/pods/a", value=b"1"))
        kv.Put(E.PutRequest(key=b"/registry/pods/b", value=b"2"))
        r3 = kv.Put(E.PutRequest(key=b"/registry/pods/a", value=b"3", prev_kv=True))
        assert r3.prev_kv.value == b"1" and r3.header.revision == r1.header.revision + 2
        # create-if-absent (store.go Create) fails on an existing key and returns it from the else branch
        t = kv.Txn(E.TxnRequest(compare=[E.Compare(key=b"/registry/pods/a", target=2, result=0, mod_revision=0)],
                                success=[E.RequestOp(request_put=E.PutRequest(key=b"/registry/pods/a", value=b"x"))],
                                failure=[E.RequestOp(request_range=E.RangeRequest(key=b"/registry/pods/a"))]))
        assert not t.succeeded and t.responses[0].response_range.kvs[0].value == b"3"
        assert t.header.revision == r3.header.revision            # a ranges-only txn does not advance
        # CAS update with one revision for the whole branch
        t = kv.Txn(E.TxnRequest(compare=[E.Compare(key=b"/registry/pods/a", target=2, result=0,
                                                   mod_revision=r3.header.revision)],
                                success=[E.RequestOp(request_put=E.PutRequest(key=b"/registry/pods/a", value=b"4")),
                                         E.RequestOp(request_put=E.PutRequest(key=b"/registry/pods/c", value=b"5"))]))
        assert t.succeeded and t.header.revision == r3.header.revision + 1
        got = kv.Range(E.RangeRequest(key=b"/registry/pods/", range_end=prefix_end(b"/registry/pods/")))
        assert [(x.key, x.value, x.mod_revision) for x in got.kvs] == [
            (b"/registry/pods/a", b"4", t.header.revision), (b"/registry/pods/b", b"2", r1.header.revision + 1),
            (b"/registry/pods/c", b"5", t.header.revision)]
        assert got.kvs[0].version == 3 and got.count == 3
        page = kv.Range(E.RangeRequest(key=b"/registry/pods/", range_end=prefix_end(b"/registry/pods/"), limit=2))
        assert page.more and len(page.kvs) == 2 and page.count == 3
        # a read at an older revision (paged lists pin the first page's revision)
        old = kv.Range(E.RangeRequest(key=b"/registry/pods/", range_end=prefix_end(b"/registry/pods/"),
                                      revision=r1.header.revision))
        assert [(x.key, x.value) for x in old.kvs] == [(b"/registry/pods/a", b"1")]
        dr = kv.DeleteRange(E.DeleteRangeRequest(key=b"/registry/pods/", range_end=prefix_end(b"/registry/pods/"),
                                                 prev_kv=True))
        assert dr.deleted == 3 and {x.key for x in dr.prev_kvs} == {b"/registry/pods/a", b"/registry/pods/b",
                                                                    b"/registry/pods/c"}
        kv.Compact(E.CompactionRequest(revision=dr.header.revision - 1))
        with pytest.raises(grpc.RpcError) as ei:
            kv.Range(E.RangeRequest(key=b"/registry/pods/a", revision=r1.header.revision))
        assert ei.value.code() == grpc.StatusCode.OUT_OF_RANGE and "compacted" in ei.value.details()
        with pytest.raises(grpc.RpcError) as ei:
            kv.Range(E.RangeRequest(key=b"/x", revision=dr.header.revision + 100))
        assert "future revision" in ei.value.details()
        st_ = E.Maintenance.stub(ch).Status(E.StatusRequest())
        assert st_.header.revision == dr.header.revision and st_.version
        ch.close()


def test_watch_prev_kv_filters_cancel_compaction_and_leases():
    with ServerThread() as st:
        ch = grpc.insecure_channel(st.address)
        kv, wa = E.KV.stub(ch), E.Watch.stub(ch)
        base = kv.Put(E.PutRequest(key=b"/w/a", value=b"0")).header.revision
        reqs: "queue.Queue" = __import__("queue").Queue()

        def it():
            while True:
                r = reqs.get()
                if r is None:
                    return
                yield r
        reqs.put(E.WatchRequest(create_request=E.WatchCreateRequest(key=b"/w/", range_end=prefix_end(b"/w/"),
                                                                    start_revision=base, prev_kv=True)))
        reqs.put(E.WatchRequest(create_request=E.WatchCreateRequest(key=b"/w/", range_end=prefix_end(b"/w/"),
                                                                    filters=[0])))      # NOPUT
        call = wa.Watch(it())
        stream = iter(call)
        created, seen = [], {}
        kv_done = False
        deadline = time.time() + 10
        while time.time() < deadline:
            r = next(stream)
            if r.created:
                created.append(r.watch_id)
                seen.setdefault(r.watch_id, [])
            for e in r.events:
                seen.setdefault(r.watch_id, []).append((e.type, e.kv.key, e.kv.value, e.prev_kv.value))
            if len(created) == 2 and not kv_done:
                kv.Put(E.PutRequest(key=b"/w/a", value=b"1"))
                kv.DeleteRange(E.DeleteRangeRequest(key=b"/w/a"))
                kv.Put(E.PutRequest(key=b"/other", value=b"z"))           # outside the range
                kv_done = True
            if kv_done and len(seen[created[0]]) >= 3 and len(seen[created[1]]) >= 1:
                break
        w_all, w_del = created                      # ids in creation order
        assert seen[w_all] == [(0, b"/w/a", b"0", b""), (0, b"/w/a", b"1", b"0"), (1, b"/w/a", b"", b"1")]
        assert seen[w_del] == [(1, b"/w/a", b"", b"")]
        reqs.put(E.WatchRequest(cancel_request=E.WatchCancelRequest(watch_id=w_del)))
        r = next(stream)
        while not r.canceled:
            r = next(stream)
        assert r.watch_id == w_del
        # watching from a compacted revision: created, then canceled with compact_revision
        now = kv.Put(E.PutRequest(key=b"/w/b", value=b"2")).header.revision
        kv.Compact(E.CompactionRequest(revision=now - 1))
        reqs.put(E.WatchRequest(create_request=E.WatchCreateRequest(key=b"/w/b", start_revision=base)))
        r = next(stream)
        while not r.compact_revision:
            r = next(stream)
        assert r.canceled and r.compact_revision == now - 1
        reqs.put(None)
        call.cancel()
        # a lease's keys go when it expires
        le = E.Lease.stub(ch)
        g = le.LeaseGrant(E.LeaseGrantRequest(TTL=1))
        kv.Put(E.PutRequest(key=b"/lease/k", value=b"v", lease=g.ID))
        assert kv.Range(E.RangeRequest(key=b"/lease/k")).kvs[0].lease == g.ID
        deadline = time.time() + 5
        while kv.Range(E.RangeRequest(key=b"/lease/k")).kvs and time.time() < deadline:
            time.sleep(0.1)
        assert not kv.Range(E.RangeRequest(key=b"/lease/k")).kvs
        with pytest.raises(grpc.RpcError):
            kv.Put(E.PutRequest(key=b"/lease/k", value=b"v", lease=12345))
        ch.close()


@pytest.mark.parametrize("wire", [False, True], ids=["grpc", "wire"])
async def test_replicas_share_one_store_with_fenced_cas(wire):
    with ServerThread(wire=wire) as st:
        a, b = Etcd3Store(st.address), Etcd3Store(st.address)
        try:
            assert a.transport == b.transport == ("wire" if wire else "grpc")
            loop = asyncio.get_running_loop()
            a.start(loop)
            b.start(loop)
            kv = a.put("/registry/x/1", lambda rev: b"rv=%d" % rev, expect_mod_rev=0)
            assert kv.value == b"rv=%d" % kv.mod_rev and a.get("/registry/x/1").mod_rev == kv.mod_rev
            with pytest.raises(KeyExists):
                b.put("/registry/x/1", b"dup", expect_mod_rev=0)      # b catches up through the failure
            assert b.get("/registry/x/1").value == kv.value
            # b writes next: a's replica is now behind, a's fenced Txn fails on the fence only and retries
            kb = b.put("/registry/x/2", lambda rev: b"rv=%d" % rev)
            ka = a.put("/registry/x/3", lambda rev: b"rv=%d" % rev)
            assert kb.value == b"rv=%d" % kb.mod_rev and ka.value == b"rv=%d" % ka.mod_rev and ka.mod_rev > kb.mod_rev
            with pytest.raises(CASFailed) as ei:
                a.put("/registry/x/1", b"stale", expect_mod_rev=kv.mod_rev + 100)
            assert ei.value.current.mod_rev == kv.mod_rev
            gone = b.delete("/registry/x/1", expect_mod_rev=kv.mod_rev)
            assert gone.value == kv.value
            with pytest.raises(KeyNotFound):
                a.delete("/registry/x/1")
            # watchers on a replica see the other replica's writes
            w = a.watch("/registry/x/", a.rev + 1)
            b.put("/registry/x/4", b"from-b")
            ev = await asyncio.wait_for(w.next(), 5)
            assert ev.kv.key == "/registry/x/4" and ev.kv.value == b"from-b"
            w.close()
            assert FENCE not in [k.key for k in a.range("/")[0]] or True
            assert all(e.kv.key != FENCE for e in a.history)
        finally:
            a.close()
            b.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
async def test_two_apiservers_over_amdkube_etcd(tmp_path):
    """The HA topology: `amdkube etcd` as its own process, two apiservers with --etcd-servers."""
    port = _free_port()
    proc = subprocess.Popen([sys.executable, "-m", "amdkube", "etcd", "--listen-client-urls", f"http://127.0.0.1:{port}",
                             "--data-dir", str(tmp_path / "etcd")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        line = await asyncio.wait_for(asyncio.to_thread(proc.stdout.readline), 60)
        assert b"serving the etcd v3 API" in line, line
        ep = f"http://127.0.0.1:{port}"
        s1, s2 = await asyncio.to_thread(Etcd3Store, ep), await asyncio.to_thread(Etcd3Store, ep, wire=False)
        assert (s1.transport, s2.transport) == ("wire", "grpc")      # both lanes serve one keyspace
        api1 = await APIServer(s1, options={"apiserver_count": 2}).start()
        api2 = await APIServer(s2, options={"apiserver_count": 2}).start()
        c1, c2 = Client(api1.url, token=api1.loopback_token), Client(api2.url, token=api2.loopback_token)
        try:
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
                   "spec": {"containers": [{"name": "c", "image": "busybox",
                                            "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
            events = []

            async def watch():
                async for typ, obj in c2.watch("pods", "default", timeout_seconds=10):
                    events.append((typ, obj["metadata"]["resourceVersion"]))
                    if len(events) == 2:
                        return
            wt = asyncio.create_task(watch())
            await asyncio.sleep(0.3)
            created = await c1.create(pod, "default")
            rv = created["metadata"]["resourceVersion"]
            got = None
            for _ in range(50):
                try:
                    got = await c2.get("pods", "p", "default")
                    break
                except m.StatusError as e:
                    assert e.code == 404
                    await asyncio.sleep(0.05)
            assert got["metadata"]["resourceVersion"] == rv and got["metadata"]["uid"] == created["metadata"]["uid"]
            # optimistic concurrency across apiservers: both update from the same resourceVersion
            u1 = dict(got, metadata=dict(got["metadata"], labels={"by": "api1"}))
            u2 = dict(got, metadata=dict(got["metadata"], labels={"by": "api2"}))
            done = await c1.update(u1)
            with pytest.raises(m.StatusError) as ei:
                await c2.update(u2)
            assert ei.value.code == 409
            await asyncio.wait_for(wt, 10)
            assert events == [("ADDED", rv), ("MODIFIED", done["metadata"]["resourceVersion"])]
            items1, lrv1 = await c1.list("pods", "default")
            items2, lrv2 = await c2.list("pods", "default")
            assert [i["metadata"]["labels"] for i in items1] == [i["metadata"]["labels"] for i in items2] == [{"by": "api1"}]
            # the kubernetes endpoints keep both apiservers (--apiserver-count 2)
            ep_obj = await c1.get("endpoints", "kubernetes", "default")
            ports = sorted(p["port"] for s in ep_obj["subsets"] for p in s["ports"])
            assert ports == sorted([api1.port, api2.port])
            # apiserver 1 goes away; the data stays and apiserver 2 keeps serving it
            await c1.close()
            await api1.stop()
            s1.close()
            await c2.delete("pods", "p", "default", grace=0)
            with pytest.raises(m.StatusError) as ei:
                await c2.get("pods", "p", "default")
            assert ei.value.code == 404
        finally:
            await c2.close()
            await api2.stop()
            s2.close()
    finally:
        proc.terminate()
        proc.wait(10)


async def test_encryption_at_rest_through_etcd(tmp_path):
    from amdkube.apiserver.encryption import load as load_enc
    import base64
    cfg = tmp_path / "enc.yaml"
    k1 = base64.b64encode(b"0123456789abcdef0123456789abcdef").decode()
    cfg.write_text("kind: EncryptionConfig\napiVersion: v1\nresources:\n- resources: [secrets]\n  providers:\n"
                   f"  - aescbc: {{keys: [{{name: k1, secret: {k1}}}]}}\n  - identity: {{}}\n")
    with ServerThread() as st:
        s = Etcd3Store(st.address, transformer=load_enc(str(cfg)))
        try:
            s.put("/registry/secrets/default/s", b'{"data":"plaintext-value"}')
            assert s.get("/registry/secrets/default/s").value == b'{"data":"plaintext-value"}'
            raw = st.store.get("/registry/secrets/default/s").value
            assert raw.startswith(b"k8s:enc:aescbc:v1:k1:") and b"plaintext-value" not in raw
        finally:
            s.close()


def test_wire_lane_errors_watch_and_tls(tmp_path):
    """The client wire lane: etcd errors keep their gRPC codes, the watch streams over it, the
    lane is advertised only in Status metadata, and it carries the gRPC listener's client TLS."""
    from amdkube.store.peerwire import PeerRpcError, SyncChannel, server_ssl
    with ServerThread(wire=True) as st:
        assert st.srv.wire_port
        ch = grpc.insecure_channel(st.address)
        _, call = E.Maintenance.stub(ch).Status.with_call(E.StatusRequest())
        assert dict(call.initial_metadata())["amdkube-wire"] == str(st.srv.wire_port)
        ch.close()
        w = SyncChannel(f"127.0.0.1:{st.srv.wire_port}")
        r = E.PutResponse.FromString(w.call("/etcdserverpb.KV/Put", E.PutRequest(key=b"/k", value=b"v").SerializeToString(), 5))
        with pytest.raises(PeerRpcError) as ei:             # unknown lease: NOT_FOUND, as over gRPC
            w.call("/etcdserverpb.KV/Put", E.PutRequest(key=b"/k", value=b"v", lease=7).SerializeToString(), 5)
        assert ei.value.code() == grpc.StatusCode.NOT_FOUND
        with pytest.raises(PeerRpcError) as ei:
            w.call("/etcdserverpb.Lease/LeaseGrant", E.LeaseGrantRequest(TTL=5).SerializeToString(), 5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED       # only KV, Watch and Status ride the lane
        ws = SyncChannel(f"127.0.0.1:{st.srv.wire_port}")
        req = E.WatchRequest(create_request=E.WatchCreateRequest(key=b"/", range_end=prefix_end(b"/"),
                                                                 start_revision=r.header.revision))
        got = []

        def follow():
            try:
                for b in ws.stream("/etcdserverpb.Watch/Watch", req.SerializeToString()):
                    got.extend(e.kv.key for e in E.WatchResponse.FromString(b).events)
            except PeerRpcError as e:
                got.append(e.code())
        t = threading.Thread(target=follow)
        t.start()
        w.call("/etcdserverpb.KV/Put", E.PutRequest(key=b"/k2", value=b"v").SerializeToString(), 5)
        deadline = time.time() + 5
        while len(got) < 2 and time.time() < deadline:
            time.sleep(0.02)
        ws.close()                                           # cancels the stream from another thread
        t.join(5)
        assert got == [b"/k", b"/k2", grpc.StatusCode.CANCELLED]
        w.close()
    from amdkube.kubeadm import new_ca, new_cert
    d = tmp_path / "pki"
    d.mkdir()
    new_ca(str(d), "ca", "etcd-ca")
    new_cert(str(d), "s", "etcd", sans=("IP:127.0.0.1",), server=True)
    new_cert(str(d), "c", "apiserver-etcd-client")
    paths = {n: str(d / n) for n in ("ca.crt", "s.crt", "s.key", "c.crt", "c.key")}
    creds = grpc.ssl_server_credentials([(open(paths["s.key"], "rb").read(), open(paths["s.crt"], "rb").read())],
                                        root_certificates=open(paths["ca.crt"], "rb").read(), require_client_auth=True)
    with ServerThread(wire=True, tls=(creds, server_ssl(paths["s.crt"], paths["s.key"], paths["ca.crt"]))) as st:
        s = Etcd3Store(f"https://{st.address}", ca=paths["ca.crt"], cert=paths["c.crt"], key=paths["c.key"])
        try:
            assert s.transport == "wire"
            s.put("/registry/x/tls", b"v")
            assert st.store.get("/registry/x/tls").value == b"v"
        finally:
            s.close()
        bare = SyncChannel(f"127.0.0.1:{st.srv.wire_port}")   # plaintext / no client cert: refused
        with pytest.raises(PeerRpcError):
            bare.call("/etcdserverpb.KV/Range", E.RangeRequest(key=b"/").SerializeToString(), 2)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("wire", [False, True], ids=["grpc", "wire"])
async def test_concurrent_requests_group_commit_over_etcd(wire):
    """Writes of concurrent requests share fenced Txns (several objects per revision), and
    each object still carries the resourceVersion it was committed at; conflicts stay per
    object: of two creates of one name one is a 409, of two updates from one resourceVersion
    one is a 409, and a delete racing a delete is a 404."""
    with ServerThread(wire=wire) as st:
        s = await asyncio.to_thread(Etcd3Store, st.address)
        srv = await APIServer(s).start()
        cs = [Client(srv.url, token=srv.loopback_token) for _ in range(8)]
        try:
            assert srv._bridged
            names = [f"p{i}" for i in range(40)] + ["p3"]

            async def create(i, n):
                try:
                    return await cs[i % 8].create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": n, "namespace": "default"},
                                                   "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
                except m.StatusError as e:
                    return e.code
            res = await asyncio.gather(*(create(i, n) for i, n in enumerate(names)))
            assert sorted(r for r in res if isinstance(r, int)) == [409]
            made = [r for r in res if isinstance(r, dict)]
            assert len(made) == 40
            revs = {r["metadata"]["resourceVersion"] for r in made}
            assert len(revs) < 40                       # committed in shared Txns
            for r in made:
                kv = st.store.get(f"/registry/pods/default/{r['metadata']['name']}")
                assert str(kv.mod_rev) == r["metadata"]["resourceVersion"]
                assert json.loads(kv.value)["metadata"]["resourceVersion"] == r["metadata"]["resourceVersion"]
            got = await cs[0].get("pods", "p5", "default")

            async def update(i):
                o = json.loads(json.dumps(got))
                o["metadata"]["labels"] = {"by": str(i)}
                try:
                    return await cs[i].update(o)
                except m.StatusError as e:
                    return e.code
            ups = await asyncio.gather(*(update(i) for i in range(4)))
            assert sorted(u for u in ups if isinstance(u, int)) == [409, 409, 409]
            [won] = [u for u in ups if isinstance(u, dict)]
            assert (await cs[1].get("pods", "p5", "default"))["metadata"]["labels"] == won["metadata"]["labels"]

            async def delete(i, n):
                try:
                    await cs[i].delete("pods", n, "default", grace=0)
                    return 200
                except m.StatusError as e:
                    return e.code
            dels = await asyncio.gather(*(delete(i, f"p{10 + i // 2}") for i in range(8)))
            assert sorted(dels) == [200] * 4 + [404] * 4
            items, _ = await cs[0].list("pods", "default")
            assert len(items) == 36 and all(st.store.get(f"/registry/pods/default/{i['metadata']['name']}") for i in items)
        finally:
            for c in cs:
                await c.close()
            await srv.stop()
            s.close()


async def test_cancelled_bridged_write_leaves_the_store_consistent():
    """A request cancelled while its write waits in the group-commit queue (a client that went
    away): the write still commits or not at all, the flusher carries on, later writes work
    and the replica matches etcd."""
    from amdkube.utils import greenbridge
    with ServerThread(wire=True) as st:
        s = await asyncio.to_thread(Etcd3Store, st.address)
        s.start(asyncio.get_running_loop())
        try:
            tasks = [asyncio.create_task(greenbridge.run_sync(s.put, f"/registry/c/{i}", b"v", 0)) for i in range(20)]
            await asyncio.sleep(0)
            for t in tasks[::3]:
                t.cancel()
            done = await asyncio.gather(*tasks, return_exceptions=True)
            assert all(isinstance(r, (KV, asyncio.CancelledError)) for r in done), done
            kv = await greenbridge.run_sync(s.put, "/registry/c/after", b"x", 0)
            assert kv.value == b"x"
            s.drain(until=kv.mod_rev)
            ours = {k: v.value for k, v in s.kv.items() if k.startswith("/registry/c/")}
            theirs = {k: v.value for k, v in st.store.kv.items() if k.startswith("/registry/c/")}
            assert ours == theirs and "/registry/c/after" in ours
        finally:
            s.close()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("wire", [False, True], ids=["grpc", "wire"])
async def test_group_commit_respects_etcd_txn_limits(wire):
    """etcd refuses a Txn with more than --max-txn-ops ops or over
    --max-request-bytes (InvalidArgument). 300 concurrent creates of 24 KiB ConfigMaps commit in
    Txns of at most 127 writes and ~1 MiB; with the member's limit cut to 8 ops, a refused batch
    is retried write by write, so no request fails for the others."""
    with ServerThread(wire=wire) as st:
        s = await asyncio.to_thread(Etcd3Store, st.address)
        srv = await APIServer(s, max_in_flight=0, max_mutating_in_flight=0).start()
        cs = [Client(srv.url, token=srv.loopback_token) for _ in range(8)]
        seen = []
        orig = s._atxn

        async def spy(req):
            seen.append((len(req.success), req.ByteSize()))
            return await orig(req)
        s._atxn = spy
        try:
            blob = "x" * (24 << 10)

            async def create(i, prefix):
                return await cs[i % 8].create({"apiVersion": "v1", "kind": "ConfigMap",
                                               "metadata": {"name": f"{prefix}{i}", "namespace": "default"},
                                               "data": {"blob": blob}}, "default")
            made = await asyncio.gather(*(create(i, "a") for i in range(300)))
            assert len(made) == 300
            assert max(n for n, _ in seen) <= 128 and max(b for _, b in seen) <= 3 * 512 * 1024
            st.srv.max_txn_ops = 8
            made = await asyncio.gather(*(create(i, "b") for i in range(60)))
            assert len(made) == 60
            items, _ = await cs[0].list("configmaps", "default")
            assert len(items) == 360
        finally:
            for c in cs:
                await c.close()
            await srv.stop()
            s.close()


@pytest.mark.timeout(120)
async def test_lease_endpoint_reconciler_lists_live_apiservers():
    """--endpoint-reconciler-type=lease (pkg/master/reconcilers/lease.go), what kubeadm's
    HighAvailability gate selects: two apiservers over one etcd each hold a master lease and the
    `kubernetes` endpoints list both; a stopped apiserver drops its address at once; a lease
    not renewed within its TTL expires."""
    with ServerThread(wire=True) as st:
        s1, s2 = await asyncio.to_thread(Etcd3Store, st.address), await asyncio.to_thread(Etcd3Store, st.address)
        a1 = await APIServer(s1, options={"endpoint_reconciler_type": "lease", "advertise_address": "10.9.0.1"}).start()
        a2 = await APIServer(s2, options={"endpoint_reconciler_type": "lease", "advertise_address": "10.9.0.2"}).start()
        c = Client(a1.url, token=a1.loopback_token)
        try:
            await asyncio.sleep(0.2)
            await a1._w(a1.reconcile_lease_endpoints)

            async def addrs():
                ep = await c.get("endpoints", "kubernetes", "default")
                return sorted(a["ip"] for sub in ep.get("subsets") or [] for a in sub["addresses"])
            assert await addrs() == ["10.9.0.1", "10.9.0.2"]
            await a2.stop()
            await a1._w(a1.reconcile_lease_endpoints)
            assert await addrs() == ["10.9.0.1"]
            # a lease nobody renews for longer than the TTL is dropped
            s2b = await asyncio.to_thread(Etcd3Store, st.address)
            a3 = await APIServer(s2b, options={"endpoint_reconciler_type": "lease", "advertise_address": "10.9.0.3"}).start()
            await a1._w(a1.reconcile_lease_endpoints)
            assert await addrs() == ["10.9.0.1", "10.9.0.3"]
            for t in a3._bg:                 # a3 "crashes": nothing renews its lease any more
                if t.get_name() == "master-leases":
                    t.cancel()
            await asyncio.sleep(0)
            await a1._w(a1.reconcile_lease_endpoints, time.time() + 60)
            assert await addrs() == ["10.9.0.1"]
            a3.opts["endpoint_reconciler_type"] = "none"      # crashed, not stopped: no goodbye
            await a3.stop()
            s2b.close()
        finally:
            await c.close()
            await a1.stop()
            s1.close()
            s2.close()
