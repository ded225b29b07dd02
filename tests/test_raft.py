"""A 3-member `amdkube etcd` raft group (reference role: the etcd cluster under the apiservers;
the raft behaviour itself follows the Raft paper — leader election, log replication, commit by
majority, InstallSnapshot — and is checked here end to end with real processes):

* one leader; writes through any member land on all of them at the same revisions;
* a linearizable read on a follower is answered by the leader;
* the leader is killed: a new one is elected and a client with every endpoint carries on,
  including its watch;
* the killed member restarts from its data dir, far enough behind that the compacted log
  forces an InstallSnapshot, and converges on the same keyspace and revision.
"""
import asyncio
import os
import signal
import socket
import subprocess
import sys
import time

import grpc
import pytest

from amdkube.grpcdesc.etcd import ETCD as E
from amdkube.store.etcd3 import Etcd3Store
from amdkube.store.etcdserver import _hash_id, prefix_end


def _ports(n):
    socks, out = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        out.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return out


class Cluster:
    def __init__(self, tmp, n=3):
        ports = _ports(2 * n)
        self.names = [f"m{i}" for i in range(n)]
        self.client = {nm: f"127.0.0.1:{ports[i]}" for i, nm in enumerate(self.names)}
        self.peer = {nm: f"127.0.0.1:{ports[n + i]}" for i, nm in enumerate(self.names)}
        self.tmp, self.procs = tmp, {}

    def start(self, nm):
        ic = ",".join(f"{k}=http://{v}" for k, v in self.peer.items())
        self.procs[nm] = subprocess.Popen(
            [sys.executable, "-m", "amdkube", "etcd", "--name", nm, "--initial-cluster", ic,
             "--listen-client-urls", f"http://{self.client[nm]}", "--listen-peer-urls", f"http://{self.peer[nm]}",
             "--data-dir", str(self.tmp / nm), "--heartbeat-interval", "50", "--election-timeout", "400",
             "--snapshot-count", "40"], stdout=subprocess.DEVNULL, stderr=open(self.tmp / f"{nm}.log", "ab"))

    def kill(self, nm):
        p = self.procs.pop(nm)
        p.send_signal(signal.SIGKILL)
        p.wait(10)

    def stop(self):
        for p in self.procs.values():
            p.terminate()
        for p in self.procs.values():
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()

    def status(self, nm, timeout=1.0):
        with grpc.insecure_channel(self.client[nm]) as ch:
            return E.Maintenance.stub(ch).Status(E.StatusRequest(), timeout=timeout)

    def leader(self, among=None, timeout=20.0):
        """The member every live member agrees leads, once there is one."""
        end = time.time() + timeout
        ids = {_hash_id(nm): nm for nm in self.names}
        while time.time() < end:
            seen = set()
            for nm in (among or list(self.procs)):
                try:
                    seen.add(self.status(nm).leader)
                except grpc.RpcError:
                    seen.add(None)
            if len(seen) == 1 and None not in seen and 0 not in seen and ids.get(next(iter(seen))) in (among or self.procs):
                return ids[seen.pop()]
            time.sleep(0.1)
        raise AssertionError(f"no agreed leader: {seen}")

    def local(self, nm, prefix=b"/r/"):
        """Serializable (member-local) view of a prefix."""
        with grpc.insecure_channel(self.client[nm]) as ch:
            r = E.KV.stub(ch).Range(E.RangeRequest(key=prefix, range_end=prefix_end(prefix), serializable=True), timeout=2)
        return [(kv.key, kv.value, kv.mod_revision) for kv in r.kvs]


@pytest.mark.timeout(180)
async def test_three_member_raft_group(tmp_path):
    c = Cluster(tmp_path)
    try:
        for nm in c.names:
            c.start(nm)
        leader = await asyncio.to_thread(c.leader)
        followers = [nm for nm in c.names if nm != leader]
        store = await asyncio.to_thread(Etcd3Store, [c.client[followers[0]], c.client[leader], c.client[followers[1]]])
        try:
            store.start(asyncio.get_running_loop())
            for i in range(10):                     # writes through a follower are forwarded to the leader
                kv = store.put(f"/r/k{i}", f"v{i}".encode(), expect_mod_rev=0)
                assert kv.value == f"v{i}".encode()
            want = sorted((f"/r/k{i}".encode(), f"v{i}".encode(), store.get(f"/r/k{i}").mod_rev) for i in range(10))

            async def converged(members, expect, timeout=15):
                end = time.time() + timeout
                while time.time() < end:
                    views = list((await views_of(members)).values())
                    if all(v == expect for v in views):
                        return
                    await asyncio.sleep(0.1)
                raise AssertionError(f"members diverge: {views}")

            async def views_of(members):
                out = {}
                for nm in members:
                    try:
                        out[nm] = await asyncio.to_thread(c.local, nm)
                    except grpc.RpcError as e:
                        out[nm] = f"{e.code()} (proc rc={c.procs[nm].poll() if nm in c.procs else 'killed'})"
                return out
            await converged(c.names, want)
            # a linearizable read on a follower is answered by the leader
            with grpc.insecure_channel(c.client[followers[1]]) as ch:
                r = E.KV.stub(ch).Range(E.RangeRequest(key=b"/r/k3"), timeout=5)
                assert r.kvs[0].value == b"v3"

            # the watch keeps flowing across a leader failure
            w = store.watch("/r/", store.rev + 1)
            c.kill(leader)
            new_leader = await asyncio.to_thread(c.leader, followers)
            assert new_leader in followers
            for i in range(10, 70):                 # > --snapshot-count: the survivors compact their logs
                store.put(f"/r/k{i}", f"v{i}".encode())
            got = []
            while len(got) < 60:
                ev = await asyncio.wait_for(w.next(), 20)
                got.append(ev.kv.key)
            assert got == [f"/r/k{i}" for i in range(10, 70)]
            w.close()
            want = sorted((f"/r/k{i}".encode(), f"v{i}".encode(), store.get(f"/r/k{i}").mod_rev) for i in range(70))
            await converged(followers, want)
            # the old leader comes back from its data dir, behind the compacted log: snapshot + catch-up
            c.start(leader)
            await converged(c.names, want, timeout=30)
            assert (await asyncio.to_thread(c.leader)) in c.names
            assert len({(await asyncio.to_thread(c.status, nm)).header.revision for nm in c.names}) == 1
            assert os.path.exists(tmp_path / leader / "raft" / "snap.bin")
        finally:
            store.close()
    finally:
        c.stop()


class _SM:
    def __init__(self):
        self.applied = []

    def apply(self, i, data):
        self.applied.append((i, data))
        return data

    def snapshot(self):
        return repr(self.applied).encode()

    def restore(self, data):
        import ast
        self.applied = ast.literal_eval(data.decode())


async def test_raft_log_matching_votes_and_persistence(tmp_path):
    """Handler-level Raft rules (§5.1-5.4 of the paper) on one member, no network."""
    from amdkube.store.raft import RAFT as R, Raft
    sm = _SM()
    r = Raft("b", {"a": "127.0.0.1:1", "b": "127.0.0.1:2", "c": "127.0.0.1:3"}, str(tmp_path), sm)

    def ents(*spec):
        return [R.Entry(term=t, index=i, data=f"{i}@{t}".encode()) for i, t in spec]
    ok = await r.AppendEntries(R.AppendRequest(term=1, leader="a", prev_log_index=0, prev_log_term=0,
                                               entries=ents((1, 1), (2, 1), (3, 1)), leader_commit=1), None)
    assert ok.success and ok.match_index == 3 and r.commit == 1 and sm.applied == [(1, b"1@1")]
    # a gap is refused with a hint at our end of log
    gap = await r.AppendEntries(R.AppendRequest(term=1, leader="a", prev_log_index=7, prev_log_term=1), None)
    assert not gap.success and gap.conflict_index == 4
    # a new leader (term 2) overwrites the uncommitted tail from index 3 on
    ok = await r.AppendEntries(R.AppendRequest(term=2, leader="c", prev_log_index=2, prev_log_term=1,
                                               entries=ents((3, 2), (4, 2)), leader_commit=4), None)
    assert ok.success and [(e.index, e.term) for e in r.log] == [(1, 1), (2, 1), (3, 2), (4, 2)]
    assert sm.applied[-1] == (4, b"4@2") and r.leader == "c"
    # mismatched prev term: hint back to the first index of that term
    bad = await r.AppendEntries(R.AppendRequest(term=2, leader="c", prev_log_index=4, prev_log_term=9), None)
    assert not bad.success and bad.conflict_index == 3
    # stale terms are refused; votes need an up-to-date log and one vote per term
    assert not (await r.AppendEntries(R.AppendRequest(term=1, leader="a"), None)).success
    assert not (await r.RequestVote(R.VoteRequest(term=3, candidate="a", last_log_index=9, last_log_term=1), None)).granted
    assert (await r.RequestVote(R.VoteRequest(term=3, candidate="c", last_log_index=4, last_log_term=2), None)).granted
    assert not (await r.RequestVote(R.VoteRequest(term=3, candidate="a", last_log_index=4, last_log_term=2), None)).granted
    await r.stop()
    # term, vote and log survive a restart
    r2 = Raft("b", {"a": "127.0.0.1:1", "b": "127.0.0.1:2", "c": "127.0.0.1:3"}, str(tmp_path), _SM())
    assert (r2.term, r2.voted_for, r2.last_index(), r2.last_term()) == (3, "c", 4, 2)
    await r2.stop()


async def _inproc_cluster(tmp_path, peer_tls=None, n=3):
    from amdkube.store import MVCCStore
    from amdkube.store.etcdserver import EtcdServer
    ps = _ports(n)
    peers = {f"m{i}": f"127.0.0.1:{ps[i]}" for i in range(n)}
    srvs = {}
    for nm in peers:
        srvs[nm] = await EtcdServer(MVCCStore(None), name=nm, peers=peers, data_dir=str(tmp_path / nm), heartbeat=0.05,
                                    election=0.4, peer_tls=peer_tls).start("127.0.0.1:0", None, peers[nm])
    end = time.time() + 20
    while time.time() < end:
        leaders = [nm for nm, s in srvs.items() if s.raft.role == "leader"]
        if len(leaders) == 1 and all(s.raft.leader == leaders[0] for s in srvs.values()):
            return srvs, leaders[0], peers
        await asyncio.sleep(0.05)
    raise AssertionError("no leader")


@pytest.mark.timeout(120)
async def test_group_commit_batches_concurrent_proposals(tmp_path, monkeypatch):
    """256 concurrent Puts through a follower: every one commits at its own revision, and the
    leader persisted them with far fewer log writes (one write + fdatasync per flush) than
    proposals — the Ready batching of etcd (raft/node.go:52, etcdserver/raft.go:134)."""
    from amdkube.store.raft import Raft
    writes = {"n": 0}
    orig = Raft._write_entries

    def counting(self, f, entries):
        if self.role == "leader":
            writes["n"] += 1
        return orig(self, f, entries)
    monkeypatch.setattr(Raft, "_write_entries", counting)
    srvs, leader, _ = await _inproc_cluster(tmp_path)
    try:
        follower = next(nm for nm in srvs if nm != leader)
        ch = grpc.aio.insecure_channel(srvs[follower].address)
        kv = E.KV.stub(ch)
        base = writes["n"]
        rs = await asyncio.gather(*(kv.Put(E.PutRequest(key=f"/g/{i}".encode(), value=b"v"), timeout=20) for i in range(256)))
        revs = sorted(r.header.revision for r in rs)
        assert revs == list(range(revs[0], revs[0] + 256))
        flushes = writes["n"] - base
        assert flushes < 128, flushes
        # a follower's linearizable read (ReadIndex over the peer channel) sees every write
        r = await kv.Range(E.RangeRequest(key=b"/g/", range_end=prefix_end(b"/g/")), timeout=10)
        assert r.count == 256
        await ch.close()
    finally:
        for s in srvs.values():
            await s.stop()


@pytest.mark.timeout(120)
async def test_peer_listener_serves_only_member_traffic_under_mutual_tls(tmp_path):
    """The client API is not reachable on the peer listener and raft is not reachable on the
    client listener; with peer TLS a client without a member certificate cannot reach the peer
    services at all (advisor r3: the peer port bypassed client TLS)."""
    from amdkube.kubeadm import new_ca, new_cert
    from amdkube.store.etcdserver import PEER
    from amdkube.store.raft import RAFT
    d = tmp_path / "pki"
    d.mkdir()
    new_ca(str(d), "peer-ca", "etcd-peer-ca")
    new_cert(str(d), "peer", "etcd-peer", sans=("IP:127.0.0.1", "DNS:localhost"), server="peer", ca="peer-ca")
    tls = (str(d / "peer.crt"), str(d / "peer.key"), str(d / "peer-ca.crt"))
    srvs, leader, peers = await _inproc_cluster(tmp_path, peer_tls=tls)
    try:
        s = srvs[leader]
        async with grpc.aio.insecure_channel(s.address) as ch:
            await E.KV.stub(ch).Put(E.PutRequest(key=b"/t/a", value=b"1"), timeout=10)
        # raft is not on the client port
        async with grpc.aio.insecure_channel(s.address) as ch:
            with pytest.raises(grpc.RpcError) as ei:
                await RAFT.Raft.stub(ch).InstallSnapshot(RAFT.SnapshotRequest(term=99, leader="x"), timeout=5)
            assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        # plaintext to the peer port fails
        async with grpc.aio.insecure_channel(peers[leader]) as ch:
            with pytest.raises(grpc.RpcError):
                await PEER.Peer.stub(ch).Propose(PEER.ProposeRequest(data=b"\x02"), timeout=3)
        # TLS without a client certificate fails the handshake
        ca = open(tls[2], "rb").read()
        async with grpc.aio.secure_channel(peers[leader], grpc.ssl_channel_credentials(root_certificates=ca)) as ch:
            with pytest.raises(grpc.RpcError):
                await PEER.Peer.stub(ch).ReadIndex(PEER.ReadIndexRequest(), timeout=3)
        # a member certificate reaches Peer, but never the client services
        from amdkube.store.peerwire import PeerChannel, stub
        async with s._peer_channel(peers[leader]) as ch:
            r = await stub(PEER.Peer, ch).ReadIndex(PEER.ReadIndexRequest(), timeout=5)
            assert r.index >= 1 and not r.code
            with pytest.raises(grpc.RpcError) as ei:
                await stub(E.KV, ch).Range(E.RangeRequest(key=b"/t/a"), timeout=5)
            assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        # the peer transport without TLS cannot talk to the TLS listener either
        async with PeerChannel(peers[leader]) as ch:
            with pytest.raises(grpc.RpcError):
                await stub(PEER.Peer, ch).ReadIndex(PEER.ReadIndexRequest(), timeout=3)
        # writes through a follower still commit over the TLS peer channel
        follower = next(nm for nm in srvs if nm != leader)
        async with grpc.aio.insecure_channel(srvs[follower].address) as ch:
            await E.KV.stub(ch).Put(E.PutRequest(key=b"/t/b", value=b"2"), timeout=10)
            r = await E.KV.stub(ch).Range(E.RangeRequest(key=b"/t/b"), timeout=10)
            assert r.kvs[0].value == b"2"
    finally:
        for s in srvs.values():
            await s.stop()


async def test_peerwire_server_survives_malformed_frames():
    """Garbage on a peerwire listener (truncated, oversized, undecodable, unknown kinds) ends
    that connection only; the server keeps answering well-formed calls."""
    import random
    import struct
    from amdkube.grpcdesc.etcd import ETCD as E
    from amdkube.store.etcdserver import EtcdServer
    from amdkube.store.mvcc import MVCCStore
    from amdkube.store.peerwire import SyncChannel
    srv = await EtcdServer(MVCCStore()).start("127.0.0.1:0", None, None, "127.0.0.1:0")
    rnd = random.Random(7)
    try:
        good = E.PutRequest(key=b"/k", value=b"v").SerializeToString()
        path = b"/etcdserverpb.KV/Put"
        frames = [b"\x00\x00\x00\x05\x00\x00\x00\x00\x01",                          # REQ without a path length
                  b"\x00\x00\x00\x06\x00\x00\x00\x00\x01\xff",                      # path longer than the frame
                  b"\xff\xff\xff\xff",                                              # oversized
                  struct.pack(">IBIB", 6 + len(path) + 3, 0, 1, len(path)) + path + b"\xff\xff\xff",   # undecodable body
                  struct.pack(">IBIB", 6 + 9, 0, 2, 9) + b"/\xff\xfe\x00x/yz",     # non-UTF-8 path
                  struct.pack(">IBI", 5, 9, 3),                                      # unknown kind
                  struct.pack(">IBIB", 6 + 26, 0, 4, 26) + b"/etcdserverpb.Watch/Watch" + b"\x0a\xff"]   # bad stream opener
        frames += [bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 64))) for _ in range(40)]
        for f in frames:
            r, w = await asyncio.open_connection("127.0.0.1", srv.wire_port)
            w.write(f)
            try:
                await asyncio.wait_for(r.read(1 << 16), 1.0)
            except (asyncio.TimeoutError, ConnectionError):
                pass
            w.close()
        ch = SyncChannel(f"127.0.0.1:{srv.wire_port}")
        resp = E.PutResponse.FromString(await asyncio.to_thread(ch.call, "/etcdserverpb.KV/Put", good, 5))
        assert resp.header.revision >= 1
        ch.close()
    finally:
        await srv.stop()
