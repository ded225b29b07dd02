"""`amdkube etcd`: the etcd v3 gRPC API (KV, Watch, Lease, Maintenance.Status) served from the
MVCC store, so several apiservers can share one store the way the reference's apiservers share
etcd (staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go:152-260 drives exactly these
calls: Create = Txn(If mod_revision==0 Then Put), GuaranteedUpdate / Delete = Txn(If
mod_revision==X Then Put|DeleteRange Else Range), List = Range(prefix, prefix+1[, revision]),
Watch = Watch(create{key, range_end, start_revision, prev_kv}), compact.go = Compact).

Semantics follow etcd's (etcdserver/apply.go, mvcc/kvstore_txn.go):
* a Txn's chosen branch commits at ONE revision (MVCCStore.batch), a Txn of ranges only
  does not advance it; Range at an old `revision` is rebuilt from the store's event history
  (compacted: OUT_OF_RANGE "required revision has been compacted"; future: "required revision
  is a future revision");
* a watch from a compacted revision is created and immediately canceled with
  `compact_revision` set (the client re-lists), events are batched per response with prev_kv
  on request and NOPUT/NODELETE filters;
* leases carry keys; an expired or revoked lease deletes them in one revision.
Not provided: members/auth/cluster RPCs, defragment/snapshot/hash, multi-op txn nesting.

Clustered (`--initial-cluster`), the client API and the peer API listen apart, as etcd's
--listen-client-urls / --listen-peer-urls do. The peer listener carries only member-to-member
traffic: the raft service and `amdkube.etcdpeer.Peer` — Propose (a follower hands a client
mutation to the leader as a raft proposal, etcd's MsgProp), ReadIndex (a follower's
linearizable read: the leader confirms its lease and returns its commit index, the follower
serves once it has applied that far — etcd's ReadIndex) and KeepAlive (lease renewals relayed to
the leader's lessor, etcd's /leases peer handler). With --peer-cert-file/--peer-key-file/
--peer-trusted-ca-file the peer listener and every peer channel use mutual TLS; the client
services are never reachable on it.
"""
from __future__ import annotations

import asyncio
import bisect
import logging
import random
import time

import grpc

from ..grpcdesc.compiler import ProtoModule
from ..grpcdesc.etcd import (EQUAL, ETCD as E, EV_DELETE, EV_PUT, GREATER, LESS, NOT_EQUAL, T_CREATE, T_MOD,
                             T_VALUE, T_VERSION)
from .mvcc import PUT, MVCCStore
from .peerwire import stub as peer_stub

log = logging.getLogger("amdkube.etcd")
VERSION = "3.1.11-amdkube"
WIRE_METADATA = "amdkube-wire"     # Status initial metadata: the client wire lane's port
NOPUT, NODELETE = 0, 1


def _s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


def _b(s: str) -> bytes:
    return s.encode("utf-8", "surrogateescape")


def prefix_end(key: bytes) -> bytes:
    """clientv3.GetPrefixRangeEnd: the key with its last non-0xff byte incremented."""
    k = bytearray(key)
    for i in range(len(k) - 1, -1, -1):
        if k[i] < 0xFF:
            k[i] += 1
            return bytes(k[:i + 1])
    return b"\x00"


K_TXN, K_PUT, K_DELETE, K_COMPACT, K_LEASE_GRANT, K_LEASE_REVOKE = 1, 2, 3, 4, 5, 6
_REQ = {K_TXN: E.TxnRequest, K_PUT: E.PutRequest, K_DELETE: E.DeleteRangeRequest, K_COMPACT: E.CompactionRequest,
        K_LEASE_GRANT: E.LeaseGrantRequest, K_LEASE_REVOKE: E.LeaseRevokeRequest}
_KV_KINDS = {K_TXN, K_PUT, K_DELETE, K_COMPACT}
_RESP = {K_TXN: E.TxnResponse, K_PUT: E.PutResponse, K_DELETE: E.DeleteRangeResponse, K_COMPACT: E.CompactionResponse,
         K_LEASE_GRANT: E.LeaseGrantResponse, K_LEASE_REVOKE: E.LeaseRevokeResponse}
_CODES = {c.value[0]: c for c in grpc.StatusCode}
_SRV_OPTS = [("grpc.max_receive_message_length", 256 << 20), ("grpc.max_send_message_length", 256 << 20)]

PEER = ProtoModule("""
syntax = "proto3";
package amdkube.etcdpeer;

service Peer {
  rpc Propose(ProposeRequest) returns (ProposeResponse) {}
  rpc ReadIndex(ReadIndexRequest) returns (ReadIndexResponse) {}
  rpc KeepAlive(KeepAliveRequest) returns (KeepAliveResponse) {}
}
message ProposeRequest { bytes data = 1; }
message ProposeResponse { bytes result = 1; int32 code = 2; string message = 3; string leader = 4; }
message ReadIndexRequest {}
message ReadIndexResponse { uint64 index = 1; int32 code = 2; string leader = 3; }
message KeepAliveRequest { int64 id = 1; }
message KeepAliveResponse { int64 ttl = 1; bool found = 2; }
""", "amdkube/etcdpeer.proto")


def _hash_id(name: str) -> int:
    import hashlib
    return int.from_bytes(hashlib.sha256(name.encode()).digest()[:8], "big") & ((1 << 63) - 1)


# etcd's request limits: --max-txn-ops (embed/config.go DefaultMaxTxnOps) and
# --max-request-bytes (DefaultMaxRequestBytes = 1.5 MiB); refused as InvalidArgument
# (v3rpc/key.go checkTxnRequest ErrGRPCTooManyOps; v3_server.go ErrRequestTooLarge)
DEFAULT_MAX_TXN_OPS = 128
DEFAULT_MAX_REQUEST_BYTES = 3 * 512 * 1024


class _Abort(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code, self.msg = code, msg


class EtcdServer:
    def __init__(self, store: MVCCStore, cluster_id: int | None = None, member_id: int | None = None,
                 name: str = "default", peers: dict[str, str] | None = None, data_dir: str | None = None,
                 heartbeat: float = 0.1, election: float = 1.0, compact_every: int = 10_000,
                 peer_tls: tuple[str, str, str | None] | None = None, max_txn_ops: int = DEFAULT_MAX_TXN_OPS,
                 max_request_bytes: int = DEFAULT_MAX_REQUEST_BYTES):
        self.store = store
        self.max_txn_ops, self.max_request_bytes = max_txn_ops, max_request_bytes
        self.compact_every = compact_every
        self.name = name
        self.peers = peers or {}
        self.cluster_id = cluster_id or (_hash_id(",".join(f"{k}={v}" for k, v in sorted(self.peers.items())))
                                         if self.peers else random.getrandbits(63))
        self.member_id = member_id or _hash_id(name)
        self.leases: dict[int, list] = {}          # id -> [ttl, deadline, set(keys)]
        self.key_lease: dict[str, int] = {}
        self.server: grpc.aio.Server | None = None
        self.port = 0
        self._tasks: list[asyncio.Task] = []
        self.raft = None
        self._raft_args = (data_dir, heartbeat, election)
        self._fwd: dict = {}            # member name -> peerwire.PeerChannel
        # (cert file, key file, trusted CA file or None): mutual TLS between members
        self.peer_tls = peer_tls
        self.peer_server = None         # peerwire.PeerServer
        self.peer_port = 0
        self.wire_server = None         # peerwire.PeerServer carrying the client API (KV, Watch, Status)
        self.wire_port = 0

    # ------------------------------------------------------------------ lifecycle
    def _peer_channel(self, target: str):
        """A connection to another member's peer listener (raft + Peer), under peer TLS if set."""
        from .peerwire import PeerChannel, client_ssl
        return PeerChannel(target, client_ssl(*self.peer_tls) if self.peer_tls else None)

    async def start(self, address: str = "127.0.0.1:0", credentials=None, peer_address: str | None = None,
                    wire_address: str | None = None, wire_ssl=None):
        """Serve the client API (KV, Watch, Lease, Maintenance) on `address`. With a cluster, a
        second server on `peer_address` (default: this member's --initial-cluster URL) carries
        the raft and Peer services and nothing else. With `wire_address`, the KV, Watch and
        Status methods are also served over peerwire framing (under `wire_ssl`, the client TLS
        of the gRPC listener) and the port is advertised in Status's initial metadata."""
        self.server = grpc.aio.server(options=_SRV_OPTS)
        for svc in ("KV", "Watch", "Lease", "Maintenance"):
            self.server.add_generic_rpc_handlers((E.services[svc].handler(self),))
        self.port = (self.server.add_secure_port(address, credentials) if credentials is not None
                     else self.server.add_insecure_port(address))
        if wire_address is not None:
            from .peerwire import PeerServer
            self.wire_server = PeerServer([(E.services[svc], self) for svc in ("KV", "Watch", "Maintenance")], wire_ssl)
            self.wire_port = await self.wire_server.start(wire_address)
        if len(self.peers) > 1:
            from .raft import RAFT, Raft
            data_dir, hb, el = self._raft_args
            self.raft = Raft(self.name, self.peers, data_dir, self, heartbeat=hb, election=el,
                             compact_every=self.compact_every, channel=self._peer_channel)
            from .peerwire import PeerServer, server_ssl
            self.peer_server = PeerServer([(RAFT.Raft, self.raft), (PEER.Peer, self)],
                                          server_ssl(*self.peer_tls) if self.peer_tls else None)
            self.peer_port = await self.peer_server.start(peer_address or self.peers[self.name])
        await self.server.start()
        if self.raft is not None:
            await self.raft.start()
        self._tasks.append(asyncio.create_task(self._lease_reaper()))
        self.address = f"{address.rsplit(':', 1)[0]}:{self.port}"
        return self

    async def stop(self, grace: float = 0.5):
        from ..utils import cancel_and_wait
        await cancel_and_wait(self._tasks)
        if self.raft is not None:
            await self.raft.stop()
        for ch in self._fwd.values():
            await ch.close()
        if self.server is not None:
            await self.server.stop(grace)
        if self.peer_server is not None:
            await self.peer_server.stop()
        if self.wire_server is not None:
            await self.wire_server.stop()
        for w in self.store.all_watchers():
            w.close()

    # ------------------------------------------------------------------ raft state machine
    def apply(self, index: int, data: bytes):
        """Raft apply: one committed client mutation, deterministic on every member."""
        kind, body = data[0], data[1:]
        return self._exec(kind, _REQ[kind].FromString(body))

    def snapshot(self) -> bytes:
        import json as _json
        return _json.dumps({"store": self.store.dump_state(),
                            "leases": {str(k): [v[0], sorted(v[2])] for k, v in self.leases.items()}}).encode()

    def restore(self, data: bytes):
        import json as _json
        d = _json.loads(data)
        self.store.load_state(d["store"])
        self.leases, self.key_lease = {}, {}
        for lid, (ttl, keys) in d["leases"].items():
            self.leases[int(lid)] = [ttl, time.monotonic() + ttl, set(keys)]
            for k in keys:
                self.key_lease[k] = int(lid)

    def on_leader(self):
        """A new leader restarts every lease's clock (etcd lessor Promote)."""
        now = time.monotonic()
        for ent in self.leases.values():
            ent[1] = now + ent[0]

    def _leader_channel(self, leader: str):
        ch = self._fwd.get(leader)
        if ch is None:
            ch = self._fwd[leader] = self._peer_channel(self.peers[leader])
        return ch

    def _leader_or_abort(self, hint: str | None = None) -> str:
        leader = hint or self.raft.leader
        if not leader or leader == self.name:
            raise _Abort(grpc.StatusCode.UNAVAILABLE, "etcdserver: no leader")
        return leader

    async def _propose(self, data: bytes):
        """Commit one entry through raft: proposed here when leading, else handed to the leader
        over the peer channel (a hop to a stale leader is redirected by its hint)."""
        from .raft import NotLeader
        kind = data[0]
        hint = None
        for _ in range(3):
            try:
                return await self.raft.propose(data)
            except NotLeader as e:
                hint = e.leader or hint
            leader = self._leader_or_abort(hint)
            try:
                r = await peer_stub(PEER.Peer, self._leader_channel(leader)).Propose(PEER.ProposeRequest(data=data), timeout=10)
            except grpc.RpcError as ge:
                raise _Abort(ge.code(), ge.details()) from None
            if not r.code:
                return _RESP[kind].FromString(r.result)
            if r.code != grpc.StatusCode.UNAVAILABLE.value[0] or not r.leader:
                raise _Abort(_CODES.get(r.code, grpc.StatusCode.UNKNOWN), r.message)
            hint = r.leader
            await asyncio.sleep(0.05)
        raise _Abort(grpc.StatusCode.UNAVAILABLE, "etcdserver: leader changed")

    async def _submit(self, kind: int, req, ctx):
        """A mutation: applied here (single member) or committed through raft."""
        try:
            if self.raft is None:
                return self._exec(kind, req)
            try:
                return await self._propose(bytes([kind]) + req.SerializeToString())
            except asyncio.TimeoutError:
                raise _Abort(grpc.StatusCode.UNAVAILABLE, "etcdserver: request timed out") from None
        except _Abort as e:
            await ctx.abort(e.code, e.msg)

    # ------------------------------------------------------------------ Peer service (peer listener only)
    async def Propose(self, req, ctx):
        """A follower's client mutation, proposed by this member if it leads."""
        from .raft import NotLeader
        try:
            result = await self.raft.propose(req.data)
            return PEER.ProposeResponse(result=result.SerializeToString())
        except NotLeader as e:
            return PEER.ProposeResponse(code=grpc.StatusCode.UNAVAILABLE.value[0], message="etcdserver: not leader",
                                        leader=e.leader or "")
        except _Abort as e:
            return PEER.ProposeResponse(code=e.code.value[0], message=e.msg)
        except asyncio.TimeoutError:
            return PEER.ProposeResponse(code=grpc.StatusCode.UNAVAILABLE.value[0], message="etcdserver: request timed out")

    async def ReadIndex(self, req, ctx):
        from .raft import NotLeader
        try:
            return PEER.ReadIndexResponse(index=await self.raft.read_barrier())
        except (NotLeader, TimeoutError):
            return PEER.ReadIndexResponse(code=grpc.StatusCode.UNAVAILABLE.value[0], leader=self.raft.leader or "")

    async def KeepAlive(self, req, ctx):
        ent = self.leases.get(req.id)
        if ent is None or self.raft.role != "leader":
            return PEER.KeepAliveResponse(found=False)
        ent[1] = time.monotonic() + ent[0]
        return PEER.KeepAliveResponse(ttl=ent[0], found=True)

    def _exec(self, kind: int, req):
        if kind == K_TXN:
            ok = all(self._compare(c) for c in req.compare)
            rev, out = self._apply_ops(req.success if ok else req.failure)
            resp = E.TxnResponse(header=self.header(rev), succeeded=ok)
            resp.responses.extend(out)
            return resp
        if kind == K_PUT:
            _, [r] = self._apply_ops([E.RequestOp(request_put=req)])
            return r.response_put
        if kind == K_DELETE:
            _, [r] = self._apply_ops([E.RequestOp(request_delete_range=req)])
            return r.response_delete_range
        if kind == K_COMPACT:
            st = self.store
            if req.revision > st.rev:
                raise _Abort(grpc.StatusCode.OUT_OF_RANGE, "etcdserver: mvcc: required revision is a future revision")
            if req.revision <= st.compact_rev:
                raise _Abort(grpc.StatusCode.OUT_OF_RANGE, "etcdserver: mvcc: required revision has been compacted")
            st.compact(req.revision)
            return E.CompactionResponse(header=self.header())
        if kind == K_LEASE_GRANT:
            if req.ID in self.leases:
                return E.LeaseGrantResponse(header=self.header(), ID=req.ID, TTL=req.TTL, error="lease already exists")
            ttl = max(req.TTL, 1)
            self.leases[req.ID] = [ttl, time.monotonic() + ttl, set()]
            return E.LeaseGrantResponse(header=self.header(), ID=req.ID, TTL=ttl)
        if kind == K_LEASE_REVOKE:
            if not self._expire(req.ID):
                raise _Abort(grpc.StatusCode.NOT_FOUND, "etcdserver: requested lease not found")
            return E.LeaseRevokeResponse(header=self.header())
        raise _Abort(grpc.StatusCode.INTERNAL, f"unknown entry kind {kind}")

    def header(self, rev: int | None = None):
        return E.ResponseHeader(cluster_id=self.cluster_id, member_id=self.member_id,
                                revision=self.store.rev if rev is None else rev, raft_term=1)

    def _kv(self, kv, keys_only=False):
        return E.KeyValue(key=_b(kv.key), create_revision=kv.create_rev, mod_revision=kv.mod_rev, version=kv.version,
                          value=b"" if keys_only else kv.value, lease=self.key_lease.get(kv.key, 0))

    # ------------------------------------------------------------------ ranges
    def _keys(self, key: bytes, end: bytes) -> list[str]:
        st = self.store
        if not end:
            return [_s(key)] if _s(key) in st.kv else []
        if end == prefix_end(key) and key:
            return st._candidates(_s(key))
        lo = _s(key)
        ks = sorted(st.kv) if end == b"\x00" else sorted(k for k in st.kv if lo <= k < _s(end))
        return ks[bisect.bisect_left(ks, lo):]

    def _at(self, req_key: bytes, end: bytes, rev: int) -> dict[str, object]:
        """The range as it was at `rev`: the current state with every later event undone."""
        st = self.store
        if rev <= st.compact_rev:
            raise _Abort(grpc.StatusCode.OUT_OF_RANGE, "etcdserver: mvcc: required revision has been compacted")
        if rev > st.rev:
            raise _Abort(grpc.StatusCode.OUT_OF_RANGE, "etcdserver: mvcc: required revision is a future revision")
        lo, hi = _s(req_key), _s(end)

        def inside(k):
            if not end:
                return k == lo
            return k >= lo and (end == b"\x00" or k < hi)
        state = {k: st.kv[k] for k in self._keys(req_key, end)}
        for ev in reversed(st.history):
            if ev.rev <= rev:
                break
            k = ev.kv.key
            if not inside(k):
                continue
            if ev.prev is None:
                state.pop(k, None)
            else:
                state[k] = ev.prev
        return state

    def _range(self, r):
        st = self.store
        if r.revision and r.revision != st.rev:
            state = self._at(r.key, r.range_end, r.revision)
            kvs = [state[k] for k in sorted(state)]
        else:
            kvs = [st.kv[k] for k in self._keys(r.key, r.range_end) if k in st.kv]
        if r.min_mod_revision or r.max_mod_revision or r.min_create_revision or r.max_create_revision:
            kvs = [kv for kv in kvs if (not r.min_mod_revision or kv.mod_rev >= r.min_mod_revision)
                   and (not r.max_mod_revision or kv.mod_rev <= r.max_mod_revision)
                   and (not r.min_create_revision or kv.create_rev >= r.min_create_revision)
                   and (not r.max_create_revision or kv.create_rev <= r.max_create_revision)]
        if r.sort_target or r.sort_order:
            target = {0: lambda kv: kv.key, 1: lambda kv: kv.version, 2: lambda kv: kv.create_rev,
                      3: lambda kv: kv.mod_rev, 4: lambda kv: kv.value}[r.sort_target]
            kvs.sort(key=target, reverse=r.sort_order == 2)
        count = len(kvs)
        more = bool(r.limit and count > r.limit)
        if r.limit:
            kvs = kvs[:r.limit]
        resp = E.RangeResponse(header=self.header(), more=more, count=count)
        if not r.count_only:
            resp.kvs.extend(self._kv(kv, r.keys_only) for kv in kvs)
        return resp

    # ------------------------------------------------------------------ KV service
    async def Range(self, req, ctx):
        try:
            if self.raft is not None and not req.serializable:
                from .raft import NotLeader
                try:
                    await self.raft.read_barrier()
                except (NotLeader, TimeoutError):
                    # ReadIndex: the leader vouches for its commit index; serve it once applied here
                    leader = self._leader_or_abort()
                    try:
                        r = await peer_stub(PEER.Peer, self._leader_channel(leader)).ReadIndex(PEER.ReadIndexRequest(), timeout=10)
                    except grpc.RpcError as ge:
                        raise _Abort(ge.code(), ge.details()) from None
                    if r.code:
                        raise _Abort(grpc.StatusCode.UNAVAILABLE, "etcdserver: leader changed") from None
                    try:
                        await self.raft.wait_applied(r.index, timeout=10)
                    except asyncio.TimeoutError:
                        raise _Abort(grpc.StatusCode.UNAVAILABLE, "etcdserver: request timed out") from None
            return self._range(req)
        except _Abort as e:
            await ctx.abort(e.code, e.msg)

    def _check_lease(self, lease: int):
        if lease and lease not in self.leases:
            raise _Abort(grpc.StatusCode.NOT_FOUND, "etcdserver: requested lease not found")

    def _attach(self, key: str, lease: int):
        old = self.key_lease.pop(key, 0)
        if old in self.leases:
            self.leases[old][2].discard(key)
        if lease:
            self.key_lease[key] = lease
            self.leases[lease][2].add(key)

    def _detach(self, key: str):
        self._attach(key, 0)

    def _apply_ops(self, ops):
        """Commit a list of RequestOp (one revision); returns ResponseOps."""
        batch, plan = [], []
        for op in ops:
            kind = op.WhichOneof("request")
            if kind == "request_put":
                p = op.request_put
                self._check_lease(p.lease)
                batch.append(("put", _s(p.key), p.value))
                plan.append(("put", p, len(batch) - 1))
            elif kind == "request_delete_range":
                d = op.request_delete_range
                keys = self._keys(d.key, d.range_end)
                first = len(batch)
                batch.extend(("delete", k) for k in keys)
                plan.append(("del", d, (first, len(batch))))
            elif kind == "request_range":
                plan.append(("range", op.request_range, None))
        ranges_before = {i: self._range(p) for i, (k, p, _) in enumerate(plan) if k == "range"}
        rev, prevs = self.store.batch(batch) if batch else (self.store.rev, [])
        out = []
        for i, (kind, p, where) in enumerate(plan):
            if kind == "put":
                self._attach(_s(p.key), p.lease)
                r = E.PutResponse(header=self.header(rev))
                if p.prev_kv and prevs[where] is not None:
                    r.prev_kv.CopyFrom(self._kv(prevs[where]))
                out.append(E.ResponseOp(response_put=r))
            elif kind == "del":
                lo, hi = where
                gone = [pv for pv in prevs[lo:hi] if pv is not None]
                for pv in gone:
                    self._detach(pv.key)
                r = E.DeleteRangeResponse(header=self.header(rev), deleted=len(gone))
                if p.prev_kv:
                    r.prev_kvs.extend(self._kv(pv) for pv in gone)
                out.append(E.ResponseOp(response_delete_range=r))
            else:
                out.append(E.ResponseOp(response_range=ranges_before[i]))
        return rev, out

    async def _too_large(self, req, ctx) -> bool:
        if req.ByteSize() > self.max_request_bytes:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "etcdserver: request is too large")
            return True
        return False

    async def Put(self, req, ctx):
        if await self._too_large(req, ctx):
            return None
        return await self._submit(K_PUT, req, ctx)

    async def DeleteRange(self, req, ctx):
        return await self._submit(K_DELETE, req, ctx)

    def _compare(self, c) -> bool:
        kv = self.store.kv.get(_s(c.key))
        which = c.WhichOneof("target_union")
        if c.target == T_VALUE:
            if kv is None:
                return False            # etcd: a value compare on a missing key is false
            have, want = kv.value, c.value
        else:
            have = 0 if kv is None else {T_VERSION: kv.version, T_CREATE: kv.create_rev, T_MOD: kv.mod_rev}[c.target]
            want = getattr(c, which) if which else 0
        return {EQUAL: have == want, NOT_EQUAL: have != want, GREATER: have > want, LESS: have < want}[c.result]

    async def Txn(self, req, ctx):
        n = self.max_txn_ops
        if len(req.compare) > n or len(req.success) > n or len(req.failure) > n:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "etcdserver: too many operations in txn request")
            return None
        if await self._too_large(req, ctx):
            return None
        return await self._submit(K_TXN, req, ctx)

    async def Compact(self, req, ctx):
        return await self._submit(K_COMPACT, req, ctx)

    # ------------------------------------------------------------------ Watch service
    def _watch_scope(self, c):
        """(prefix, exact, in_range) for an MVCCStore watcher covering [key, range_end)."""
        lo, end = c.key, c.range_end
        if not end:
            return _s(lo), True, None
        if lo and end == prefix_end(lo):
            return _s(lo), False, None
        slo, send = _s(lo), _s(end)
        common = ""
        if end != b"\x00":
            for a, b in zip(slo, send):
                if a != b:
                    break
                common += a
        return common, False, (lambda k: k >= slo and (end == b"\x00" or k < send))

    async def Watch(self, requests, ctx):
        out: asyncio.Queue = asyncio.Queue()
        watches: dict[int, tuple] = {}
        next_id = iter(range(1, 1 << 62))

        async def pump(wid, w, c):
            filters = set(c.filters)
            try:
                while True:
                    ev = await w.next()
                    if ev is None:
                        out.put_nowait(E.WatchResponse(header=self.header(), watch_id=wid, canceled=True))
                        return
                    batch = [ev]
                    while not w.queue.empty():
                        nxt = w.queue.get_nowait()
                        if nxt is None:
                            w.queue.put_nowait(None)
                            break
                        batch.append(nxt)
                    resp = E.WatchResponse(header=self.header(), watch_id=wid)
                    for e in batch:
                        typ = EV_PUT if e.type == PUT else EV_DELETE
                        if (typ == EV_PUT and NOPUT in filters) or (typ == EV_DELETE and NODELETE in filters):
                            continue
                        pe = resp.events.add(type=typ)
                        pe.kv.CopyFrom(self._kv(e.kv) if e.type == PUT else
                                       E.KeyValue(key=_b(e.kv.key), mod_revision=e.rev))
                        if c.prev_kv and e.prev is not None:
                            pe.prev_kv.CopyFrom(self._kv(e.prev))
                    if resp.events:
                        out.put_nowait(resp)
            except asyncio.CancelledError:
                pass

        async def progress(wid):
            while True:
                await asyncio.sleep(10)
                out.put_nowait(E.WatchResponse(header=self.header(), watch_id=wid))

        async def reader():
            async for req in requests:
                kind = req.WhichOneof("request_union")
                if kind == "create_request":
                    c = req.create_request
                    wid = next(next_id)
                    prefix, exact, inside = self._watch_scope(c)
                    st = self.store
                    if c.start_revision and c.start_revision <= st.compact_rev:
                        out.put_nowait(E.WatchResponse(header=self.header(), watch_id=wid, created=True))
                        out.put_nowait(E.WatchResponse(header=self.header(), watch_id=wid, canceled=True,
                                                       compact_revision=st.compact_rev))
                        continue
                    transform = (lambda ev, f=inside: ev if f(ev.kv.key) else None) if inside else None
                    w = st.watch(prefix, c.start_revision, exact=exact, transform=transform)
                    out.put_nowait(E.WatchResponse(header=self.header(), watch_id=wid, created=True))
                    tasks = [asyncio.create_task(pump(wid, w, c))]
                    if c.progress_notify:
                        tasks.append(asyncio.create_task(progress(wid)))
                    watches[wid] = (w, tasks)
                elif kind == "cancel_request":
                    wid = req.cancel_request.watch_id
                    ent = watches.pop(wid, None)
                    if ent is not None:
                        ent[0].close()
                        for t in ent[1]:
                            t.cancel()
                        out.put_nowait(E.WatchResponse(header=self.header(), watch_id=wid, canceled=True))
        rd = asyncio.create_task(reader())
        try:
            while True:
                get = asyncio.ensure_future(out.get())
                done, _ = await asyncio.wait({get, rd} if not rd.done() else {get}, return_when=asyncio.FIRST_COMPLETED)
                if get in done:
                    yield get.result()
                    continue
                get.cancel()
                if rd.exception() is not None:
                    return
        finally:
            rd.cancel()
            for w, tasks in watches.values():
                w.close()
                for t in tasks:
                    t.cancel()

    # ------------------------------------------------------------------ Lease service
    async def LeaseGrant(self, req, ctx):
        if not req.ID:                                 # the ID is chosen before replication
            req = E.LeaseGrantRequest(TTL=req.TTL, ID=random.getrandbits(62) + 1)
        return await self._submit(K_LEASE_GRANT, req, ctx)

    def _expire(self, lid: int):
        ent = self.leases.pop(lid, None)
        if ent is None:
            return False
        keys = sorted(k for k in ent[2] if k in self.store.kv)
        for k in ent[2]:
            self.key_lease.pop(k, None)
        if keys:
            self.store.batch([("delete", k) for k in keys])
        return True

    async def LeaseRevoke(self, req, ctx):
        return await self._submit(K_LEASE_REVOKE, req, ctx)

    async def LeaseKeepAlive(self, requests, ctx):
        async for req in requests:
            if self.raft is not None and self.raft.role != "leader":
                leader = self.raft.leader                  # relay to the leader's lessor
                ttl = 0
                if leader and leader != self.name:
                    try:
                        r = await peer_stub(PEER.Peer, self._leader_channel(leader)).KeepAlive(
                            PEER.KeepAliveRequest(id=req.ID), timeout=5)
                        ttl = r.ttl if r.found else 0
                    except grpc.RpcError as ge:
                        log.debug("lease %d keepalive relay to %s failed: %s", req.ID, leader, ge.code())
                yield E.LeaseKeepAliveResponse(header=self.header(), ID=req.ID, TTL=ttl)
                continue
            ent = self.leases.get(req.ID)
            if ent is None:
                yield E.LeaseKeepAliveResponse(header=self.header(), ID=req.ID, TTL=0)
                continue
            ent[1] = time.monotonic() + ent[0]
            yield E.LeaseKeepAliveResponse(header=self.header(), ID=req.ID, TTL=ent[0])

    async def _lease_reaper(self):
        while True:
            await asyncio.sleep(0.25)
            if self.raft is not None and self.raft.role != "leader":
                continue                               # only the leader's lessor expires leases
            now = time.monotonic()
            for lid in [lid for lid, ent in self.leases.items() if ent[1] <= now]:
                if self.raft is None:
                    self._expire(lid)
                else:
                    try:
                        await self.raft.propose(bytes([K_LEASE_REVOKE]) + E.LeaseRevokeRequest(ID=lid).SerializeToString())
                    except Exception as e:     # lost leadership or the lease went meanwhile
                        log.debug("lease %d expiry not committed: %s", lid, e)

    # ------------------------------------------------------------------ Maintenance
    async def Status(self, req, ctx):
        if self.wire_port and hasattr(ctx, "send_initial_metadata"):
            await ctx.send_initial_metadata(((WIRE_METADATA, str(self.wire_port)),))
        size = sum(len(kv.value) + len(kv.key) for kv in self.store.kv.values())
        if self.raft is None:
            return E.StatusResponse(header=self.header(), version=VERSION, dbSize=size, leader=self.member_id,
                                    raftIndex=self.store.rev, raftTerm=1)
        r = self.raft
        return E.StatusResponse(header=self.header(), version=VERSION, dbSize=size,
                                leader=_hash_id(r.leader) if r.leader else 0, raftIndex=r.commit, raftTerm=r.term)


async def serve(data_dir: str | None, listen: str, cert=None, key=None, ca=None, snapshot_every: int = 50_000,
                name: str = "default", peers: dict[str, str] | None = None, peer_listen: str | None = None,
                heartbeat: float = 0.1, election: float = 1.0, peer_cert=None, peer_key=None, peer_ca=None,
                wire_port: int = 0, max_txn_ops: int = DEFAULT_MAX_TXN_OPS,
                max_request_bytes: int = DEFAULT_MAX_REQUEST_BYTES):
    """`amdkube etcd`: run until cancelled. With `peers` (--initial-cluster) the member joins a
    raft group; its store then lives in memory and the raft log under data_dir is the WAL.
    `wire_port` (-1: off, 0: any free port) is the client wire lane on the client listener's host."""
    creds = wire_ssl = None
    if cert and key:
        creds = grpc.ssl_server_credentials([(open(key, "rb").read(), open(cert, "rb").read())],
                                            root_certificates=open(ca, "rb").read() if ca else None,
                                            require_client_auth=bool(ca))
        from .peerwire import server_ssl
        wire_ssl = server_ssl(cert, key, ca)
    wire_address = None if wire_port < 0 else f"{listen.rsplit(':', 1)[0]}:{wire_port}"
    clustered = bool(peers) and len(peers) > 1
    store = MVCCStore(None if clustered else data_dir, snapshot_every=snapshot_every)
    srv = await EtcdServer(store, name=name, peers=peers if clustered else None, data_dir=data_dir,
                           heartbeat=heartbeat, election=election, compact_every=snapshot_every,
                           peer_tls=(peer_cert, peer_key, peer_ca) if peer_cert and peer_key else None,
                           max_txn_ops=max_txn_ops, max_request_bytes=max_request_bytes,
                           ).start(listen, creds, peer_listen if clustered else None, wire_address, wire_ssl)
    print(f"amdkube etcd: serving the etcd v3 API on {srv.address} (revision {store.rev})"
          + (f", client wire lane on port {srv.wire_port}" if srv.wire_port else ""), flush=True)
    try:
        await asyncio.Event().wait()
    finally:
        await srv.stop()
        store.close()
