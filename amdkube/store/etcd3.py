"""An apiserver store backed by a remote etcd v3 (`amdkube etcd` or any etcd speaking the v3
API), so several apiservers share one keyspace (`--etcd-servers`).

Reference: staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go (writes are etcd Txns:
Create `If(ModRevision==0).Then(Put)` :152-200, GuaranteedUpdate/Delete `If(ModRevision==X)
.Then(Put|Delete).Else(Get)` :263, :208-256) and pkg/storage/cacher.go (reads and watches are
served from a watch-fed in-memory cache).

Etcd3Store IS an MVCCStore: a full local replica the apiserver reads, indexes and watches
exactly as it does the embedded store (commit hooks, trigger-indexed watchers, history for
watch-from-revision), fed by ONE etcd watch over the whole keyspace from a background thread.
Mutations go to etcd as CAS Txns over a blocking gRPC channel, then wait until the replica
has applied the Txn's revision, so a write is visible to its writer's next read (and to its
watchers) before the call returns. Other apiservers' writes arrive through the watch.

Stored objects embed metadata.resourceVersion (amdkube serves stored bytes as-is), so a value
must be rendered for the revision its Txn will commit at. Every apiserver Txn therefore also
puts a fence key and compares its mod_revision with the replica's: success proves no other
apiserver committed in between, so the commit revision is the replica's + 1 (the reference
never stores the version and sets it from mod_revision on decode instead — etcd3/store.go
versioner). Writes from several apiservers are linearised through the fence; a fence-only
conflict catches the replica up and retries.

Transport: gRPC, the etcd v3 API, works against any etcd. An `amdkube etcd` member also
advertises its client wire lane (store/peerwire.py framing, in the Status initial metadata);
when it does, the KV calls and the watch go over that lane instead (a blocking socket per
call site, no gRPC stack on either end), which takes most of a Txn's cost out of every
apiserver write.
"""
from __future__ import annotations

import logging
import queue
import threading
import time

import grpc

from ..grpcdesc.etcd import ETCD as E, EQUAL, EV_PUT, GREATER, T_MOD, T_VERSION
from .etcdserver import WIRE_METADATA, prefix_end
from .peerwire import PeerChannel, SyncChannel, client_ssl
from ..utils import greenbridge
from .mvcc import DELETE, KV, PUT, CASFailed, Event, KeyExists, KeyNotFound, MVCCStore

log = logging.getLogger("amdkube.etcd3")
ALL = b"\x00"          # key "\0" with range_end "\0": the whole keyspace
FENCE = "/amdkube.io/revision-fence"       # written by every apiserver Txn (see Etcd3Store._write)
_FENCE_B = FENCE.encode()


# etcd refuses a Txn with more than --max-txn-ops (default 128) compares or success/failure ops
# (v3rpc/key.go checkTxnRequest) and a request over --max-request-bytes (1.5 MiB, v3_server.go):
# a group-committed Txn carries the fence plus at most 127 writes, and about 1 MiB of values
MAX_BATCH = 127
MAX_BATCH_BYTES = 1 << 20


class _Op:
    __slots__ = ("key", "value", "expect", "delete", "fut", "data", "tries", "solo")

    def __init__(self, key, value, expect, delete, fut):
        self.key, self.value, self.expect, self.delete, self.fut = key, value, expect, delete, fut
        self.data, self.tries, self.solo = None, 0, False


def _invalid_argument(e: BaseException) -> bool:
    code = getattr(e, "code", None)
    if callable(code):
        try:
            return code() == grpc.StatusCode.INVALID_ARGUMENT
        except Exception:       # noqa: BLE001
            return False
    return "INVALID_ARGUMENT" in str(e)


_KV_RESP = {name: resp for name, _req, resp, _s, _c in E.services["KV"].methods}


def _s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


def _b(s: str) -> bytes:
    return s.encode("utf-8", "surrogateescape")


def _channel(endpoint: str, ca=None, cert=None, key=None):
    target = endpoint.split("://", 1)[-1].rstrip("/")
    opts = [("grpc.max_receive_message_length", 256 << 20), ("grpc.max_send_message_length", 64 << 20)]
    if endpoint.startswith("https://") or ca:
        creds = grpc.ssl_channel_credentials(root_certificates=open(ca, "rb").read() if ca else None,
                                             private_key=open(key, "rb").read() if key else None,
                                             certificate_chain=open(cert, "rb").read() if cert else None)
        return grpc.secure_channel(target, creds, options=opts)
    return grpc.insecure_channel(target, options=opts)


class Etcd3Store(MVCCStore):
    def __init__(self, endpoints, ca: str | None = None, cert: str | None = None, key: str | None = None,
                 history: int = 200_000, max_queue: int = 500_000, timeout: float = 10.0, transformer=None,
                 wire: bool = True):
        # `transformer` (encryption at rest) applies to the bytes etcd holds; the replica keeps plaintext
        super().__init__(None, history=history, max_queue=max_queue, transformer=transformer)
        self.endpoints = [e for e in (endpoints.split(",") if isinstance(endpoints, str) else endpoints) if e]
        self.timeout = timeout
        self._creds = (ca, cert, key)
        self._use_wire = wire
        self._wire_ports: dict[int, int] = {}       # endpoint index -> advertised wire port (0: none)
        self._wire: SyncChannel | None = None
        self._watch_wire: SyncChannel | None = None
        self._achan: PeerChannel | None = None      # the loop's own connection for group commits
        self._pending: list[_Op] = []
        self._flusher = None
        self._ep = 0
        self._chan = None
        self._connect(self._leader_endpoint())
        self._events: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._loop = None
        self._thread: threading.Thread | None = None
        self._watch_call = None
        self.synced_rev = 0
        self.resyncs = 0
        self._initial_sync()
        self._thread = threading.Thread(target=self._follow, name="etcd3-watch", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ endpoints
    def _leader_endpoint(self) -> int:
        """Index of the endpoint that currently leads its raft group (0 when none answers or
        the cluster is one member). Any member accepts writes and forwards them, but the
        forward is a peer round trip and a follower's watch only sees a commit one more
        AppendEntries later, so writes go to the leader when it is known."""
        if len(self.endpoints) < 2:
            return 0
        for i in range(len(self.endpoints)):
            st = self._probe(i)
            if st is not None and st.leader and st.leader == st.header.member_id:
                return i
        return 0

    def _probe(self, i: int):
        """Status of endpoint i (None when it does not answer); notes its wire lane port."""
        ch = _channel(self.endpoints[i], *self._creds)
        try:
            st, call = E.Maintenance.stub(ch).Status.with_call(E.StatusRequest(), timeout=1.0)
            port = dict(call.initial_metadata() or ()).get(WIRE_METADATA)
            self._wire_ports[i] = int(port) if port and port.isdigit() else 0
            return st
        except grpc.RpcError:
            return None
        finally:
            ch.close()

    def _wire_channel(self, i: int) -> SyncChannel | None:
        if not self._use_wire:
            return None
        if i not in self._wire_ports:
            self._probe(i)
        port = self._wire_ports.get(i, 0)
        if not port:
            return None
        ep = self.endpoints[i]
        host = ep.split("://", 1)[-1].rstrip("/").rpartition(":")[0]
        ca, cert, key = self._creds
        tls = client_ssl(cert, key, ca) if (ep.startswith("https://") or ca) else None
        return SyncChannel(f"{host}:{port}", tls)

    def _connect(self, i: int):
        """Talk to endpoint i (a member of an etcd cluster; any member forwards to the leader)."""
        if self._chan is not None:
            self._chan.close()
        if self._wire is not None:
            self._wire.close()
        self._ep = i % len(self.endpoints)
        self.endpoint = self.endpoints[self._ep]
        self._chan = _channel(self.endpoint, *self._creds)
        self._kvs = E.KV.stub(self._chan)
        self._maint = E.Maintenance.stub(self._chan)
        self._wire = self._wire_channel(self._ep)

    @property
    def async_writes(self) -> bool:
        """Writes from greenbridge.run_sync handlers are group-committed without blocking."""
        return greenbridge.available()

    @property
    def transport(self) -> str:
        return "wire" if self._wire is not None else "grpc"

    def _call(self, method: str, req, retry_timeouts: bool = False):
        """A unary KV call with fail-over: an unreachable member (or one without a leader) sends
        the call to the next endpoint. A timed-out write is not retried (it may have committed)."""
        retry = {grpc.StatusCode.UNAVAILABLE} | ({grpc.StatusCode.DEADLINE_EXCEEDED} if retry_timeouts else set())
        deadline = time.monotonic() + max(self.timeout, 3.0)
        while True:
            try:
                if self._wire is not None:
                    return _KV_RESP[method].FromString(
                        self._wire.call(f"/etcdserverpb.KV/{method}", req.SerializeToString(), self.timeout))
                return getattr(self._kvs, method)(req, timeout=self.timeout)
            except grpc.RpcError as e:
                if e.code() not in retry or time.monotonic() > deadline:
                    raise
                log.warning("etcd %s: %s (%s); trying the next endpoint", self.endpoint, method, e.code().name)
                lead = self._leader_endpoint()
                self._connect(lead if lead != self._ep else self._ep + 1)
                time.sleep(0.1)

    # ------------------------------------------------------------------ sync
    def status(self):
        return self._maint.Status(E.StatusRequest(), timeout=self.timeout)

    def _initial_sync(self):
        r = self._call("Range", E.RangeRequest(key=ALL, range_end=ALL), retry_timeouts=True)
        with self._lock:
            for kv in r.kvs:
                k = _s(kv.key)
                new = KV(k, self._plain(k, kv.value), kv.create_revision, kv.mod_revision, kv.version)
                self.kv[k] = new
                self._index_put(k, new)
            self.rev = self.compact_rev = self.synced_rev = r.header.revision

    def start(self, loop):
        """Apply followed events on `loop` (the apiserver's) as they arrive; until then they wait
        in the queue for the next write or drain()."""
        self._loop = loop
        self._kick()

    def _requests(self, first):
        yield first
        self._stop.wait()

    def _follow(self):
        backoff, ep, chan = 0.1, self._ep, None
        while not self._stop.is_set():
            req = E.WatchRequest(create_request=E.WatchCreateRequest(key=ALL, range_end=ALL,
                                                                     start_revision=self.synced_rev + 1, prev_kv=True))
            if chan is None:
                chan = _channel(self.endpoints[ep % len(self.endpoints)], *self._creds)
                self._watch_wire = self._wire_channel(ep % len(self.endpoints))
            try:
                # every member applies the same log, so a watch resumes at the same revision on any of them
                if self._watch_wire is not None:
                    stream = (E.WatchResponse.FromString(b) for b in
                              self._watch_wire.stream("/etcdserverpb.Watch/Watch", req.SerializeToString()))
                else:
                    self._watch_call = stream = E.Watch.stub(chan).Watch(self._requests(req))
                for resp in stream:
                    if resp.compact_revision:
                        self._events.put(("resync", None))
                        self._kick()
                        break
                    if resp.canceled:
                        break
                    if resp.events:
                        self.synced_rev = max(self.synced_rev, resp.events[-1].kv.mod_revision)
                        self._events.put(("events", list(resp.events)))
                        self._kick()
                        backoff = 0.1
            except grpc.RpcError as e:
                if self._stop.is_set():
                    break
                log.warning("etcd watch on %s broke (%s); re-watching from %d", self.endpoints[ep % len(self.endpoints)],
                            e.code(), self.synced_rev + 1)
                chan.close()
                if self._watch_wire is not None:
                    self._watch_wire.close()
                chan, ep = None, ep + 1
            if self._stop.wait(backoff):
                break
            backoff = min(backoff * 2, 2.0)
        if chan is not None:
            chan.close()
        if self._watch_wire is not None:
            self._watch_wire.close()

    def _kick(self):
        loop = self._loop
        if loop is not None and not loop.is_closed():
            try:
                loop.call_soon_threadsafe(self.drain)
            except RuntimeError:
                pass

    def drain(self, until: int = 0, timeout: float | None = None):
        """Apply queued watch events (on the loop thread). With `until`, block until the replica
        has reached that revision."""
        deadline = time.monotonic() + (timeout or self.timeout)
        while True:
            try:
                if until and self.rev < until:
                    item = self._events.get(timeout=max(0.0, deadline - time.monotonic()))
                else:
                    item = self._events.get_nowait()
            except queue.Empty:
                if until and self.rev < until:
                    raise TimeoutError(f"etcd replica did not reach revision {until} (at {self.rev})")
                return
            kind, payload = item
            if kind == "resync":
                self._resync()
            else:
                for ev in payload:
                    self._apply(ev)

    def _apply(self, ev):
        key, rev = _s(ev.kv.key), ev.kv.mod_revision
        with self._lock:
            if rev <= self.rev and key in self.kv and self.kv[key].mod_rev >= rev:
                return                                   # already applied (re-watch overlap)
            cur = self.kv.get(key)
            if ev.type == EV_PUT:
                new = KV(key, self._plain(key, ev.kv.value), ev.kv.create_revision, rev, ev.kv.version)
                self.kv[key] = new
                self._index_put(key, new)
                self.rev = max(self.rev, rev)
                if key != FENCE:                        # the fence is bookkeeping, not an object
                    self._commit(Event(PUT, new, cur, rev), None)
            else:
                self.rev = max(self.rev, rev)
                if cur is None:
                    return
                del self.kv[key]
                self._index_del(key)
                self._commit(Event(DELETE, KV(key, cur.value, cur.create_rev, rev, 0), cur, rev), None)

    def _plain(self, key: str, value: bytes) -> bytes:
        return self.transformer.from_disk(key, value) if self.transformer is not None and key != FENCE else value

    def _sealed(self, key: str, value: bytes) -> bytes:
        return self.transformer.to_disk(key, value) if self.transformer is not None else value

    def _resync(self):
        """The watch fell behind a compaction: re-list and turn the difference into events."""
        self.resyncs += 1
        r = self._call("Range", E.RangeRequest(key=ALL, range_end=ALL), retry_timeouts=True)
        seen = set()
        with self._lock:
            for kv in r.kvs:
                k = _s(kv.key)
                seen.add(k)
                cur = self.kv.get(k)
                if cur is None or cur.mod_rev != kv.mod_revision:
                    self._apply(E.Event(type=EV_PUT, kv=kv))
            for k in [k for k in self.kv if k not in seen]:
                self._apply(E.Event(type=1, kv=E.KeyValue(key=_b(k), mod_revision=r.header.revision)))
            self.rev = max(self.rev, r.header.revision)
            self.synced_rev = max(self.synced_rev, r.header.revision)

    # ------------------------------------------------------------------ writes
    def _txn(self, compare, success, failure):
        try:
            return self._call("Txn", E.TxnRequest(compare=compare, success=success, failure=failure))
        except grpc.RpcError as e:
            raise ConnectionError(f"etcd {self.endpoint}: {e.code().name}: {e.details()}") from None

    @staticmethod
    def _object_compare(bkey: bytes, expect_mod_rev: int | None, delete: bool):
        if expect_mod_rev is not None and (expect_mod_rev or not delete):
            return E.Compare(key=bkey, target=T_MOD, result=EQUAL, mod_revision=expect_mod_rev)
        if delete:
            return E.Compare(key=bkey, target=T_VERSION, result=GREATER, version=0)      # must exist
        return None

    @staticmethod
    def _object_ok(cur_mod: int, expect_mod_rev: int | None, delete: bool) -> bool:
        if expect_mod_rev is not None and (expect_mod_rev or not delete):
            return cur_mod == expect_mod_rev
        return not delete or cur_mod != 0

    def _conflict(self, key: str, orr, expect_mod_rev: int | None, delete: bool) -> Exception:
        """The caller's error for an object compare that failed (replica caught up first)."""
        self.drain(until=orr.header.revision)
        cur = self.kv.get(key)
        if cur is None and orr.kvs:
            kv = orr.kvs[0]
            cur = KV(key, self._plain(key, kv.value), kv.create_revision, kv.mod_revision, kv.version)
        if expect_mod_rev == 0 and not delete:
            return KeyExists(key)
        if cur is None:
            return KeyNotFound(key)
        return CASFailed(cur)

    def _write(self, key: str, value, expect_mod_rev: int | None, delete: bool):
        """One fenced CAS Txn. The fence compare fails when any other apiserver committed since
        this replica's view, so a success means the commit revision is exactly rev+1 and the
        resourceVersion rendered into the value is right; a fence-only failure catches up and
        retries, an object compare failure is the caller's conflict. Returns (the op's
        ResponseOp, commit revision, the bytes written)."""
        bkey = _b(key)
        for _ in range(1000):
            self.drain()
            fence = self.kv.get(FENCE)
            guess = self.rev + 1
            cmp = [E.Compare(key=_FENCE_B, target=T_MOD, result=EQUAL, mod_revision=fence.mod_rev if fence else 0)]
            oc = self._object_compare(bkey, expect_mod_rev, delete)
            if oc is not None:
                cmp.append(oc)
            data = None
            if delete:
                op = E.RequestOp(request_delete_range=E.DeleteRangeRequest(key=bkey, prev_kv=True))
            else:
                data = value(guess) if callable(value) else value
                op = E.RequestOp(request_put=E.PutRequest(key=bkey, value=self._sealed(key, data)))
            resp = self._txn(cmp, [E.RequestOp(request_put=E.PutRequest(key=_FENCE_B)), op],
                             [E.RequestOp(request_range=E.RangeRequest(key=_FENCE_B)),
                              E.RequestOp(request_range=E.RangeRequest(key=bkey))])
            if resp.succeeded:
                rev = resp.header.revision
                if data is not None and callable(value) and rev != guess:
                    # a writer outside the fence committed in between: re-render at the real revision
                    log.warning("etcd3: %s committed at %d, rendered for %d; rewriting", key, rev, guess)
                    self.drain(until=rev)
                    return self._write(key, value, rev, False)
                if rev == guess and self.rev == guess - 1:
                    # nothing else committed in between (the revision moved by exactly this Txn), so
                    # the replica is exact at rev-1 and this write can be applied now; the watch's
                    # copy of the same events is skipped when it arrives
                    self._apply_own([(key, data, delete)], rev)
                else:
                    self.drain(until=rev)
                return resp.responses[1], rev, data
            frr, orr = resp.responses[0].response_range, resp.responses[1].response_range
            cur_mod = orr.kvs[0].mod_revision if orr.kvs else 0
            if not self._object_ok(cur_mod, expect_mod_rev, delete):
                raise self._conflict(key, orr, expect_mod_rev, delete)
            self.drain(until=frr.kvs[0].mod_revision if frr.kvs else 0)     # only the fence moved
        raise ConnectionError(f"etcd3: {key}: the revision fence kept moving")

    def _apply_own(self, ops, rev: int):
        """Apply this replica's own committed Txn (fence + ops, all at `rev`) without waiting
        for the watch to bring it back."""
        fence = self.kv.get(FENCE)
        self._apply(E.Event(type=EV_PUT, kv=E.KeyValue(key=_FENCE_B, create_revision=fence.create_rev if fence else rev,
                                                        mod_revision=rev, version=(fence.version + 1) if fence else 1)))
        for key, data, delete in ops:
            cur = self.kv.get(key)
            if delete:
                self._apply(E.Event(type=1, kv=E.KeyValue(key=_b(key), mod_revision=rev)))
            else:
                self._apply(E.Event(type=EV_PUT, kv=E.KeyValue(key=_b(key), value=self._sealed(key, data),
                                                               create_revision=cur.create_rev if cur else rev,
                                                               mod_revision=rev, version=(cur.version + 1) if cur else 1)))

    # ------------------------------------------------------------------ group commit (bridged writes)
    async def _submit_op(self, key: str, value, expect_mod_rev: int | None, delete: bool):
        """A write from a request handler running under greenbridge.run_sync: queued, and
        committed together with every other write queued meanwhile in ONE fenced Txn (one
        revision, one raft entry), so concurrent requests share the round trip instead of
        each stalling the loop for one."""
        op = _Op(key, value, expect_mod_rev, delete, self._loop.create_future())
        self._pending.append(op)
        if self._flusher is None:
            self._flusher = self._loop.create_task(self._flush())
        return await op.fut

    async def _flush(self):
        try:
            while self._pending:
                batch, rest, keys = [], [], set()
                for op in self._pending:          # one op per key per Txn (etcd refuses duplicates)
                    if op.solo and not batch:
                        batch.append(op)          # an op etcd refused in a batch is retried alone
                        keys.add(op.key)
                    elif op.key in keys or len(batch) >= MAX_BATCH or op.solo or (batch and batch[0].solo):
                        rest.append(op)
                    else:
                        keys.add(op.key)
                        batch.append(op)
                self._pending = rest
                try:
                    redo = await self._commit_batch(batch)
                except Exception as e:        # noqa: BLE001
                    redo = []
                    if len(batch) > 1 and _invalid_argument(e):
                        # etcd refused the Txn as a whole (too many ops / too large): each write
                        # alone may well succeed, so none fails for the others
                        log.warning("etcd3: batch of %d refused (%s); retrying one by one", len(batch), e)
                        for op in batch:
                            op.solo = True
                        redo = batch
                    else:
                        for op in batch:          # every waiter gets the failure
                            if not op.fut.done():
                                op.fut.set_exception(e)
                self._pending[:0] = redo
        finally:
            self._flusher = None

    async def _commit_batch(self, batch: list) -> list:
        """One fenced Txn for `batch`; resolves the ops it settles, returns those to retry."""
        self.drain()
        fence = self.kv.get(FENCE)
        guess = self.rev + 1
        cmp = [E.Compare(key=_FENCE_B, target=T_MOD, result=EQUAL, mod_revision=fence.mod_rev if fence else 0)]
        success = [E.RequestOp(request_put=E.PutRequest(key=_FENCE_B))]
        failure = [E.RequestOp(request_range=E.RangeRequest(key=_FENCE_B))]
        size, over = 0, []
        for n, op in enumerate(batch):
            bkey = _b(op.key)
            if n and size > MAX_BATCH_BYTES:
                over = batch[n:]                  # past the request-size budget: next Txn
                batch = batch[:n]
                break
            oc = self._object_compare(bkey, op.expect, op.delete)
            if oc is not None:
                cmp.append(oc)
            if op.delete:
                op.data = None
                success.append(E.RequestOp(request_delete_range=E.DeleteRangeRequest(key=bkey, prev_kv=True)))
            else:
                op.data = op.value(guess) if callable(op.value) else op.value
                sealed = self._sealed(op.key, op.data)
                size += len(sealed)
                success.append(E.RequestOp(request_put=E.PutRequest(key=bkey, value=sealed)))
            size += 2 * len(bkey) + 32
            failure.append(E.RequestOp(request_range=E.RangeRequest(key=bkey)))
        redo = await self._commit_ops(batch, cmp, success, failure, guess)
        return over + redo

    async def _commit_ops(self, batch, cmp, success, failure, guess) -> list:
        resp = await self._atxn(E.TxnRequest(compare=cmp, success=success, failure=failure))
        if resp.succeeded:
            rev = resp.header.revision
            redo = []
            if rev != guess:
                self.drain(until=rev)
                # a writer outside the fence committed in between: re-render at the real revision
                redo = [op for op in batch if callable(op.value) and not op.delete]
                for op in redo:
                    log.warning("etcd3: %s committed at %d, rendered for %d; rewriting", op.key, rev, guess)
                    op.expect = rev
            elif self.rev == guess - 1:
                self._apply_own([(op.key, op.data, op.delete) for op in batch], rev)
            else:
                self.drain(until=rev)
            for i, op in enumerate(batch):
                if op not in redo and not op.fut.done():     # a cancelled request's write still commits
                    op.fut.set_result((resp.responses[1 + i], rev, op.data))
            return redo
        redo = []
        self.drain(until=resp.header.revision)
        for i, op in enumerate(batch):
            orr = resp.responses[1 + i].response_range
            cur_mod = orr.kvs[0].mod_revision if orr.kvs else 0
            if self._object_ok(cur_mod, op.expect, op.delete):
                redo.append(op)                   # failed only with the rest: next Txn
            elif not op.fut.done():
                op.fut.set_exception(self._conflict(op.key, orr, op.expect, op.delete))
        if redo and len(redo) == len(batch):
            op = redo[0]                          # the fence alone moved: caught up above
            op.tries += 1
            if op.tries > 1000:
                for o in redo:
                    if not o.fut.done():
                        o.fut.set_exception(ConnectionError(f"etcd3: {o.key}: the revision fence kept moving"))
                return []
        return redo

    async def _atxn(self, req):
        """The Txn without blocking the loop: over the wire lane's async connection when the
        member has one, else the blocking gRPC call in a worker thread. A lost connection
        falls back to the blocking path, which fails over between endpoints."""
        try:
            if self._wire is not None:
                target = self._wire.target
                if self._achan is None or self._achan.target != target:
                    if self._achan is not None:
                        await self._achan.close()
                    self._achan = PeerChannel(target, self._wire.ssl)
                return E.TxnResponse.FromString(await self._achan.call("/etcdserverpb.KV/Txn", req.SerializeToString(),
                                                                       self.timeout))
            return await self._loop.run_in_executor(None, lambda: self._kvs.Txn(req, timeout=self.timeout))
        except grpc.RpcError as e:
            if e.code() != grpc.StatusCode.UNAVAILABLE:
                raise ConnectionError(f"etcd {self.endpoint}: {e.code().name}: {e.details()}") from None
        return self._txn(req.compare, req.success, req.failure)

    def put(self, key: str, value, expect_mod_rev: int | None = None) -> KV:
        if expect_mod_rev:
            self._inject_conflict(self.kv.get(key))
        if self._loop is not None and greenbridge.bridged():
            _, rev, data = greenbridge.await_only(self._submit_op(key, value, expect_mod_rev, False))
        else:
            _, rev, data = self._write(key, value, expect_mod_rev, False)
        got = self.kv.get(key)
        if got is not None and got.mod_rev == rev:
            return got
        return KV(key, data, got.create_rev if got else rev, rev, 0)     # already replaced in the replica

    def delete(self, key: str, expect_mod_rev: int | None = None) -> KV:
        if expect_mod_rev:
            self._inject_conflict(self.kv.get(key))
        if self._loop is not None and greenbridge.bridged():
            r, _, _ = greenbridge.await_only(self._submit_op(key, None, expect_mod_rev, True))
        else:
            r, _, _ = self._write(key, None, expect_mod_rev, True)
        pk = r.response_delete_range.prev_kvs[0]
        return KV(key, self._plain(key, pk.value), pk.create_revision, pk.mod_revision, pk.version)

    def batch(self, ops):
        raise NotImplementedError("Etcd3Store writes go through put/delete (one etcd Txn each)")

    def compact(self, rev: int):
        try:
            self._call("Compact", E.CompactionRequest(revision=rev))
        except grpc.RpcError as e:
            if e.code() != grpc.StatusCode.OUT_OF_RANGE:
                raise
        super().compact(rev)

    def snapshot(self):
        pass                       # etcd owns durability

    def close(self):
        self._stop.set()
        if self._watch_call is not None:
            self._watch_call.cancel()
        if self._watch_wire is not None:
            self._watch_wire.close()            # unblocks the watch thread's read
        if self._thread is not None:
            self._thread.join(timeout=5)
        super().close()
        self._chan.close()
        if self._wire is not None:
            self._wire.close()
        ach, self._achan = self._achan, None
        if ach is not None and ach._writer is not None:
            ach.closed = True
            ach._writer.close()                 # its reader task ends with the connection


def prefix_range(prefix: str) -> tuple[bytes, bytes]:
    return _b(prefix), prefix_end(_b(prefix))
