"""Raft consensus for `amdkube etcd --initial-cluster`: a replicated log in front of the MVCC
store, so the store survives the loss of a minority of members (the role etcd's raft plays
under the reference's apiservers; SURVEY §5.4 scoped the store to one process, this lifts it).

The algorithm is Raft as published (Ongaro & Ousterhout): terms, randomized election timeouts,
RequestVote with the up-to-date check, AppendEntries with the log-matching property and a
conflict-index hint for fast back-off, commit only of current-term entries by majority match,
a no-op entry on election, InstallSnapshot for followers behind the compacted log. Membership
is static (`--initial-cluster`). Linearizable reads use the leader lease: a majority
acknowledged an AppendEntries within the election timeout.

Durability, per member under `<data-dir>/raft/`: `state.json` (term, vote; fsynced before a
vote or a term change is answered), `log.bin` (length-prefixed Entry records, fdatasynced
before AppendEntries is acknowledged), `snap.bin` (state-machine snapshot + last included
index/term; the log is cut behind it every `compact_every` applied entries).

Group commit (etcd's Ready batching, vendor/github.com/coreos/etcd/raft/node.go:52 and
etcdserver/raft.go:134): a proposal only appends to the leader's in-memory log and wakes the
flusher and the replicators. The flusher writes every entry appended since its last write with
ONE write + fdatasync in a worker thread, while proposals keep arriving on the loop; the
replicators ship everything a follower lacks in one AppendEntries (≤ MAX_BATCH entries), and a
follower persists the batch with one fdatasync before acknowledging. The leader counts itself
toward the commit quorum only up to its own persisted index (`persisted`), so N concurrent
proposals cost about one leader fsync + one round trip + one follower fsync, not N of each.

The state machine is the caller's: `apply(index, data) -> result` (deterministic: every
member applies the same entries in the same order, so every member's store has the same
revisions), `snapshot() -> bytes`, `restore(bytes)`. Peers call the `amdkube.raft.Raft` methods
over the peer transport (store/peerwire.py: framed protobuf over TCP, like etcd's rafthttp
rather than gRPC) on the peer listener only (store/etcdserver.py serves it apart from the
client API, under peer TLS when configured); `channel(target)` makes the peer channels.

Commit notification has its own lane per follower (`_notify_commit`), so the empty
AppendEntries that tells a follower about a new commit index never holds the next batch of
entries back by a round trip.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import random
import struct
import time

import grpc

from ..grpcdesc.compiler import ProtoModule
from .peerwire import PeerChannel, stub as peer_stub

log = logging.getLogger("amdkube.raft")

RAFT = ProtoModule("""
syntax = "proto3";
package amdkube.raft;

service Raft {
  rpc RequestVote(VoteRequest) returns (VoteResponse) {}
  rpc AppendEntries(AppendRequest) returns (AppendResponse) {}
  rpc InstallSnapshot(SnapshotRequest) returns (SnapshotResponse) {}
}
message Entry { uint64 term = 1; uint64 index = 2; bytes data = 3; }
message VoteRequest { uint64 term = 1; string candidate = 2; uint64 last_log_index = 3; uint64 last_log_term = 4; }
message VoteResponse { uint64 term = 1; bool granted = 2; }
message AppendRequest {
  uint64 term = 1;
  string leader = 2;
  uint64 prev_log_index = 3;
  uint64 prev_log_term = 4;
  repeated Entry entries = 5;
  uint64 leader_commit = 6;
}
message AppendResponse { uint64 term = 1; bool success = 2; uint64 match_index = 3; uint64 conflict_index = 4; }
message SnapshotRequest { uint64 term = 1; string leader = 2; uint64 last_index = 3; uint64 last_term = 4; bytes data = 5; }
message SnapshotResponse { uint64 term = 1; }
""", "amdkube/raft.proto")

FOLLOWER, CANDIDATE, LEADER = "follower", "candidate", "leader"
MAX_BATCH = 512


class NotLeader(Exception):
    def __init__(self, leader: str | None):
        super().__init__(f"not the leader (leader: {leader or 'unknown'})")
        self.leader = leader


class Raft:
    def __init__(self, name: str, peers: dict[str, str], data_dir: str | None, sm,
                 heartbeat: float = 0.1, election: float = 1.0, compact_every: int = 10_000, fsync: bool = True,
                 channel=None):
        self.name, self.peers, self.sm = name, dict(peers), sm
        self._channel = channel or PeerChannel
        self.others = [p for p in sorted(peers) if p != name]
        self.heartbeat, self.election, self.compact_every, self.fsync = heartbeat, election, compact_every, fsync
        self.dir = os.path.join(data_dir, "raft") if data_dir else None
        self.term, self.voted_for = 0, None
        self.log: list = []                      # Entry messages, log[0].index == snap_index + 1
        self.snap_index = self.snap_term = 0
        self.commit = self.applied = 0
        self.role, self.leader = FOLLOWER, None
        self.next_index: dict[str, int] = {}
        self.match_index: dict[str, int] = {}
        self.acked: dict[str, float] = {}
        self._pending: dict[int, tuple[int, asyncio.Future]] = {}
        self._kick: dict[str, asyncio.Event] = {}
        self._commit_kick: dict[str, asyncio.Event] = {}
        self._tasks: list[asyncio.Task] = []
        self._repl: list[asyncio.Task] = []
        self._stubs: dict[str, object] = {}
        self._chans: list = []
        self._last_heard = time.monotonic()
        self._timeout = self._new_timeout()
        self._logf = None
        self.persisted = 0                       # highest log index durably on this member's disk
        self._disk = asyncio.Lock()              # log file writers: the flusher, AppendEntries, snapshots
        self._flushing = False                   # a flusher write is in flight in its worker thread
        self._flush_ev = asyncio.Event()
        self._apply_waiters: list[tuple[int, asyncio.Future]] = []
        self.leader_changed = asyncio.Event()
        self._load()
        self.persisted = self.last_index()

    # ------------------------------------------------------------------ persistence
    def _load(self):
        if not self.dir:
            return
        from .mvcc import lock_data_dir
        self._dir_lock = lock_data_dir(self.dir)
        st = os.path.join(self.dir, "state.json")
        if os.path.exists(st):
            d = json.load(open(st))
            self.term, self.voted_for = d["term"], d["vote"]
        sp = os.path.join(self.dir, "snap.bin")
        if os.path.exists(sp):
            raw = open(sp, "rb").read()
            snap = RAFT.SnapshotRequest.FromString(raw)
            self.snap_index, self.snap_term = snap.last_index, snap.last_term
            self.sm.restore(snap.data)
            self.commit = self.applied = self.snap_index
        lp = os.path.join(self.dir, "log.bin")
        if os.path.exists(lp):
            data = open(lp, "rb").read()
            i = 0
            while i + 4 <= len(data):
                (n,) = struct.unpack_from(">I", data, i)
                if i + 4 + n > len(data):
                    break                                   # torn tail
                e = RAFT.Entry.FromString(data[i + 4:i + 4 + n])
                i += 4 + n
                if e.index <= self.snap_index:
                    continue
                if e.index != self.last_index() + 1:
                    break
                self.log.append(e)
            if i != len(data):
                self._rewrite_log()
        self._logf = open(lp, "ab")

    def _save_state(self):
        if not self.dir:
            return
        p = os.path.join(self.dir, "state.json")
        with open(p + ".tmp", "w") as f:
            json.dump({"term": self.term, "vote": self.voted_for}, f)
            f.flush()
            if self.fsync:
                os.fsync(f.fileno())
        os.replace(p + ".tmp", p)

    def _write_entries(self, f, entries):
        f.write(b"".join(struct.pack(">I", len(b)) + b for b in (e.SerializeToString() for e in entries)))
        f.flush()
        if self.fsync:
            os.fdatasync(f.fileno())

    def _append_disk(self, entries):
        if self._logf is not None:
            self._write_entries(self._logf, entries)
        self.persisted = self.last_index()

    def _rewrite_log(self):
        if not self.dir:
            return
        p = os.path.join(self.dir, "log.bin")
        if self._logf is not None:
            self._logf.close()
        with open(p + ".tmp", "wb") as f:
            f.write(b"".join(struct.pack(">I", len(b)) + b for b in (e.SerializeToString() for e in self.log)))
            f.flush()
            if self.fsync:
                os.fsync(f.fileno())
        os.replace(p + ".tmp", p)
        self._logf = open(p, "ab")
        self.persisted = self.last_index()

    def _save_snapshot(self, data: bytes):
        if not self.dir:
            return
        p = os.path.join(self.dir, "snap.bin")
        with open(p + ".tmp", "wb") as f:
            f.write(RAFT.SnapshotRequest(last_index=self.snap_index, last_term=self.snap_term, data=data).SerializeToString())
            f.flush()
            if self.fsync:
                os.fsync(f.fileno())
        os.replace(p + ".tmp", p)

    # ------------------------------------------------------------------ log helpers
    def last_index(self) -> int:
        return self.log[-1].index if self.log else self.snap_index

    def last_term(self) -> int:
        return self.log[-1].term if self.log else self.snap_term

    def term_at(self, i: int) -> int | None:
        if i == self.snap_index:
            return self.snap_term
        j = i - self.snap_index - 1
        if 0 <= j < len(self.log):
            return self.log[j].term
        return None

    def _new_timeout(self) -> float:
        return self.election * (1 + random.random())

    def quorum(self) -> int:
        return len(self.peers) // 2 + 1

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        for p in self.others:
            ch = self._channel(self.peers[p])
            self._chans.append(ch)
            self._stubs[p] = peer_stub(RAFT.Raft, ch)
        self._last_heard = time.monotonic()
        self._tasks.append(asyncio.create_task(self._ticker(), name="raft-ticker"))
        self._tasks.append(asyncio.create_task(self._flusher(), name="raft-flusher"))
        if len(self.peers) == 1:
            await self._become_leader()
        return self

    async def stop(self):
        from ..utils import cancel_and_wait
        await cancel_and_wait(self._repl + self._tasks)
        for ch in self._chans:
            await ch.close()
        self._fail_pending(NotLeader(None))
        for _, fut in self._apply_waiters:
            if not fut.done():
                fut.cancel()
        async with self._disk:                 # a flusher write still in its thread finishes first
            if self._logf is not None:
                self._logf.close()
                self._logf = None
        if getattr(self, "_dir_lock", None) is not None:
            self._dir_lock.close()
            self._dir_lock = None

    def handler(self):
        return RAFT.Raft.handler(self)

    # ------------------------------------------------------------------ roles
    def _step_down(self, term: int, leader: str | None = None):
        if term > self.term:
            self.term, self.voted_for = term, None
            self._save_state()
        was_leader = self.role == LEADER
        self.role = FOLLOWER
        if leader is not None and leader != self.leader:
            self.leader = leader
            self.leader_changed.set()
        if was_leader:
            for t in self._repl:
                t.cancel()
            self._repl = []
            self._fail_pending(NotLeader(self.leader))

    def _fail_pending(self, exc):
        for _, (_, fut) in list(self._pending.items()):
            if not fut.done():
                fut.set_exception(exc)
        self._pending.clear()

    async def _ticker(self):
        while True:
            await asyncio.sleep(self.heartbeat / 2)
            if self.role != LEADER and time.monotonic() - self._last_heard > self._timeout:
                await self._campaign()

    async def _campaign(self):
        self.role = CANDIDATE
        self.term += 1
        self.voted_for = self.name
        self._save_state()
        self.leader = None
        self._last_heard = time.monotonic()
        self._timeout = self._new_timeout()
        term = self.term
        req = RAFT.VoteRequest(term=term, candidate=self.name, last_log_index=self.last_index(), last_log_term=self.last_term())

        async def ask(p):
            try:
                return await self._stubs[p].RequestVote(req, timeout=self.election)
            except grpc.RpcError:
                return None
        votes = 1
        for r in await asyncio.gather(*(ask(p) for p in self.others)):
            if r is None:
                continue
            if r.term > self.term:
                self._step_down(r.term)
                return
            votes += bool(r.granted)
        if self.role == CANDIDATE and self.term == term and votes >= self.quorum():
            await self._become_leader()

    async def _become_leader(self):
        self.role, self.leader = LEADER, self.name
        self.leader_changed.set()
        log.info("raft %s: leader for term %d", self.name, self.term)
        nxt = self.last_index() + 1
        self.next_index = {p: nxt for p in self.others}
        self.match_index = {p: 0 for p in self.others}
        self.acked = {}
        self._kick = {p: asyncio.Event() for p in self.others}
        self._commit_kick = {p: asyncio.Event() for p in self.others}
        self._repl = [asyncio.create_task(self._replicate(p, self.term), name=f"raft-repl-{p}") for p in self.others]
        self._repl += [asyncio.create_task(self._notify_commit(p, self.term), name=f"raft-commit-{p}")
                       for p in self.others]
        self._append_local(b"")                       # a no-op of this term lets the commit index move
        if hasattr(self.sm, "on_leader"):
            self.sm.on_leader()
        self._advance_commit()

    # ------------------------------------------------------------------ proposals
    def _append_local(self, data: bytes) -> int:
        """Leader append: memory only; the flusher persists it with whatever else arrives
        meanwhile (group commit) and the replicators ship it in their next batch."""
        e = RAFT.Entry(term=self.term, index=self.last_index() + 1, data=data)
        self.log.append(e)
        self._flush_ev.set()
        for ev in self._kick.values():
            ev.set()
        return e.index

    async def _flusher(self):
        """One write + fdatasync for every entry appended since the previous one."""
        while True:
            await self._flush_ev.wait()
            self._flush_ev.clear()
            async with self._disk:
                lo, hi = self.persisted + 1, self.last_index()
                if hi < lo:
                    continue
                entries = self.log[max(0, lo - self.snap_index - 1):hi - self.snap_index]
                if self._logf is not None and entries:
                    self._flushing = True
                    try:
                        await asyncio.to_thread(self._write_entries, self._logf, entries)
                    except OSError as e:
                        log.error("raft %s: log write failed: %s", self.name, e)
                        await asyncio.sleep(self.heartbeat)
                        self._flush_ev.set()
                        continue
                    finally:
                        self._flushing = False
                self.persisted = max(self.persisted, hi)
            self._advance_commit()

    async def propose(self, data: bytes, timeout: float = 10.0):
        """Replicate `data`; the state machine's result once a majority has it and it is applied here."""
        if self.role != LEADER:
            raise NotLeader(self.leader)
        idx = self._append_local(data)
        fut = asyncio.get_running_loop().create_future()
        self._pending[idx] = (self.term, fut)
        return await asyncio.wait_for(fut, timeout)

    def has_lease(self) -> bool:
        """Leader lease for linearizable reads: a majority heard from us within the election timeout."""
        if self.role != LEADER:
            return False
        now = time.monotonic()
        return 1 + sum(1 for p in self.others if now - self.acked.get(p, 0) < self.election) >= self.quorum()

    async def read_barrier(self, timeout: float = 5.0):
        """Wait until this leader may serve a linearizable read (lease held, own term committed)."""
        end = time.monotonic() + timeout
        while True:
            if self.role != LEADER:
                raise NotLeader(self.leader)
            if self.has_lease() and self.term_at(self.commit) == self.term and self.applied >= self.commit:
                return self.commit
            if time.monotonic() > end:
                raise TimeoutError("raft: leadership not confirmed")
            for ev in self._kick.values():
                ev.set()
            await asyncio.sleep(self.heartbeat / 4)

    # ------------------------------------------------------------------ replication (leader)
    async def _replicate(self, p: str, term: int):
        stub, kick = self._stubs[p], self._kick[p]
        while self.role == LEADER and self.term == term:
            kick.clear()             # anything appended or committed from here on triggers another send
            ni = self.next_index[p]
            try:
                if ni <= self.snap_index:
                    data = self.sm.snapshot() if self.applied == self.snap_index else None
                    if data is None:
                        async with self._disk:
                            self._compact(force=True)
                        continue
                    r = await stub.InstallSnapshot(RAFT.SnapshotRequest(term=term, leader=self.name, last_index=self.snap_index,
                                                                         last_term=self.snap_term, data=data),
                                                   timeout=max(self.election * 5, 10))
                    if r.term > self.term:
                        self._step_down(r.term)
                        return
                    self.match_index[p] = max(self.match_index[p], self.snap_index)
                    self.next_index[p] = self.snap_index + 1
                    self.acked[p] = time.monotonic()
                    continue
                prev = ni - 1
                start = ni - self.snap_index - 1
                entries = self.log[start:start + MAX_BATCH]
                req = RAFT.AppendRequest(term=term, leader=self.name, prev_log_index=prev, prev_log_term=self.term_at(prev) or 0,
                                         leader_commit=self.commit)
                req.entries.extend(entries)
                sent = time.monotonic()
                r = await stub.AppendEntries(req, timeout=self.election)
            except grpc.RpcError:
                await asyncio.sleep(self.heartbeat)
                continue
            if r.term > self.term:
                self._step_down(r.term)
                return
            if self.role != LEADER or self.term != term:
                return
            self.acked[p] = sent
            if r.success:
                self.match_index[p] = max(self.match_index[p], prev + len(entries))
                self.next_index[p] = self.match_index[p] + 1
                self._advance_commit()
                if self.next_index[p] <= self.last_index():
                    continue                                # more to send right away
            else:
                self.next_index[p] = max(1, min(r.conflict_index or ni - 1, ni - 1))
                continue
            try:
                await asyncio.wait_for(kick.wait(), self.heartbeat)
            except asyncio.TimeoutError:
                pass

    async def _notify_commit(self, p: str, term: int):
        """The commit lane: an empty AppendEntries at the follower's known match point carrying
        the new commit index (etcd's bcastAppend after maybeCommit), on its own call so it never
        delays the next batch of entries behind a round trip, as one in-flight call per peer
        would. Followers apply at once, so their watches and ReadIndex reads see the write."""
        stub, kick = self._stubs[p], self._commit_kick[p]
        told = 0
        while self.role == LEADER and self.term == term:
            await kick.wait()
            kick.clear()
            prev = self.match_index.get(p, 0)
            commit = min(self.commit, prev)
            if commit <= told or prev < self.snap_index:
                continue
            pt = self.term_at(prev)
            if pt is None:
                continue
            try:
                r = await stub.AppendEntries(RAFT.AppendRequest(term=term, leader=self.name, prev_log_index=prev,
                                                                prev_log_term=pt, leader_commit=commit),
                                             timeout=self.election)
            except grpc.RpcError:
                continue
            if r.term > self.term:
                self._step_down(r.term)
                return
            if r.success:
                told = commit

    def _advance_commit(self):
        if self.role != LEADER:
            return
        matches = sorted([self.persisted] + [self.match_index[p] for p in self.others], reverse=True)
        n = matches[self.quorum() - 1]
        if n > self.commit and self.term_at(n) == self.term:
            self.commit = n
            self._apply()
            for ev in self._commit_kick.values():     # tell followers about the new commit index now
                ev.set()

    # ------------------------------------------------------------------ apply
    def _apply(self):
        while self.applied < self.commit:
            i = self.applied + 1
            e = self.log[i - self.snap_index - 1]
            try:
                result, err = self.sm.apply(i, e.data) if e.data else None, None
            except Exception as ex:                     # a failing entry fails identically everywhere
                result, err = None, ex
            self.applied = i
            ent = self._pending.pop(i, None)
            if ent is not None and not ent[1].done():
                if ent[0] != e.term:
                    ent[1].set_exception(NotLeader(self.leader))
                elif err is not None:
                    ent[1].set_exception(err)
                else:
                    ent[1].set_result(result)
        if self._apply_waiters:
            keep = []
            for idx, fut in self._apply_waiters:
                if idx <= self.applied:
                    if not fut.done():
                        fut.set_result(None)
                else:
                    keep.append((idx, fut))
            self._apply_waiters = keep
        self._compact()

    async def wait_applied(self, index: int, timeout: float = 5.0):
        """Until this member has applied `index` (a follower serving a ReadIndex read)."""
        if self.applied >= index:
            return
        fut = asyncio.get_running_loop().create_future()
        self._apply_waiters.append((index, fut))
        await asyncio.wait_for(fut, timeout)

    def _compact(self, force: bool = False):
        if self._flushing:
            return                  # the flusher's thread holds the log file; the next apply compacts
        if not force and self.applied - self.snap_index < self.compact_every:
            return
        if self.applied <= self.snap_index:
            return
        data = self.sm.snapshot()
        cut = self.applied - self.snap_index
        self.snap_term = self.term_at(self.applied)
        self.snap_index = self.applied
        self.log = self.log[cut:]
        self._save_snapshot(data)
        self._rewrite_log()

    # ------------------------------------------------------------------ RPC handlers
    async def RequestVote(self, req, ctx):
        if req.term > self.term:
            self._step_down(req.term)
        granted = False
        if req.term == self.term and self.voted_for in (None, req.candidate):
            up_to_date = (req.last_log_term, req.last_log_index) >= (self.last_term(), self.last_index())
            if up_to_date:
                self.voted_for = req.candidate
                self._save_state()
                self._last_heard = time.monotonic()
                granted = True
        return RAFT.VoteResponse(term=self.term, granted=granted)

    async def AppendEntries(self, req, ctx):
        async with self._disk:
            return self._append_entries(req)

    def _append_entries(self, req):
        if req.term < self.term:
            return RAFT.AppendResponse(term=self.term, success=False)
        if req.term > self.term or self.role != FOLLOWER or self.leader != req.leader:
            self._step_down(req.term, req.leader)
        self._last_heard = time.monotonic()
        self._timeout = self._new_timeout()
        prev = req.prev_log_index
        if prev > self.last_index():
            return RAFT.AppendResponse(term=self.term, success=False, conflict_index=self.last_index() + 1)
        if prev >= self.snap_index:
            t = self.term_at(prev)
            if t != req.prev_log_term:
                # back off to the first index of the conflicting term
                k = prev
                while k > self.snap_index + 1 and self.term_at(k - 1) == t:
                    k -= 1
                return RAFT.AppendResponse(term=self.term, success=False, conflict_index=max(k, self.snap_index + 1))
        new, truncated = [], False
        for e in req.entries:
            if e.index <= self.snap_index:
                continue
            have = self.term_at(e.index)
            if have is not None and not new:
                if have == e.term:
                    continue
                del self.log[e.index - self.snap_index - 1:]            # conflict: drop it and all after
                truncated = True
            new.append(e)
        if new:
            self.log.extend(new)
        if truncated:
            self._rewrite_log()
        elif self.persisted < self.last_index():
            # the new entries, plus any a deposed leader appended but had not flushed yet: one
            # write + fdatasync before the acknowledgement
            self._append_disk(self.log[max(0, self.persisted - self.snap_index):])
        last_new = prev + len(req.entries)
        if req.leader_commit > self.commit:
            self.commit = min(req.leader_commit, max(last_new, self.commit))
            self._apply()
        return RAFT.AppendResponse(term=self.term, success=True, match_index=last_new)

    async def InstallSnapshot(self, req, ctx):
        async with self._disk:
            return self._install_snapshot(req)

    def _install_snapshot(self, req):
        if req.term < self.term:
            return RAFT.SnapshotResponse(term=self.term)
        self._step_down(req.term, req.leader)
        self._last_heard = time.monotonic()
        if req.last_index <= self.applied:
            return RAFT.SnapshotResponse(term=self.term)
        keep = [e for e in self.log if e.index > req.last_index] if self.term_at(req.last_index) == req.last_term else []
        self.sm.restore(req.data)
        self.snap_index, self.snap_term = req.last_index, req.last_term
        self.log = keep
        self.commit = max(self.commit, req.last_index)
        self.applied = req.last_index
        self._save_snapshot(req.data)
        self._rewrite_log()
        self._apply()
        return RAFT.SnapshotResponse(term=self.term)

    def status(self) -> dict:
        return {"name": self.name, "role": self.role, "term": self.term, "leader": self.leader, "commit": self.commit,
                "applied": self.applied, "last_index": self.last_index(), "persisted": self.persisted,
                "snap_index": self.snap_index}
