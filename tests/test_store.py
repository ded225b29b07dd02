"""MVCC store: CAS, watch-from-revision, compaction, WAL+snapshot recovery, and a
Hypothesis model check that the store is linearizable against a dict model."""
import json
import time

import pytest
from hypothesis import given, settings, strategies as st

from amdkube.store import CASFailed, Compacted, KeyExists, MVCCStore, Storage, Filter, DELETE
from amdkube.store.storage import FilteredWatch
from amdkube.api import labels as L
from amdkube.api import meta as m
from tests.conftest import run


def test_cas_and_revisions():
    s = MVCCStore()
    a = s.put("/a", b"1", expect_mod_rev=0)
    assert (a.create_rev, a.mod_rev, a.version) == (1, 1, 1)
    with pytest.raises(KeyExists):
        s.put("/a", b"x", expect_mod_rev=0)
    b = s.put("/a", b"2", expect_mod_rev=1)
    assert (b.create_rev, b.mod_rev, b.version) == (1, 2, 2)
    with pytest.raises(CASFailed):
        s.put("/a", b"3", expect_mod_rev=1)
    s.delete("/a")
    assert s.get("/a") is None and s.rev == 3


def test_watch_from_revision_and_compaction():
    async def go():
        s = MVCCStore(history=3)
        for i in range(5):
            s.put(f"/p/{i}", str(i).encode())
        with pytest.raises(Compacted):
            s.watch("/p/", 1)
        w = s.watch("/p/", 4)
        evs = [await w.next(1), await w.next(1)]
        assert [e.rev for e in evs] == [4, 5]
        s.put("/q/x", b"ignored")
        s.delete("/p/0")
        ev = await w.next(1)
        assert ev.type == DELETE and ev.kv.key == "/p/0"
        w.close()
    run(go())


def test_wal_snapshot_recovery(tmp_path):
    d = str(tmp_path / "data")
    s = MVCCStore(data_dir=d, snapshot_every=3)
    for i in range(7):
        s.put(f"/k/{i % 4}", json.dumps({"i": i}).encode())
    s.delete("/k/0")
    rev = s.rev
    state = {k: v.value for k, v in s.kv.items()}
    s.close()
    s2 = MVCCStore(data_dir=d)
    assert s2.rev == rev
    assert {k: v.value for k, v in s2.kv.items()} == state
    assert s2.put("/k/9", b"{}").mod_rev == rev + 1


def test_storage_guaranteed_update_and_filtered_watch():
    async def go():
        s = MVCCStore()
        st_ = Storage(s, "pods")
        st_.create("/registry/pods/default/a", {"metadata": {"name": "a", "labels": {"app": "x"}}})
        w = st_.watch("/registry/pods/", "0", Filter(L.parse_selector("app=x")))

        def relabel(cur):
            cur["metadata"]["labels"]["app"] = "y"
            return cur
        obj = st_.guaranteed_update("/registry/pods/default/a", relabel)
        assert obj["metadata"]["resourceVersion"] == str(s.rev)
        typ, o, _ = await w.next(1)
        assert typ == m.DELETED  # left the filter → DELETED (cacher semantics)
        with pytest.raises(m.StatusError) as ei:
            st_.guaranteed_update("/registry/pods/default/a", relabel, precond_rv="1")
        assert ei.value.code == 409
        w.close()
    run(go())


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["put", "cas", "del"]), st.integers(0, 4), st.integers(0, 6)), max_size=40))
def test_store_matches_model(ops):
    s, model = MVCCStore(), {}
    for op, k, r in ops:
        key = f"/k/{k}"
        try:
            if op == "put":
                s.put(key, str(r).encode())
                model[key] = (str(r).encode(), s.rev)
            elif op == "cas":
                s.put(key, b"c", expect_mod_rev=r)
                assert (r == 0 and key not in model) or (key in model and model[key][1] == r)
                model[key] = (b"c", s.rev)
            else:
                s.delete(key)
                assert key in model
                del model[key]
        except (KeyExists, CASFailed, Exception) as e:
            if op == "cas":
                assert not ((r == 0 and key not in model) or (key in model and model[key][1] == r)), e
            elif op == "del":
                assert key not in model
        assert {kk: (v.value, v.mod_rev) for kk, v in s.kv.items()} == model


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["create", "bind", "status", "del"]), st.integers(0, 5),
                          st.sampled_from(["", "n1", "n2"])), max_size=40))
def test_triggered_watch_equals_filtered_watch(ops):
    """The spec.nodeName trigger index (store.triggered) is an optimisation only: a watch it
    indexes must deliver exactly the events an unindexed watch with the same filter delivers."""
    from amdkube.apiserver.registry import pod_fields

    async def go():
        s = MVCCStore()
        st_ = Storage(s, "pods")
        flt = lambda: Filter(None, L.parse_field_selector("spec.nodeName=n1"), pod_fields)  # noqa: E731
        indexed = st_.watch("/registry/pods/", "0", flt())
        assert indexed.w.trigger is not None and indexed.w not in s.watchers
        plain = FilteredWatch(None, flt())
        plain.w = s.watch("/registry/pods/", 0, transform=plain._translate)  # no trigger
        for op, i, node in ops:
            key = f"/registry/pods/default/p{i}"
            try:
                if op == "create":
                    st_.create(key, {"metadata": {"name": f"p{i}"}, "spec": {"nodeName": node}, "status": {}})
                elif op == "bind":
                    st_.guaranteed_update(key, lambda c: {**c, "spec": {"nodeName": node}})
                elif op == "status":
                    st_.guaranteed_update(key, lambda c: {**c, "status": {"phase": node or "Pending"}})
                else:
                    st_.delete(key)
            except m.StatusError:
                pass

        def drain(w):
            out = []
            while not w.w.queue.empty():
                typ, obj, ev = w.w.queue.get_nowait()
                out.append((typ, obj["metadata"]["name"], ev.rev))
            return out
        assert drain(indexed) == drain(plain)
        indexed.close()
        plain.close()
        assert not s.triggered
    run(go())


def test_data_dir_is_locked_while_a_store_holds_it(tmp_path):
    """A second store (here: same process, its own open file) on a held data directory waits
    for the lock and then refuses; closing the first releases it."""
    from amdkube.store.mvcc import DataDirLocked
    d = str(tmp_path / "data")
    s = MVCCStore(data_dir=d)
    s.put("/k", b"1")
    t0 = time.monotonic()
    with pytest.raises(DataDirLocked, match="in use by another process"):
        MVCCStore(data_dir=d, lock_wait=0.3)
    assert time.monotonic() - t0 >= 0.25
    s.close()
    s2 = MVCCStore(data_dir=d, lock_wait=0.3)
    assert s2.get("/k").value == b"1"
    s2.close()
