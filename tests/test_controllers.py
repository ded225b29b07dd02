"""Controller-manager: ReplicaSet / Deployment / DaemonSet / Job / Namespace / GC / node
lifecycle / pod GC on an in-process cluster (hollow nodes provide extra nodes)."""
import asyncio
import time

from amdkube.api import meta as m
from amdkube.controllers.lifecycle import NodeLifecycleController
from amdkube.hollow.hollow_node import HollowNode
from amdkube.localcluster import LocalCluster
from tests.conftest import run


async def until(pred, timeout=20.0, step=0.05):
    end = time.time() + timeout
    last = None
    while time.time() < end:
        last = await pred()
        if last:
            return last
        await asyncio.sleep(step)
    raise AssertionError(f"condition not met: {last!r}")


def tpl(labels, cmd=("sleep", "60"), gpus=0):
    c = {"name": "c", "image": "busybox", "command": list(cmd)}
    if gpus:
        c["resources"] = {"limits": {"amd.com/gpu": str(gpus)}}
    return {"metadata": {"labels": labels}, "spec": {"containers": [c]}}


def test_replicaset_deployment_and_gc():
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=4, relist_period=0.2) as lc:
            c = lc.client
            await lc.wait_gpus(4)
            await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "rs", "namespace": "default"},
                            "spec": {"replicas": 3, "selector": {"matchLabels": {"app": "rs"}}, "template": tpl({"app": "rs"}, gpus=1)}})

            async def rs_ready():
                rs = await c.get("replicasets.apps", "rs", "default")
                return (rs.get("status") or {}).get("readyReplicas") == 3 and rs
            await until(rs_ready, 30)
            pods, _ = await c.list("pods", "default", label_selector="app=rs")
            ids = [d for p in pods for d in p["spec"]["extendedResources"][0]["assigned"]]
            assert len(set(ids)) == 3
            await c.patch("replicasets.apps", "rs", {"spec": {"replicas": 1}}, "default")

            async def scaled():
                pods, _ = await c.list("pods", "default", label_selector="app=rs")
                return len([p for p in pods if not p["metadata"].get("deletionTimestamp")]) == 1
            await until(scaled, 30)
            # cascading delete via the garbage collector
            await c.delete("replicasets.apps", "rs", "default")

            async def gone():
                pods, _ = await c.list("pods", "default", label_selector="app=rs")
                return not pods
            await until(gone, 30)
            # deployment: new template → new ReplicaSet, old scaled to zero
            await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d", "namespace": "default"},
                            "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "d"}}, "template": tpl({"app": "d"})}})

            async def d_ready():
                d = await c.get("deployments.apps", "d", "default")
                return (d.get("status") or {}).get("readyReplicas") == 2
            await until(d_ready, 30)
            await c.patch("deployments.apps", "d", {"spec": {"template": {"metadata": {"labels": {"app": "d", "v": "2"}}}}}, "default",
                          patch_type="application/strategic-merge-patch+json")

            async def rolled():
                rss, _ = await c.list("replicasets.apps", "default")
                mine = [r for r in rss if (m.controller_ref(r) or {}).get("name") == "d"]
                return len(mine) == 2 and sorted(int(r["spec"]["replicas"]) for r in mine) == [0, 2]
            await until(rolled, 30)
    run(go(), 150)


def test_job_and_daemonset_on_hollow_nodes():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            hollow = [await HollowNode(lc.api.url, f"hollow-{i}", gpus=8, run_seconds=0.3).start() for i in range(2)]
            try:
                await c.create({"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "j", "namespace": "default"},
                                "spec": {"completions": 4, "parallelism": 2,
                                         "template": {"spec": {"restartPolicy": "Never", "containers": [
                                             {"name": "c", "image": "busybox", "command": ["true"], "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})

                async def done():
                    j = await c.get("jobs.batch", "j", "default")
                    return any(x["type"] == "Complete" for x in (j.get("status") or {}).get("conditions") or []) and j
                j = await until(done, 40)
                assert j["status"]["succeeded"] >= 4
                await c.create({"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "ds", "namespace": "kube-system"},
                                "spec": {"selector": {"matchLabels": {"app": "ds"}}, "template": tpl({"app": "ds"})}})

                async def ds_ok():
                    pods, _ = await c.list("pods", "kube-system", label_selector="app=ds")
                    return sorted(p["spec"]["nodeName"] for p in pods) == sorted([lc.node_name, "hollow-0", "hollow-1"])
                await until(ds_ok, 30)
            finally:
                for h in hollow:
                    await h.stop()
    run(go(), 150)


def test_namespace_deletion_and_node_lifecycle():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x", "namespace": "team"}, "data": {}})
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "team"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}})
            await c.delete("namespaces", "team")

            async def ns_gone():
                return await c.get_or_none("namespaces", "team") is None
            await until(ns_gone, 40)
            # node lifecycle: a node whose heartbeat stops goes Unknown, is tainted, pods evicted
            await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "ghost"},
                            "status": {"capacity": {"cpu": "4", "memory": "4Gi", "pods": "10"},
                                       "conditions": [{"type": "Ready", "status": "True", "lastHeartbeatTime": "2000-01-01T00:00:00Z"}]}})
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "stuck", "namespace": "default"},
                            "spec": {"nodeName": "ghost", "containers": [{"name": "c", "image": "busybox"}],
                                     "tolerations": [{"key": "node.kubernetes.io/unreachable", "operator": "Exists",
                                                      "effect": "NoExecute", "tolerationSeconds": 0}]}})
            # (the kubelet's own node stays within the grace period: with every node down the
            # controller would enter master disruption mode and evict nothing)
            nlc = NodeLifecycleController(lc.controllers, grace=30.0, eviction_timeout=0.0)
            nlc.setup()
            await until(lambda: _has(lc, "ghost"), 10)
            await nlc.monitor_once()
            node = await c.get("nodes", "ghost")
            assert any(x["type"] == "Ready" and x["status"] == "Unknown" for x in node["status"]["conditions"])
            assert any(t["key"] == "node.kubernetes.io/unreachable" for t in node["spec"]["taints"])
            await asyncio.sleep(0.3)
            await nlc.monitor_once()
            p = await c.get_or_none("pods", "stuck", "default")
            assert p is None or p["metadata"].get("deletionTimestamp")
    run(go(), 120)


async def _has(lc, name):
    return any(m.name_of(n) == name for n in lc.controllers.nodes.list())


def test_node_lifecycle_zones_rate_limits_and_taint_manager():
    """node_controller_test.go (zone states, rate-limited tainting and eviction, master
    disruption) and taint_controller_test.go (tolerationSeconds)."""
    from amdkube.controllers.lifecycle import FULL, NORMAL, PARTIAL, zone_state
    assert zone_state(3, 0, 0.55) == NORMAL and zone_state(0, 2, 0.55) == FULL
    assert zone_state(2, 3, 0.55) == PARTIAL and zone_state(10, 3, 0.55) == NORMAL and zone_state(1, 2, 0.55) == NORMAL

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False) as lc:
            c = lc.client
            dead = "2000-01-01T00:00:00Z"

            async def node(name, hb, zone="z1"):
                await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": {
                    "failure-domain.beta.kubernetes.io/region": "r", "failure-domain.beta.kubernetes.io/zone": zone}},
                    "status": {"conditions": [{"type": "Ready", "status": "True", "lastHeartbeatTime": hb}]}})

            async def pod(name, node_name, tols=None):
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
                                "spec": {"nodeName": node_name, "containers": [{"name": "c", "image": "busybox"}],
                                         "tolerations": tols or []}})
                p = await c.get("pods", name, "default")
                p["status"] = {"phase": "Running", "conditions": [{"type": "Ready", "status": "True"}]}
                await c.update_status(p)
            for n in ("a1", "a2"):
                await node(n, dead)
            await node("b1", m.now_rfc3339(), "z2")
            await pod("on-a1", "a1")      # DefaultTolerationSeconds admission: tolerates unreachable for 300 s
            await pod("forever", "a1", [{"key": "node.kubernetes.io/unreachable", "operator": "Exists", "effect": "NoExecute"}])
            await until(lambda: _count(lc, 3), 10)
            await until(lambda: _pods(lc, 2), 10)
            t0 = time.time()
            # taint-based evictions: one node tainted per token (0.5/s)
            nlc = NodeLifecycleController(lc.controllers, grace=1000.0, eviction_rate=0.5)
            nlc.setup()
            await nlc.monitor_once(now=t0)
            assert nlc.zone_states == {"r:\x00:z1": FULL, "r:\x00:z2": NORMAL}
            tainted = lambda ns: [n for n in ns if any(t["key"] == "node.kubernetes.io/unreachable"  # noqa: E731
                                                       for t in (n.get("spec") or {}).get("taints") or [])]
            nodes = [await c.get("nodes", n) for n in ("a1", "a2")]
            assert len(tainted(nodes)) == 1
            p = await c.get("pods", "on-a1", "default")
            assert [x["status"] for x in p["status"]["conditions"] if x["type"] == "Ready"] == ["False"]
            await until(lambda: _tainted(lc, "a1") if tainted(nodes)[0]["metadata"]["name"] == "a1" else _tainted(lc, "a2"), 10)
            await nlc.monitor_once(now=t0 + 0.5)
            assert len(tainted([await c.get("nodes", n) for n in ("a1", "a2")])) == 1
            await nlc.monitor_once(now=t0 + 2.5)
            assert len(tainted([await c.get("nodes", n) for n in ("a1", "a2")])) == 2
            await until(lambda: _tainted(lc, "a1"), 10)
            # the taint manager: the 300 s default toleration, the forever toleration
            added = m.parse_time(next(t["timeAdded"] for t in (await c.get("nodes", "a1"))["spec"]["taints"]))
            await nlc.taint_manager.process_once(now=added + 299)
            assert not await _deleted(c, "on-a1")
            await nlc.taint_manager.process_once(now=added + 301)
            assert await _deleted(c, "on-a1") and not await _deleted(c, "forever")
            # the legacy path (TaintBasedEvictions off): delete pods after --pod-eviction-timeout, rate limited
            await pod("x1", "a1")
            await pod("x2", "a2")
            await until(lambda: _pods_named(lc, "x2"), 10)
            legacy = NodeLifecycleController(lc.controllers, grace=1000.0, eviction_timeout=5.0, eviction_rate=0.5,
                                             taint_based_evictions=False, enable_taint_manager=False)
            legacy.setup()
            await legacy.monitor_once(now=t0)
            await legacy.monitor_once(now=t0 + 6)
            assert sum([await _deleted(c, n) for n in ("x1", "x2")]) == 1
            await legacy.monitor_once(now=t0 + 8.5)
            assert all([await _deleted(c, n) for n in ("x1", "x2")])
            # every zone down: master disruption mode lifts the taints and evicts nothing
            b1 = await c.get("nodes", "b1")
            b1["status"]["conditions"][0]["lastHeartbeatTime"] = dead
            await c.update_status(b1)
            for _ in range(100):
                if get_cond(lc, "b1") == dead:
                    break
                await asyncio.sleep(0.05)
            await nlc.monitor_once(now=t0 + 20)
            assert nlc.master_disruption
            for n in ("a1", "a2", "b1"):
                assert not any(t["key"].startswith("node.kubernetes.io/") for t in (await c.get("nodes", n))["spec"].get("taints") or [])
            # a user NoExecute taint on a healthy node: untolerating pods go at once
            await node("g1", m.now_rfc3339(), "z3")
            await pod("plain", "g1")
            await pod("brief", "g1", [{"key": "maint", "operator": "Exists", "effect": "NoExecute", "tolerationSeconds": 30}])
            await c.patch("nodes", "g1", {"spec": {"taints": [{"key": "maint", "value": "x", "effect": "NoExecute",
                                                                "timeAdded": "2030-01-01T00:00:00Z"}]}})
            await until(lambda: _tainted(lc, "g1"), 10)
            await until(lambda: _pods_named(lc, "brief"), 10)
            start = m.parse_time("2030-01-01T00:00:00Z")
            await nlc.taint_manager.process_once(now=start + 1)
            assert await _deleted(c, "plain") and not await _deleted(c, "brief")
            await nlc.taint_manager.process_once(now=start + 31)
            assert await _deleted(c, "brief")
    run(go(), 120)


def get_cond(lc, name):
    for n in lc.controllers.nodes.list():
        if m.name_of(n) == name:
            return n["status"]["conditions"][0].get("lastHeartbeatTime")


async def _count(lc, k):
    return len(lc.controllers.nodes.list()) >= k


async def _pods(lc, k):
    return len([p for p in lc.controllers.pods.list() if (p.get("status") or {}).get("conditions")]) >= k


async def _pods_named(lc, name):
    return any(m.name_of(p) == name for p in lc.controllers.pods.list())


async def _tainted(lc, name):
    return any(m.name_of(n) == name and (n.get("spec") or {}).get("taints") for n in lc.controllers.nodes.list())


async def _deleted(c, name):
    p = await c.get_or_none("pods", name, "default")
    return p is None or bool(p["metadata"].get("deletionTimestamp"))


def test_daemonset_rolling_update_history_and_undo(capsys):
    """RollingUpdate (maxUnavailable 1): a new template replaces every node's pod, never more
    than one node without an available pod; every template is a ControllerRevision, and
    `kubectl rollout history/undo/status daemonset` work over them (update.go, history.go)."""
    from amdkube.kubectl.main import main as kubectl

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            hollow = [await HollowNode(lc.api.url, f"hollow-{i}", gpus=0).start() for i in range(3)]
            try:
                await c.create({"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "agent", "namespace": "default"},
                                "spec": {"selector": {"matchLabels": {"app": "agent"}}, "template": tpl({"app": "agent"}),
                                         "updateStrategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 1}}}})

                async def rolled(want_label):
                    ds = await c.get("daemonsets.apps", "agent", "default")
                    st = ds.get("status") or {}
                    pods, _ = await c.list("pods", "default", label_selector="app=agent")
                    live = [p for p in pods if not p["metadata"].get("deletionTimestamp")]
                    ok = (st.get("updatedNumberScheduled") == st.get("numberAvailable") == st.get("desiredNumberScheduled") == 4
                          and len(live) == 4 and all(m.labels_of(p).get("v") == want_label for p in live)
                          and st.get("observedGeneration") == ds["metadata"].get("generation"))
                    return ok and live
                first = await until(lambda: rolled(None), 40)
                h1 = {m.labels_of(p)["controller-revision-hash"] for p in first}
                assert len(h1) == 1
                # watch availability while the template changes
                worst = [0]

                async def sample():
                    while True:
                        ds = await c.get("daemonsets.apps", "agent", "default")
                        worst[0] = max(worst[0], int((ds.get("status") or {}).get("numberUnavailable", 0)))
                        await asyncio.sleep(0.02)
                sampler = asyncio.create_task(sample())
                await c.patch("daemonsets.apps", "agent", {"spec": {"template": {"metadata": {"labels": {"app": "agent", "v": "2"}}}}},
                              "default", patch_type="application/strategic-merge-patch+json")
                second = await until(lambda: rolled("2"), 60)
                sampler.cancel()
                assert worst[0] <= 1, worst
                assert {m.labels_of(p)["controller-revision-hash"] for p in second}.isdisjoint(h1)
                revs, _ = await c.list("controllerrevisions.apps", "default")
                assert sorted(r["revision"] for r in revs if (m.controller_ref(r) or {}).get("name") == "agent") == [1, 2]
                kc = ["--server", lc.api.url, "--token", lc.api.loopback_token, "-n", "default"]
                assert await asyncio.to_thread(kubectl, kc + ["rollout", "history", "daemonset/agent"]) == 0
                assert await asyncio.to_thread(kubectl, kc + ["rollout", "status", "daemonset/agent"]) == 0
                assert await asyncio.to_thread(kubectl, kc + ["rollout", "undo", "daemonset/agent"]) == 0
                third = await until(lambda: rolled(None), 60)
                assert {m.labels_of(p)["controller-revision-hash"] for p in third} == h1
                revs, _ = await c.list("controllerrevisions.apps", "default")
                assert sorted((r["revision"], r["metadata"]["labels"]["controller-revision-hash"] in h1) for r in revs
                              if (m.controller_ref(r) or {}).get("name") == "agent") == [(2, False), (3, True)]
            finally:
                for h in hollow:
                    await h.stop()
    run(go(), 200)
    out = capsys.readouterr().out
    assert 'daemonsets "agent"' in out and "REVISION" in out and 'daemon set "agent" successfully rolled out' in out
    assert "daemonset.apps/agent rolled back" in out


def test_statefulset_rollout_history_and_undo(capsys):
    """StatefulSet templates are ControllerRevisions numbered 1, 2, ...; `kubectl rollout undo`
    brings the previous template back as the newest revision and the pods follow it."""
    from amdkube.kubectl.main import main as kubectl

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "db", "namespace": "default"},
                            "spec": {"replicas": 2, "serviceName": "db", "selector": {"matchLabels": {"app": "db"}},
                                     "template": tpl({"app": "db"})}})

            async def at(label):
                sts = await c.get("statefulsets.apps", "db", "default")
                st = sts.get("status") or {}
                pods, _ = await c.list("pods", "default", label_selector="app=db")
                live = [p for p in pods if not p["metadata"].get("deletionTimestamp")]
                return (st.get("readyReplicas") == 2 == st.get("updatedReplicas") and len(live) == 2
                        and all(m.labels_of(p).get("v") == label for p in live) and st.get("updateRevision") == st.get("currentRevision")
                        and {m.labels_of(p)["controller-revision-hash"] for p in live})
            h1 = await until(lambda: at(None), 60)
            await c.patch("statefulsets.apps", "db", {"spec": {"template": {"metadata": {"labels": {"app": "db", "v": "2"}}}}},
                          "default", patch_type="application/strategic-merge-patch+json")
            h2 = await until(lambda: at("2"), 60)
            assert h1 != h2
            kc = ["--server", lc.api.url, "--token", lc.api.loopback_token, "-n", "default"]
            assert await asyncio.to_thread(kubectl, kc + ["rollout", "history", "statefulset/db"]) == 0
            assert await asyncio.to_thread(kubectl, kc + ["rollout", "undo", "statefulset/db"]) == 0
            assert await until(lambda: at(None), 60) == h1
            revs, _ = await c.list("controllerrevisions.apps", "default")
            mine = sorted((r["revision"], r["metadata"]["name"]) for r in revs          # pods carry the revision's name
                          if (m.controller_ref(r) or {}).get("name") == "db")
            assert [r for r, _ in mine] == [2, 3] and mine[-1][1] in h1
            assert await asyncio.to_thread(kubectl, kc + ["rollout", "status", "statefulset/db"]) == 0
    run(go(), 200)
    out = capsys.readouterr().out
    assert 'statefulsets "db"' in out and "statefulset.apps/db rolled back" in out
    # the defaulted rollingUpdate block (partition 0) takes rollout_status.go's partition branch
    assert "partitioned roll out complete: 2 new pods have been updated..." in out
