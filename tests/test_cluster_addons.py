"""The remaining cluster addons: dns-horizontal-autoscaler, ip-masq-agent, dashboard, fluentd-elasticsearch.

Reference: cluster/addons/{dns-horizontal-autoscaler,ip-masq-agent,dashboard,fluentd-elasticsearch}.
Their programs are third-party images (cluster-proportional-autoscaler, ip-masq-agent,
kubernetes-dashboard, fluentd + Elasticsearch + Kibana) whose sources and tests are not in the
reference tree, so the semantics tested here are those the addons' manifests and configmaps
configure (default params, config file fields, fluentd's source/filter/match settings). Parity with
those images' own test suites is unpinned. The manifests under deploy/addons are parsed and their
commands checked against amdkube's CLI.
"""
from __future__ import annotations

import asyncio
import datetime
import json
import os
import socket

import pytest
import yaml

from amdkube.clusteraddons import ipmasq as IM
from amdkube.clusteraddons import proportional as PA
from amdkube.clusterlogging import shipper as SH
from amdkube.clusterlogging.store import LogStore
from tests.conftest import run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _node(name, cpu="8", gpus=0, unschedulable=False):
    cap = {"cpu": cpu}
    if gpus:
        cap["amd.com/gpu"] = str(gpus)
    return {"metadata": {"name": name}, "spec": {"unschedulable": unschedulable} if unschedulable else {},
            "status": {"capacity": cap}}


# ------------------------------------------------------------------ cluster-proportional-autoscaler
def test_cluster_status_counts_schedulable_and_total():
    st = PA.cluster_status([_node("a", "4", 8), _node("b", "3500m", 8), _node("c", "64", unschedulable=True)])
    assert st == {"total_nodes": 3, "total_cores": 72, "total_gpus": 16, "schedulable_nodes": 2, "schedulable_cores": 8,
                  "schedulable_gpus": 16}


@pytest.mark.parametrize("params,nodes,cores,want", [
    ({"coresPerReplica": 256, "nodesPerReplica": 16, "preventSinglePointFailure": True}, 1, 4, 1),
    ({"coresPerReplica": 256, "nodesPerReplica": 16, "preventSinglePointFailure": True}, 2, 8, 2),
    ({"coresPerReplica": 256, "nodesPerReplica": 16, "preventSinglePointFailure": True}, 40, 160, 3),
    ({"coresPerReplica": 256, "nodesPerReplica": 16}, 10, 1024, 4),
    ({"coresPerReplica": 2, "nodesPerReplica": 1, "min": 1, "max": 5}, 3, 20, 5),
    ({"nodesPerReplica": 4, "min": 3}, 2, 2, 3),
    ({"coresPerReplica": 10}, 0, 0, 1),
], ids=["addon default, one node", "addon default, spof guard", "addon default, 40 nodes", "cores dominate",
        "max clamps", "min floors", "zero nodes: the zero ratio gives one"])
def test_linear_params(params, nodes, cores, want):
    st = {"schedulable_nodes": nodes, "schedulable_cores": cores, "schedulable_gpus": 0,
          "total_nodes": nodes, "total_cores": cores, "total_gpus": 0}
    assert PA.Linear(params).replicas(st) == want


def test_linear_gpus_and_unschedulable_nodes():
    st = PA.cluster_status([_node(f"n{i}", "16", 8) for i in range(4)] + [_node("x", "16", 8, unschedulable=True)])
    assert PA.Linear({"nodesPerReplica": 16, "gpusPerReplica": 8}).replicas(st) == 4
    assert PA.Linear({"nodesPerReplica": 1}).replicas(st) == 4
    assert PA.Linear({"nodesPerReplica": 1, "includeUnschedulableNodes": True}).replicas(st) == 5


@pytest.mark.parametrize("params,nodes,cores,want", [
    ({"coresToReplicas": [[1, 1], [64, 3], [512, 5], [1024, 7]], "nodesToReplicas": [[1, 1], [2, 2]]}, 1, 4, 1),
    ({"coresToReplicas": [[1, 1], [64, 3], [512, 5], [1024, 7]], "nodesToReplicas": [[1, 1], [2, 2]]}, 2, 4, 2),
    ({"coresToReplicas": [[1, 1], [64, 3], [512, 5], [1024, 7]], "nodesToReplicas": [[1, 1], [2, 2]]}, 10, 600, 5),
    ({"coresToReplicas": [[1, 1], [64, 3], [512, 5], [1024, 7]], "nodesToReplicas": [[1, 1], [2, 2]]}, 10, 5000, 7),
    ({"nodesToReplicas": [[5, 3]]}, 2, 0, 1),
])
def test_ladder_params(params, nodes, cores, want):
    st = {"schedulable_nodes": nodes, "schedulable_cores": cores, "schedulable_gpus": 0,
          "total_nodes": nodes, "total_cores": cores, "total_gpus": 0}
    assert PA.Ladder(params).replicas(st) == want


@pytest.mark.parametrize("data", [{}, {"linear": "{}", "ladder": "{}"}, {"linear": "not json"}, {"linear": "[]"},
                                  {"linear": json.dumps({"coresPerReplica": -1})}, {"linear": json.dumps({})},
                                  {"ladder": json.dumps({"coresToReplicas": [[1]]})}, {"ladder": json.dumps({})},
                                  {"linear": json.dumps({"nodesPerReplica": 1, "min": 5, "max": 2})}])
def test_params_rejected(data):
    with pytest.raises(PA.ParamsError):
        PA.parse_params(data)


def test_target_parsing():
    assert PA.parse_target("Deployment/kube-dns") == ("deployments", "kube-dns")
    assert PA.parse_target("replicationcontroller/x") == ("replicationcontrollers", "x")
    for bad in ("Deployment", "DaemonSet/x", "/x"):
        with pytest.raises(ValueError):
            PA.parse_target(bad)


def test_autoscaler_against_an_apiserver_creates_its_configmap_and_scales():
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "kube-dns", "namespace": "kube-system"},
                            "spec": {"replicas": 1, "selector": {"matchLabels": {"k8s-app": "kube-dns"}},
                                     "template": {"metadata": {"labels": {"k8s-app": "kube-dns"}},
                                                  "spec": {"containers": [{"name": "dns", "image": "busybox"}]}}}}, "kube-system")
            pa = PA.ProportionalAutoscaler(c, "kube-system", "kube-dns-autoscaler", "Deployment/kube-dns",
                                           json.dumps({"ladder": {"nodesToReplicas": [[1, 3]]}}), poll_period=0.05)
            assert await pa.poll_once() == 3
            cm = await c.get("configmaps", "kube-dns-autoscaler", "kube-system")
            assert json.loads(cm["data"]["ladder"]) == {"nodesToReplicas": [[1, 3]]}
            assert (await c.get("deployments", "kube-dns", "kube-system"))["spec"]["replicas"] == 3
            assert await pa.poll_once() is None                               # already there
            # the user retunes the ConfigMap; a broken edit keeps the last good params
            cm["data"] = {"linear": json.dumps({"nodesPerReplica": 1, "min": 2})}
            cm = await c.update(cm)
            assert await pa.poll_once() == 2
            cm["data"] = {"linear": "{broken"}
            await c.update(cm)
            assert await pa.poll_once() is None
            assert (await c.get("deployments", "kube-dns", "kube-system"))["spec"]["replicas"] == 2
    run(go(), 60)


# ------------------------------------------------------------------ ip-masq-agent
GOLDEN_DEFAULT = """*nat
:IP-MASQ-AGENT - [0:0]
-A IP-MASQ-AGENT -d 169.254.0.0/16 -m comment --comment "ip-masq-agent: local traffic is not subject to MASQUERADE" -j RETURN
-A IP-MASQ-AGENT -d 10.0.0.0/8 -m comment --comment "ip-masq-agent: local traffic is not subject to MASQUERADE" -j RETURN
-A IP-MASQ-AGENT -d 172.16.0.0/12 -m comment --comment "ip-masq-agent: local traffic is not subject to MASQUERADE" -j RETURN
-A IP-MASQ-AGENT -d 192.168.0.0/16 -m comment --comment "ip-masq-agent: local traffic is not subject to MASQUERADE" -j RETURN
-A IP-MASQ-AGENT -m comment --comment "ip-masq-agent: outbound traffic is subject to MASQUERADE (must be last in chain)" -j MASQUERADE
COMMIT
"""


def test_ip_masq_agent_default_rules():
    assert IM.render(IM.parse_config("")) == GOLDEN_DEFAULT


def test_ip_masq_agent_config_file(tmp_path):
    path = tmp_path / "ip-masq-agent"
    agent = IM.MasqAgent(str(path), dry_run=True)
    assert agent.sync() == GOLDEN_DEFAULT and agent.postrouting_ensured         # no file: the defaults
    path.write_text("nonMasqueradeCIDRs:\n  - 10.200.0.0/16\nmasqLinkLocal: true\nresyncInterval: 1m30s\n")
    rules = agent.sync()
    assert "169.254.0.0/16" not in rules and "-d 10.200.0.0/16" in rules and "192.168.0.0/16" not in rules
    assert agent.config["resyncInterval"] == 90.0
    assert rules.splitlines()[-2].endswith("-j MASQUERADE")                       # MASQUERADE stays last
    path.write_text(json.dumps({"nonMasqueradeCIDRs": ["10.0.0.300/8"]}))
    assert agent.sync() == rules                                                  # a bad file keeps the last config
    path.write_text("nonMasqueradeCIDRs: []\n")
    assert agent.sync().count("RETURN") == 1                                      # only link-local stays unmasqueraded
    path.unlink()
    assert agent.sync() == GOLDEN_DEFAULT


@pytest.mark.parametrize("text,err", [("bogus: 1", "unknown config fields"), ("nonMasqueradeCIDRs: 10.0.0.0/8", "must be a list"),
                                      ("nonMasqueradeCIDRs: [10.0.0.1]", "invalid CIDR"), ("masqLinkLocal: yes please", "boolean"),
                                      ("resyncInterval: soon", "invalid duration"), ("[1, 2]", "mapping")])
def test_ip_masq_agent_rejects_bad_configs(text, err):
    with pytest.raises(IM.ConfigError, match=err):
        IM.parse_config(text)


# ------------------------------------------------------------------ log store
def test_log_store_bulk_search_and_persistence(tmp_path):
    st = LogStore(str(tmp_path / "data"), retention_days=7)
    body = "\n".join([
        json.dumps({"index": {"_index": "logstash-2026.10.15", "_type": "fluentd"}}),
        json.dumps({"log": "GPU 0 ready\n", "@timestamp": "2026-10-15T10:00:00Z", "kubernetes": {"pod_name": "a", "namespace_name": "ml"}}),
        json.dumps({"create": {"_index": "logstash-2026.10.17"}}),
        json.dumps({"log": "training step 10 loss 0.5\n", "@timestamp": "2026-10-17T10:00:00Z",
                    "kubernetes": {"pod_name": "b", "namespace_name": "ml"}}),
        json.dumps({"index": {"_index": "Bad Index"}}),
        json.dumps({"log": "x"}),
    ]) + "\n"
    res = st.bulk(body)
    assert res["errors"] is True and [list(i.values())[0]["status"] for i in res["items"]] == [201, 201, 400]
    hits = st.search("logstash-*", {"term": {"kubernetes.pod_name": "b"}})["hits"]
    assert hits["total"] == 1 and hits["hits"][0]["_source"]["log"].startswith("training")
    assert st.search("logstash-*", q="kubernetes.namespace_name:ml loss")["hits"]["total"] == 1
    assert st.search("logstash-*", {"bool": {"must_not": [{"match": {"log": "gpu"}}]}})["hits"]["total"] == 1
    rng = {"range": {"@timestamp": {"gte": "2026-10-16T00:00:00Z"}}}
    assert st.search("logstash-2026.10.1*", rng)["hits"]["total"] == 1
    order = st.search("_all", sort=[{"@timestamp": "desc"}])["hits"]["hits"]
    assert [h["_source"]["kubernetes"]["pod_name"] for h in order] == ["b", "a"]
    again = LogStore(str(tmp_path / "data"))                                      # read back from disk
    assert again.search("logstash-*")["hits"]["total"] == 2
    assert st.enforce_retention(datetime.date(2026, 10, 23)) == ["logstash-2026.10.15"]
    assert sorted(st.indices) == ["logstash-2026.10.17"]
    assert st.bulk('{"update": {}}\n{}\n')["status"] == 400


# ------------------------------------------------------------------ log shipper
def test_container_line_formats():
    rec, partial = SH.parse_container_line('{"log":"hello\\n","stream":"stderr","time":"2026-10-17T01:02:03.5Z"}')
    assert rec == {"log": "hello\n", "stream": "stderr", "time": "2026-10-17T01:02:03.5Z"} and not partial
    rec, partial = SH.parse_container_line("2026-10-17T01:02:03.000000001Z stdout P part one ")
    assert partial and rec["log"] == "part one " and rec["stream"] == "stdout"
    rec, partial = SH.parse_container_line("plain output")
    assert rec["log"] == "plain output\n" and not partial
    g = SH.parse_glog("I1017 01:02:03.456789    1234 kubelet.go:100] Started kubelet\n  continued", year=2026)
    assert g == {"severity": "I", "pid": "1234", "source": "kubelet.go:100", "message": "Started kubelet\n  continued",
                 "time": "2026-10-17T01:02:03.456789Z"}
    assert SH.index_for("2026-10-17T01:02:03Z") == "logstash-2026.10.17"


class _FailingSession:
    def post(self, *a, **k):
        raise OSError("connection refused")


def test_shipper_tails_buffers_and_resumes(tmp_path):
    from aiohttp import web
    from amdkube.clusterlogging.store import app

    logs = tmp_path / "containers"
    logs.mkdir()
    target = tmp_path / "c0.log"
    cid = "ab" * 16
    link = logs / f"web-1_default_app-{cid}.log"
    link.symlink_to(target)
    target.write_text('{"log":"line 1\\n","stream":"stdout","time":"2026-10-17T00:00:01Z"}\n'
                      "2026-10-17T00:00:02Z stdout P multi \n2026-10-17T00:00:02Z stdout F part\n")
    comp = tmp_path / "kubelet.log"
    comp.write_text("I1017 00:00:03.000000    99 server.go:1] first\n  more\nE1017 00:00:04.000000    99 x.go:2] second\n")

    async def go():
        store = LogStore(str(tmp_path / "es"))
        runner = web.AppRunner(app(store))
        await runner.setup()
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        await web.TCPSite(runner, "127.0.0.1", port).start()
        try:
            pos = str(tmp_path / "pos.json")
            sh = SH.Shipper(f"http://127.0.0.1:{port}", str(logs / "*.log"), [f"{comp}:kubelet"], pos, node_name="node-1")
            assert await sh.collect() == 4
            assert not await sh.flush(_FailingSession()) and len(sh.queue) == 2       # store down: chunks stay queued
            assert not os.path.exists(pos)
            import aiohttp
            async with aiohttp.ClientSession() as session:
                assert await sh.flush(session) and not sh.queue
                docs = store.search("logstash-*", size=100, sort=[{"@timestamp": "asc"}])["hits"]["hits"]
                got = [h["_source"] for h in docs]
                assert [d.get("log") or d.get("message") for d in got] == ["line 1\n", "multi part\n", "first\n  more", "second"]
                k = got[0]["kubernetes"]
                assert k == {"pod_name": "web-1", "namespace_name": "default", "container_name": "app", "host": "node-1"}
                assert got[0]["docker"] == {"container_id": cid} and got[0]["tag"].startswith("kubernetes.")
                assert got[3]["severity"] == "E" and got[3]["tag"] == "kubelet"
                # a restarted shipper resumes from the saved positions; appended lines only
                with open(target, "a") as f:
                    f.write("late line\n")
                sh2 = SH.Shipper(f"http://127.0.0.1:{port}", str(logs / "*.log"), [f"{comp}:kubelet"], pos, node_name="node-1")
                assert await sh2.collect() == 1 and await sh2.flush(session)
                assert store.search("logstash-*", q="late")["hits"]["total"] == 1
                # rotation (a new inode) starts the file over
                os.unlink(target)
                target.write_text("after rotation\n")
                assert await sh2.collect() == 1
        finally:
            await runner.cleanup()
    run(go(), 60)


def test_logging_pipeline_from_a_kubelet_pod_to_the_dashboard(tmp_path):
    """A pod's output reaches the log store through the kubelet's legacy symlink and the
    shipper (with the pod's labels and uid from the API), and the dashboard's Logs view finds it."""
    import aiohttp
    from aiohttp import web
    from amdkube.clusteraddons.dashboard import Dashboard
    from amdkube.clusterlogging.store import app
    from amdkube.localcluster import LocalCluster

    async def serve(application):
        runner = web.AppRunner(application)
        await runner.setup()
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        await web.TCPSite(runner, "127.0.0.1", port).start()
        return runner, f"http://127.0.0.1:{port}"

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "talker", "labels": {"app": "talk"}},
                            "spec": {"containers": [{"name": "main", "image": "busybox",
                                                     "command": ["sh", "-c", "echo hello-from-mi355x; sleep 60"]}]}}, "default")
            from amdkube.localcluster import wait_pod
            pod = await wait_pod(c, "default", "talker", ("Running",), 30)
            legacy = lc.kubelet.runtime.legacy_logs_dir
            [link] = [f for f in os.listdir(legacy) if f.startswith("talker_default_main-")]
            assert os.path.islink(os.path.join(legacy, link))
            store_runner, es_url = await serve(app(LogStore(str(tmp_path / "es"))))
            dash = Dashboard(c, es_url)
            dash_runner, dash_url = await serve(dash.app())
            try:
                sh = SH.Shipper(es_url, os.path.join(legacy, "*.log"), (), str(tmp_path / "pos"), client=c, node_name="n")
                async with aiohttp.ClientSession() as s:
                    for _ in range(100):
                        if await sh.collect():
                            break
                        await asyncio.sleep(0.05)
                    assert await sh.flush(s)
                    async with s.get(f"{dash_url}/api/logs", params={"namespace": "default", "pod": "talker"}) as r:
                        hits = await r.json()
                    assert [h["log"] for h in hits] == ["hello-from-mi355x\n"]
                    k = hits[0]["kubernetes"]
                    assert k["labels"] == {"app": "talk"} and k["pod_id"] == pod["metadata"]["uid"]
                    # the dashboard's own API over the same cluster
                    async with s.get(f"{dash_url}/api/overview", params={"namespace": "default"}) as r:
                        ov = await r.json()
                    assert [p["name"] for p in ov["pods"]] == ["talker"] and ov["pods"][0]["phase"] == "Running"
                    assert ov["nodes"] and ov["nodes"][0]["ready"] is True
                    async with s.get(f"{dash_url}/api/pods/default/talker/log") as r:
                        assert "hello-from-mi355x" in await r.text()
                    async with s.get(f"{dash_url}/") as r:
                        assert "amdkube" in await r.text()
                    async with s.delete(f"{dash_url}/api/pods/default/talker") as r:
                        assert r.status == 200
            finally:
                await dash_runner.cleanup()
                await store_runner.cleanup()
    run(go(), 90)


def test_dashboard_scale_and_overview_summaries():
    from amdkube.clusteraddons.dashboard import Dashboard, summarize_node, summarize_pod
    from amdkube.localcluster import LocalCluster

    gpu_pod = {"metadata": {"name": "p", "namespace": "d"},
               "spec": {"nodeName": "n", "containers": [{"name": "c", "resources": {"limits": {"amd.com/gpu": "2"}}}]},
               "status": {"phase": "Running", "containerStatuses": [{"ready": True, "restartCount": 3}]}}
    assert summarize_pod(gpu_pod)["gpus"] == 2 and summarize_pod(gpu_pod)["ready"] == "1/1"
    node = {"metadata": {"name": "n", "labels": {"amd.com/gpu-type": "MI355X"}},
            "status": {"capacity": {"amd.com/gpu": "8", "cpu": "128"}, "allocatable": {"amd.com/gpu": "7"},
                       "conditions": [{"type": "Ready", "status": "True"}]}}
    assert summarize_node(node, [gpu_pod])["gpus"] == {"capacity": 8, "allocatable": 7, "allocated": 2, "unhealthy": 1,
                                                       "type": "MI355X"}

    async def go():
        async with LocalCluster(gpus="none", with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
                            "spec": {"replicas": 1, "selector": {"matchLabels": {"a": "b"}},
                                     "template": {"metadata": {"labels": {"a": "b"}},
                                                  "spec": {"containers": [{"name": "c", "image": "busybox"}]}}}}, "default")
            d = Dashboard(c)
            await d.scale("Deployment", "default", "web", 4)
            assert (await c.get("deployments", "web", "default"))["spec"]["replicas"] == 4
            ov = await d.overview("default")
            assert {"kind": "deployments", "name": "web", "namespace": "default", "desired": 4, "ready": 0} == \
                {k: v for k, v in ov["workloads"][0].items() if k != "age"}
            from aiohttp import web
            with pytest.raises(web.HTTPBadRequest):
                await d.scale("DaemonSet", "default", "web", 1)
    run(go(), 60)


# ------------------------------------------------------------------ manifests
@pytest.mark.parametrize("fname,command", [("dns-horizontal-autoscaler.yaml", "cluster-proportional-autoscaler"),
                                           ("ip-masq-agent.yaml", "ip-masq-agent"), ("dashboard.yaml", "dashboard"),
                                           ("fluentd-elasticsearch.yaml", "log-store"),
                                           ("fluentd-elasticsearch.yaml", "log-shipper")])
def test_addon_manifests_run_amdkube_commands_with_valid_flags(fname, command):
    from amdkube.cmd.components import COMPONENTS
    from amdkube.cmd.gendocs import capture_parser
    docs = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, "deploy", "addons", fname))) if d]
    assert all((d.get("metadata") or {}).get("labels", {}).get("addonmanager.kubernetes.io/mode") for d in docs)
    cmds = [c["command"] for d in docs if d["kind"] in ("Deployment", "DaemonSet", "StatefulSet")
            for c in d["spec"]["template"]["spec"]["containers"]]
    [argv] = [x for x in cmds if x[:4] == ["python", "-m", "amdkube", command]]
    parser = capture_parser(COMPONENTS[command])
    parser.parse_args(argv[4:])              # every flag the manifest passes exists
