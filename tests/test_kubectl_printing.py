"""kubectl output held to the reference's printer tests, transcribed:

* pkg/printers/customcolumn_test.go — TestNewColumnPrinterFromSpec (:55), TestNewColumnPrinter
  FromTemplate (:152, incl. the tab-indented template), TestColumnPrint (:225, exact output through
  text/tabwriter); TestMassageJSONPath lives in test_jsonpath_parity.py;
* pkg/kubectl/sorting_printer_test.go TestSortingPrinter (:39, every case incl. timestamps,
  numbers, missing fields and the not-found errors);
* the per-kind columns of pkg/printers/internalversion/printers.go (AddHandlers) for the kinds
  the verdict named, `-L` / `--show-labels`, and the describers for Deployment, ReplicaSet,
  DaemonSet, StatefulSet, Job, Service, PVC, PV and Namespace (with quotas and limits);
* end to end through kubectl against an apiserver: the verdict's jsonpath probe listing each
  pod's GPUs, custom-columns, go-template, --sort-by.
"""
import asyncio
import io
import threading
from contextlib import redirect_stdout

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import APIServer
from amdkube.client import Client
from amdkube.kubectl import describe as D
from amdkube.kubectl import printers as P
from amdkube.kubectl.main import main as kubectl


# ---------------------------------------------------------------------------- custom columns
@pytest.mark.parametrize("spec,ok", [("", False), ("invalid", False), ("invalid=foobar", False),
                                     ("invalid,foobar:blah", False), ("NAME:metadata.name,API_VERSION:apiVersion", True)])
def test_new_column_printer_from_spec(spec, ok):
    if not ok:
        with pytest.raises(ValueError):
            P.CustomColumnsPrinter.from_spec(spec)
        return
    assert P.CustomColumnsPrinter.from_spec(spec).columns == [("NAME", "{.metadata.name}"), ("API_VERSION", "{.apiVersion}")]


def test_column_printer_no_headers():
    out = P.CustomColumnsPrinter.from_spec("API_VERSION:apiVersion", no_headers=True).print([{"apiVersion": "v1"}])
    assert "API_VERSION" not in out.split()


@pytest.mark.parametrize("text,ok", [
    ("", False), ("invalid", False), ("invalid=foobar", False), ("invalid,foobar:blah", False),
    ("NAME               API_VERSION\n{metadata.name}    {apiVersion}", True),
    ("NAME               \t\tAPI_VERSION\n\t\t\t\t\t\t\t{metadata.name}    {apiVersion}", True)])
def test_new_column_printer_from_template(text, ok):
    if not ok:
        with pytest.raises(ValueError):
            P.CustomColumnsPrinter.from_template(text)
        return
    assert P.CustomColumnsPrinter.from_template(text).columns == [("NAME", "{.metadata.name}"), ("API_VERSION", "{.apiVersion}")]


POD_FOO = {"metadata": {"name": "foo"}}
COLUMN_PRINT = [
    ([("NAME", "{.metadata.name}")], [POD_FOO], "NAME\nfoo\n"),
    ([("NAME", "{.metadata.name}")], [POD_FOO, {"metadata": {"name": "bar"}}], "NAME\nfoo\nbar\n"),
    ([("NAME", "{.metadata.name}"), ("API_VERSION", "{.apiVersion}")], [{**POD_FOO, "apiVersion": "baz"}],
     "NAME      API_VERSION\nfoo       baz\n"),
    ([("NAME", "{.metadata.name}"), ("API_VERSION", "{.apiVersion}"), ("NOT_FOUND", "{.notFound}")],
     [{**POD_FOO, "apiVersion": "baz"}], "NAME      API_VERSION   NOT_FOUND\nfoo       baz           <none>\n"),
]


@pytest.mark.parametrize("columns,objs,expected", COLUMN_PRINT)
def test_column_print(columns, objs, expected):
    assert P.CustomColumnsPrinter(columns).print(objs) == expected


# ---------------------------------------------------------------------------- sorting
def _pods(*names):
    return [{"metadata": {"name": n}} for n in names]


def _names(objs):
    return [o["metadata"].get("name") for o in objs]


def _ts(secs):
    import time as _t
    return _t.strftime("%Y-%m-%dT%H:%M:%SZ", _t.gmtime(secs))


def test_sorting_printer_cases():
    assert _names(P.sort_objects(_pods("a", "b", "c"), "{.metadata.name}")) == ["a", "b", "c"]
    assert _names(P.sort_objects(_pods("b", "c", "a"), "{.metadata.name}")) == ["a", "b", "c"]
    ts = [{"metadata": {"creationTimestamp": _ts(t)}} for t in (300, 100, 200)]
    assert [o["metadata"]["creationTimestamp"] for o in P.sort_objects(ts, "{.metadata.creationTimestamp}")] == \
        [_ts(100), _ts(200), _ts(300)]
    rcs = [{"spec": {"replicas": r}} for r in (5, 1, 9)]
    assert [o["spec"]["replicas"] for o in P.sort_objects(rcs, "{.spec.replicas}")] == [1, 5, 9]
    assert _names(P.sort_objects(_pods("c", "b", "a"), "{.metadata.name}")) == ["a", "b", "c"]   # v1.List in reverse
    some = [{"status": {"availableReplicas": 2}}, {"status": {}}, {"status": {"availableReplicas": 1}}]
    assert P.sort_objects(some, "{.status.availableReplicas}") == [{"status": {}}, {"status": {"availableReplicas": 1}},
                                                                    {"status": {"availableReplicas": 2}}]
    with pytest.raises(ValueError, match=r'couldn\'t find any field with path "\{.status.availableReplicas\}" in the list'):
        P.sort_objects([{"status": {"replicas": 0}}] * 2, "{.status.availableReplicas}")
    with pytest.raises(ValueError, match=r'couldn\'t find any field with path "\{.invalid\}"'):
        P.sort_objects([{"status": {}}] * 3, "{.invalid}")


def test_natural_string_order():
    assert _names(P.sort_objects(_pods("pod-10", "pod-9", "pod-1"), "metadata.name")) == ["pod-1", "pod-9", "pod-10"]


# ---------------------------------------------------------------------------- tables
NOW = "2030-01-01T00:00:00Z"


def test_tabwriter_alignment_matches_go():
    assert P.table([["NAME", "A"], ["x", "yy"]]) == "NAME      A\nx         yy"
    assert P.table([["NAMESPACELONGER", "B", "C"], ["a", "bbbbbbbbbbbb", "c"]]) == \
        "NAMESPACELONGER   B              C\na                 bbbbbbbbbbbb   c"


@pytest.mark.parametrize("kind,obj,header,cells", [
    ("Service", {"metadata": {"name": "web"}, "spec": {"type": "NodePort", "clusterIP": "10.0.0.5",
                                                        "ports": [{"port": 80, "nodePort": 30080, "protocol": "TCP"}]}},
     ["NAME", "TYPE", "CLUSTER-IP", "EXTERNAL-IP", "PORT(S)", "AGE"], ["web", "NodePort", "10.0.0.5", "<none>", "80:30080/TCP"]),
    ("Service", {"metadata": {"name": "lb"}, "spec": {"type": "LoadBalancer", "clusterIP": "10.0.0.6", "ports": []},
                 "status": {"loadBalancer": {}}}, None, ["lb", "LoadBalancer", "10.0.0.6", "<pending>", "<none>"]),
    ("StatefulSet", {"metadata": {"name": "db"}, "spec": {"replicas": 3}, "status": {"replicas": 2}},
     ["NAME", "DESIRED", "CURRENT", "AGE"], ["db", "3", "2"]),
    ("PersistentVolumeClaim", {"metadata": {"name": "c"}, "spec": {"volumeName": "pv1", "storageClassName": "fast"},
                               "status": {"phase": "Bound", "capacity": {"storage": "1Gi"},
                                          "accessModes": ["ReadWriteOnce", "ReadOnlyMany"]}},
     ["NAME", "STATUS", "VOLUME", "CAPACITY", "ACCESS MODES", "STORAGECLASS", "AGE"],
     ["c", "Bound", "pv1", "1Gi", "RWO,ROX", "fast"]),
    ("PersistentVolume", {"metadata": {"name": "pv1"}, "spec": {"capacity": {"storage": "5Gi"}, "accessModes": ["ReadWriteMany"],
                                                                "persistentVolumeReclaimPolicy": "Retain",
                                                                "claimRef": {"namespace": "ns", "name": "c"}},
                          "status": {"phase": "Bound"}},
     ["NAME", "CAPACITY", "ACCESS MODES", "RECLAIM POLICY", "STATUS", "CLAIM", "STORAGECLASS", "REASON", "AGE"],
     ["pv1", "5Gi", "RWX", "Retain", "Bound", "ns/c"]),
    ("CronJob", {"metadata": {"name": "cj"}, "spec": {"schedule": "*/5 * * * *", "suspend": False}, "status": {}},
     ["NAME", "SCHEDULE", "SUSPEND", "ACTIVE", "LAST SCHEDULE", "AGE"], ["cj", "*/5 * * * *", "false", "0", "<none>"]),
    ("HorizontalPodAutoscaler", {"metadata": {"name": "h"}, "spec": {"scaleTargetRef": {"kind": "Deployment", "name": "d"},
                                                                     "minReplicas": 1, "maxReplicas": 5,
                                                                     "targetCPUUtilizationPercentage": 80},
                                 "status": {"currentReplicas": 2, "currentCPUUtilizationPercentage": 40}},
     ["NAME", "REFERENCE", "TARGETS", "MINPODS", "MAXPODS", "REPLICAS", "AGE"], ["h", "Deployment/d", "40% / 80%", "1", "5", "2"]),
    ("PodDisruptionBudget", {"metadata": {"name": "b"}, "spec": {"minAvailable": 2}, "status": {"disruptionsAllowed": 1}},
     ["NAME", "MIN AVAILABLE", "MAX UNAVAILABLE", "ALLOWED DISRUPTIONS", "AGE"], ["b", "2", "N/A", "1"]),
    ("Endpoints", {"metadata": {"name": "e"}, "subsets": [{"addresses": [{"ip": f"10.0.0.{i}"} for i in range(5)],
                                                            "ports": [{"port": 80}]}]},
     ["NAME", "ENDPOINTS", "AGE"], ["e", "10.0.0.0:80,10.0.0.1:80,10.0.0.2:80 + 2 more..."]),
    ("ConfigMap", {"metadata": {"name": "cm"}, "data": {"a": "1", "b": "2"}}, ["NAME", "DATA", "AGE"], ["cm", "2"]),
    ("Secret", {"metadata": {"name": "s"}, "type": "Opaque", "data": {"a": "MQ=="}}, ["NAME", "TYPE", "DATA", "AGE"],
     ["s", "Opaque", "1"]),
    ("ServiceAccount", {"metadata": {"name": "sa"}, "secrets": [{"name": "t"}]}, ["NAME", "SECRETS", "AGE"], ["sa", "1"]),
    ("StorageClass", {"metadata": {"name": "fast", "annotations": {"storageclass.kubernetes.io/is-default-class": "true"}},
                      "provisioner": "kubernetes.io/host-path"}, ["NAME", "PROVISIONER", "AGE"],
     ["fast (default)", "kubernetes.io/host-path"]),
    ("Ingress", {"metadata": {"name": "i"}, "spec": {"rules": [{"host": "a.example"}], "tls": [{"hosts": ["a.example"]}]},
                 "status": {"loadBalancer": {"ingress": [{"ip": "1.2.3.4"}]}}},
     ["NAME", "HOSTS", "ADDRESS", "PORTS", "AGE"], ["i", "a.example", "1.2.3.4", "80, 443"]),
    ("Deployment", {"metadata": {"name": "d"}, "spec": {"replicas": 3}, "status": {"replicas": 3, "updatedReplicas": 2,
                                                                                  "availableReplicas": 1}},
     ["NAME", "DESIRED", "CURRENT", "UP-TO-DATE", "AVAILABLE", "AGE"], ["d", "3", "3", "2", "1"]),
    ("Job", {"metadata": {"name": "j"}, "spec": {"completions": 4}, "status": {"succeeded": 1}},
     ["NAME", "DESIRED", "SUCCESSFUL", "AGE"], ["j", "4", "1"]),
])
def test_kind_columns(kind, obj, header, cells):
    obj = {**obj, "metadata": {**obj["metadata"], "creationTimestamp": NOW}}
    if header is not None:
        assert P.columns_for(kind, False) == header
    assert P.rows_for(obj, kind, False)[:len(cells)] == cells


def test_pod_status_reasons():
    assert P.pod_status_reason({"spec": {"initContainers": [{}, {}]}, "status": {"phase": "Pending",
                               "initContainerStatuses": [{"state": {"terminated": {"exitCode": 0}}},
                                                         {"state": {"running": {}}}]}})[0] == "Init:1/2"
    assert P.pod_status_reason({"spec": {}, "status": {"phase": "Running", "containerStatuses": [
        {"state": {"waiting": {"reason": "CrashLoopBackOff"}}, "restartCount": 3}]}}) == ("CrashLoopBackOff", 0, 3)
    assert P.pod_status_reason({"metadata": {"deletionTimestamp": NOW}, "spec": {}, "status": {"phase": "Running"}})[0] == \
        "Terminating"


def test_label_columns_and_show_labels():
    objs = [{"metadata": {"name": "a", "labels": {"app": "web", "tier": "fe"}}, "data": {}}]
    out = P.print_table(objs, "ConfigMap", label_columns=["app", "example.com/tier"], show_labels=True)
    head, row = out.splitlines()
    assert head.split() == ["NAME", "DATA", "AGE", "APP", "TIER", "LABELS"]
    assert row.split()[-2:] == ["web", "app=web,tier=fe"]
    out = P.print_table(objs, "ConfigMap", with_namespace=True, no_headers=True)
    assert len(out.splitlines()) == 1


# ---------------------------------------------------------------------------- describers
def _tpl():
    return {"metadata": {"labels": {"app": "a"}}, "spec": {"containers": [
        {"name": "c", "image": "img:1", "ports": [{"containerPort": 80}], "resources": {"limits": {"amd.com/gpu": "1"}},
         "env": [{"name": "X", "value": "1"}]}]}}


def test_describe_deployment_and_replicasets():
    d = {"kind": "Deployment", "metadata": {"name": "web", "namespace": "default", "uid": "d1", "labels": {"app": "a"}},
         "spec": {"replicas": 3, "selector": {"matchLabels": {"app": "a"}}, "template": _tpl(),
                  "strategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": "25%", "maxSurge": "25%"}}},
         "status": {"replicas": 3, "updatedReplicas": 3, "availableReplicas": 2, "unavailableReplicas": 1,
                    "conditions": [{"type": "Available", "status": "True", "reason": "MinimumReplicasAvailable"}]}}
    rs = {"metadata": {"name": "web-abc", "uid": "r1", "ownerReferences": [{"uid": "d1", "controller": True}]},
          "spec": {"replicas": 3, "template": _tpl()}, "status": {"replicas": 3}}
    out = D.describe(d, [], replicasets=[rs])
    for s in ("Replicas:", "3 desired | 3 updated | 3 total | 2 available | 1 unavailable", "StrategyType:",
              "RollingUpdateStrategy:", "25% max unavailable, 25% max surge", "Pod Template:", "Image:", "img:1",
              "amd.com/gpu:", "Available", "MinimumReplicasAvailable", "NewReplicaSet:", "web-abc (3/3 replicas created)",
              "OldReplicaSets:", "Events:"):
        assert s in out, (s, out)
    pods = [{"status": {"phase": "Running"}}, {"status": {"phase": "Pending"}}]
    out = D.describe({**rs, "kind": "ReplicaSet", "metadata": {**rs["metadata"], "namespace": "default"}}, [], pods=pods)
    assert "Replicas:" in out and "3 current / 3 desired" in out and "1 Running / 1 Waiting / 0 Succeeded / 0 Failed" in out
    assert "Controlled By:" not in out or "Deployment" not in out


def test_describe_workloads_service_storage_namespace():
    ds = {"kind": "DaemonSet", "metadata": {"name": "ds", "namespace": "kube-system"},
          "spec": {"selector": {"matchLabels": {"app": "a"}}, "template": _tpl()},
          "status": {"desiredNumberScheduled": 2, "currentNumberScheduled": 2, "numberAvailable": 1}}
    assert "Desired Number of Nodes Scheduled: 2" in D.describe(ds, [])
    ss = {"kind": "StatefulSet", "metadata": {"name": "db", "namespace": "default"},
          "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "a"}}, "template": _tpl(),
                   "volumeClaimTemplates": [{"metadata": {"name": "data"}, "spec": {"accessModes": ["ReadWriteOnce"],
                                                                                    "resources": {"requests": {"storage": "1Gi"}}}}]},
          "status": {"replicas": 2}}
    out = D.describe(ss, [])
    assert "2 desired | 2 total" in out and "Volume Claims:" in out and "1Gi" in out
    job = {"kind": "Job", "metadata": {"name": "j", "namespace": "default"},
           "spec": {"parallelism": 2, "completions": 4, "template": _tpl()}, "status": {"active": 1, "succeeded": 2}}
    assert "Pods Statuses:" in D.describe(job, []) and "1 Running / 2 Succeeded / 0 Failed" in D.describe(job, [])
    svc = {"kind": "Service", "metadata": {"name": "web", "namespace": "default"},
           "spec": {"type": "ClusterIP", "clusterIP": "10.0.0.9", "selector": {"app": "a"},
                    "ports": [{"name": "http", "port": 80, "targetPort": 8080, "protocol": "TCP"}]}}
    ep = {"subsets": [{"addresses": [{"ip": "10.1.0.1"}], "ports": [{"name": "http", "port": 8080}]}]}
    out = D.describe(svc, [], endpoints=ep)
    assert "TargetPort:" in out and "8080/TCP" in out and "10.1.0.1:8080" in out and "Session Affinity:" in out
    pvc = {"kind": "PersistentVolumeClaim", "metadata": {"name": "c", "namespace": "default"},
           "spec": {"volumeName": "pv1"}, "status": {"phase": "Bound", "capacity": {"storage": "1Gi"}, "accessModes": ["ReadWriteOnce"]}}
    users = [{"metadata": {"name": "user"}, "spec": {"volumes": [{"name": "v", "persistentVolumeClaim": {"claimName": "c"}}]}}]
    out = D.describe(pvc, [], pods=users)
    assert "Mounted By:" in out and "user" in out and "RWO" in out
    pv = {"kind": "PersistentVolume", "metadata": {"name": "pv1"},
          "spec": {"capacity": {"storage": "1Gi"}, "hostPath": {"path": "/data"}, "persistentVolumeReclaimPolicy": "Delete"},
          "status": {"phase": "Bound"}}
    out = D.describe(pv, [])
    assert "HostPath (bare host directory volume)" in out and "/data" in out and "Reclaim Policy:" in out
    ns = {"kind": "Namespace", "metadata": {"name": "team"}, "status": {"phase": "Active"}}
    quotas = [{"metadata": {"name": "q"}, "status": {"hard": {"amd.com/gpu": "8", "pods": "10"},
                                                     "used": {"amd.com/gpu": "2", "pods": "3"}}}]
    limits = [{"spec": {"limits": [{"type": "Container", "max": {"cpu": "2"}, "default": {"cpu": "500m"}}]}}]
    out = D.describe(ns, [], quotas=quotas, limits=limits)
    assert "Resource Quotas" in out and "amd.com/gpu" in out and "Resource Limits" in out and "500m" in out
    assert "No resource quota." in D.describe(ns, [], quotas=[], limits=[])


# ---------------------------------------------------------------------------- end to end
IDS: dict = {}      # pod name -> the device IDs the fixture bound it to


@pytest.fixture(scope="module")
def server():
    loop = asyncio.new_event_loop()
    box = {}
    ready = threading.Event()

    def serve():
        asyncio.set_event_loop(loop)
        box["srv"] = loop.run_until_complete(APIServer().start())
        ready.set()
        loop.run_forever()
    t = threading.Thread(target=serve, daemon=True)
    t.start()
    ready.wait(10)

    async def seed():
        c = Client(box["srv"].url)
        from amdkube.benchmark.schedperf import fake_node
        from amdkube.smi import FakeBackend
        node = await c.create(fake_node(0, 4, FakeBackend()))
        devs = sorted(node["status"]["extendedResources"]["amd.com/gpu"]["resources"])
        for i, (name, n) in enumerate((("p2", 2), ("p10", 1), ("p1", 0))):
            c0 = {"name": "c", "image": "busybox"}
            if n:
                c0["resources"] = {"limits": {"amd.com/gpu": str(n)}}
            pod = await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": {"idx": str(i)}},
                                  "spec": {"containers": [c0]}}, "default")
            if n:
                pres = pod["spec"]["extendedResources"][0]["name"]
                ids, devs = devs[:n], devs[n:]
                await c.bind("default", name, m.name_of(node), {pres: {"resources": ids}})
                box.setdefault("ids", {})[name] = ids
        await c.close()
    asyncio.run_coroutine_threadsafe(seed(), loop).result(30)
    IDS.update(box.get("ids", {}))
    yield box["srv"].url
    asyncio.run_coroutine_threadsafe(box["srv"].stop(), loop).result(30)
    loop.call_soon_threadsafe(loop.stop)
    t.join(10)
    loop.close()


def k(url, *args):
    buf = io.StringIO()
    with redirect_stdout(buf):
        rc = kubectl(["--server", url, *args])
    return rc, buf.getvalue()


def test_kubectl_jsonpath_lists_each_pods_gpus(server):
    rc, out = k(server, "get", "pods", "-o",
                'jsonpath={range .items[*]}{.metadata.name}{"\\t"}{.spec.extendedResources[*].assigned}{"\\n"}{end}')
    assert rc == 0
    lines = dict(ln.split("\t") for ln in out.splitlines())
    ids = IDS
    assert lines == {"p2": "[" + " ".join(ids["p2"]) + "]", "p10": "[" + ids["p10"][0] + "]", "p1": ""}


def test_kubectl_custom_columns_go_template_sort_by(server):
    rc, out = k(server, "get", "pods", "-o", "custom-columns=NAME:.metadata.name,IDX:.metadata.labels.idx", "--sort-by",
                ".metadata.name")
    assert [ln.split() for ln in out.splitlines()] == [["NAME", "IDX"], ["p1", "2"], ["p2", "0"], ["p10", "1"]]
    rc, out = k(server, "get", "pods", "-o", "go-template={{range .items}}{{.metadata.name}} {{end}}", "--sort-by",
                "{.metadata.labels.idx}")
    assert out == "p2 p10 p1 "
    rc, out = k(server, "get", "pods", "-L", "idx", "--show-labels")
    head = out.splitlines()[0].split()
    assert head[-2:] == ["IDX", "LABELS"] and any("idx=1" in ln for ln in out.splitlines())
    rc, out = k(server, "get", "pods", "-o", "jsonpath={.items[?(@.metadata.labels.idx==\"1\")].metadata.name}")
    assert out == "p10"
