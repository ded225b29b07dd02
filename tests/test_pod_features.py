"""Pod features the kubelet resolves (pkg/kubelet/kubelet_pods_test.go makeEnvironmentVariables,
envvars_test.go, expansion_test.go, downwardapi/projected/configmap/git_repo volume tests,
kubelet_pods.go managedHostsFileContent, lifecycle handlers_test.go, termination messages)."""
import asyncio
import os
import subprocess

from amdkube.api import meta as m
from amdkube.kubelet.podcontext import expand, hosts_file, resource_value, service_env
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def test_expand_service_env_resource_value_hosts():
    env = {"A": "1", "B": "x"}
    assert expand("$(A)-$(B)-$(C)-$$(A)", env) == "1-x-$(C)-$(A)"
    svc = {"metadata": {"name": "redis-master"}, "spec": {"clusterIP": "10.0.0.11", "ports": [
        {"name": "db", "port": 6379, "protocol": "TCP"}, {"name": "metrics", "port": 9121}]}}
    e = service_env([svc, {"metadata": {"name": "headless"}, "spec": {"clusterIP": "None", "ports": [{"port": 1}]}}])
    assert e["REDIS_MASTER_SERVICE_HOST"] == "10.0.0.11" and e["REDIS_MASTER_SERVICE_PORT"] == "6379"
    assert e["REDIS_MASTER_SERVICE_PORT_METRICS"] == "9121" and e["REDIS_MASTER_PORT"] == "tcp://10.0.0.11:6379"
    assert e["REDIS_MASTER_PORT_6379_TCP_ADDR"] == "10.0.0.11" and not any(k.startswith("HEADLESS") for k in e)
    pod = {"spec": {"containers": [{"name": "c", "resources": {"limits": {"cpu": "1500m", "memory": "128Mi"},
                                                              "requests": {"cpu": "250m"}}}]}}
    assert resource_value(pod, "c", {"resource": "limits.cpu"}, {}) == "2"                   # rounded up to cores
    assert resource_value(pod, "c", {"resource": "limits.cpu", "divisor": "1m"}, {}) == "1500"
    assert resource_value(pod, "c", {"resource": "limits.memory", "divisor": "1Mi"}, {}) == "128"
    assert resource_value(pod, "c", {"resource": "requests.cpu", "divisor": "1m"}, {}) == "250"
    nolim = {"spec": {"containers": [{"name": "c"}]}}
    assert resource_value(nolim, "c", {"resource": "limits.memory"}, {"memory": 1 << 30}) == str(1 << 30)
    h = hosts_file({"metadata": {"name": "p", "namespace": "ns"}, "spec": {
        "hostname": "web-0", "subdomain": "web", "hostAliases": [{"ip": "10.1.2.3", "hostnames": ["foo.local", "bar.local"]}]}},
        "10.244.0.9", "cluster.local")
    assert "10.244.0.9\tweb-0.web.ns.svc.cluster.local\tweb-0" in h and "10.1.2.3\tfoo.local\tbar.local" in h


def test_env_volumes_hooks_and_termination_messages(tmp_path):
    repo = tmp_path / "repo"
    repo.mkdir()
    g = lambda *a: subprocess.run(["git", *a], cwd=repo, check=True, capture_output=True)   # noqa: E731
    g("init", "-q")
    g("config", "user.email", "t@e.st")
    g("config", "user.name", "t")
    (repo / "hello.txt").write_text("v1\n")
    g("add", ".")
    g("commit", "-qm", "one")
    rev1 = subprocess.run(["git", "rev-parse", "HEAD"], cwd=repo, capture_output=True, text=True).stdout.strip()
    (repo / "hello.txt").write_text("v2\n")
    g("commit", "-qam", "two")

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "db", "namespace": "default"},
                            "spec": {"ports": [{"port": 5432, "name": "pg"}]}})
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cfg", "namespace": "default"},
                            "data": {"greeting": "hi", "other": "x", "bad.key": "skip"}})
            await c.create({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "sec", "namespace": "default"},
                            "data": {"token": "czNjcjN0"}})
            for _ in range(50):    # the kubelet's service informer has the new service
                if any(m.name_of(s) == "db" for s in lc.kubelet.svc_informer.list()):
                    break
                await asyncio.sleep(0.05)
            script = ("env | sort > $AMDKUBE_ROOTFS/out/env; ls -l $AMDKUBE_ROOTFS/proj > $AMDKUBE_ROOTFS/out/ls; "
                      "cat $AMDKUBE_ROOTFS/proj/greeting $AMDKUBE_ROOTFS/proj/mem $AMDKUBE_ROOTFS/proj/tok "
                      "$AMDKUBE_ROOTFS/git/repo/hello.txt > $AMDKUBE_ROOTFS/out/files; "
                      "cat $AMDKUBE_ROOTFS/etc/hosts > $AMDKUBE_ROOTFS/out/hosts; echo $0 $1 > $AMDKUBE_ROOTFS/out/args; "
                      "echo bye > $AMDKUBE_ROOTFS/dev/termination-log; exit 3")
            out = tmp_path / "out"
            out.mkdir()
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "feat", "labels": {"app": "f"}},
                   "spec": {"restartPolicy": "Never", "hostAliases": [{"ip": "10.9.9.9", "hostnames": ["alias.local"]}],
                            "volumes": [{"name": "out", "hostPath": {"path": str(out), "type": "Directory"}},
                                        {"name": "proj", "projected": {"sources": [
                                            {"configMap": {"name": "cfg", "items": [{"key": "greeting", "path": "greeting"}]}},
                                            {"secret": {"name": "sec", "items": [{"key": "token", "path": "tok", "mode": 0o600}]}},
                                            {"downwardAPI": {"items": [{"path": "mem", "resourceFieldRef": {
                                                "containerName": "c", "resource": "limits.memory", "divisor": "1Mi"}}]}}]}},
                                        {"name": "git", "gitRepo": {"repository": str(repo), "revision": rev1}}],
                            "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", script, "$(GREETING)", "$(MISSING)"],
                                            "resources": {"limits": {"memory": "64Mi", "cpu": "500m"}},
                                            "envFrom": [{"configMapRef": {"name": "cfg"}, "prefix": "CFG_"},
                                                        {"secretRef": {"name": "nope", "optional": True}}],
                                            "env": [{"name": "GREETING", "valueFrom": {"configMapKeyRef": {"name": "cfg", "key": "greeting"}}},
                                                    {"name": "MSG", "value": "$(GREETING) world"},
                                                    {"name": "CPU_M", "valueFrom": {"resourceFieldRef": {"resource": "limits.cpu", "divisor": "1m"}}},
                                                    {"name": "MY_IP", "valueFrom": {"fieldRef": {"fieldPath": "status.podIP"}}}],
                                            "volumeMounts": [{"name": "out", "mountPath": "/out"}, {"name": "proj", "mountPath": "/proj"},
                                                             {"name": "git", "mountPath": "/git"}]}]}}
            await c.create(pod, "default")
            p = await wait_pod(c, "default", "feat", ("Failed",), 30)
            env = dict(line.split("=", 1) for line in (out / "env").read_text().splitlines() if "=" in line)
            assert env["MSG"] == "hi world" and env["CPU_M"] == "500" and env["CFG_greeting"] == "hi"
            assert "CFG_bad.key" not in env and env["DB_SERVICE_PORT_PG"] == "5432" and env["DB_SERVICE_HOST"]
            assert env["KUBERNETES_SERVICE_HOST"] and env["MY_IP"] == lc.kubelet.cfg.node_ip
            assert (out / "files").read_text().strip() == "hi64s3cr3tv1"     # values carry no trailing newline
            assert (out / "args").read_text().split() == ["hi", "$(MISSING)"]
            assert "10.9.9.9\talias.local" in (out / "hosts").read_text()
            term = p["status"]["containerStatuses"][0]["state"]["terminated"]
            assert term["exitCode"] == 3 and term["message"].strip() == "bye"
            # FallbackToLogsOnError: the log tail when nothing was written
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "fb"}, "spec": {"restartPolicy": "Never",
                            "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "echo boom-from-log; exit 1"],
                                            "terminationMessagePolicy": "FallbackToLogsOnError"}]}}, "default")
            p = await wait_pod(c, "default", "fb", ("Failed",), 30)
            assert "boom-from-log" in p["status"]["containerStatuses"][0]["state"]["terminated"]["message"]
            # postStart: a failing hook kills the container
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hook"}, "spec": {"restartPolicy": "Never",
                            "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"],
                                            "lifecycle": {"postStart": {"exec": {"command": ["sh", "-c", "exit 7"]}}}}]}}, "default")
            for _ in range(100):
                evs, _ = await c.list("events", "default", field_selector="involvedObject.name=hook")
                if any(e["reason"] == "FailedPostStartHook" for e in evs):
                    break
                await asyncio.sleep(0.1)
            assert any(e["reason"] == "FailedPostStartHook" for e in evs)
            p = await wait_pod(c, "default", "hook", ("Failed",), 30)
    run(go(), 90)
