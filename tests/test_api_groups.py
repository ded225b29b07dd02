"""Multi-version serving and the reference release's other API groups: extensions/v1beta1
(Deployment/DaemonSet/ReplicaSet aliases of apps, Ingress, PodSecurityPolicy, NetworkPolicy),
apps/v1beta1+v1beta2, networking.k8s.io/v1, settings.k8s.io/v1alpha1 PodPreset,
admissionregistration.k8s.io/v1alpha1 InitializerConfiguration, apiregistration.k8s.io/v1beta1
APIService (validation tables after the reference *_test.go files)."""
import json

import pytest

from amdkube.api import meta as m
from amdkube.api.extgroups import (validate_apiservice, validate_ingress, validate_initializer_configuration,
                                   validate_network_policy, validate_pod_preset, validate_psp)
from amdkube.localcluster import LocalCluster
from tests.conftest import run


def _dep(api="extensions/v1beta1", name="web"):
    return {"apiVersion": api, "kind": "Deployment", "metadata": {"name": name, "namespace": "default"},
            "spec": {"replicas": 2, "template": {"metadata": {"labels": {"app": name}},
                                                 "spec": {"containers": [{"name": "c", "image": "busybox"}]}}}}


def test_served_versions_share_storage_and_rewrite_api_version():
    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            out = await c.create(_dep())                                  # no selector: v1beta1 defaults it
            assert out["apiVersion"] == "extensions/v1beta1" and out["spec"]["selector"] == {"matchLabels": {"app": "web"}}
            for gv in ("apps/v1", "apps/v1beta1", "apps/v1beta2", "extensions/v1beta1"):
                g, v = gv.split("/")
                got = await c.request("GET", f"/apis/{g}/{v}/namespaces/default/deployments/web")
                assert got["apiVersion"] == gv and got["metadata"]["uid"] == out["metadata"]["uid"]
                lst = await c.request("GET", f"/apis/{g}/{v}/namespaces/default/deployments")
                assert lst["apiVersion"] == gv and lst["kind"] == "DeploymentList"
                assert [i["apiVersion"] for i in lst["items"]] == [gv]
            # the storage version is apps/v1; an update through an old version keeps it
            raw = lc.api.registry.rs("deployments", "apps").get("default", "web")
            assert raw["apiVersion"] == "apps/v1"
            got["spec"]["replicas"] = 3
            upd = await c.request("PUT", "/apis/extensions/v1beta1/namespaces/default/deployments/web", body=got)
            assert upd["apiVersion"] == "extensions/v1beta1" and upd["spec"]["replicas"] == 3
            assert lc.api.registry.rs("deployments", "apps").get("default", "web")["spec"]["replicas"] == 3
            # discovery: every served version listed, preferred = storage version
            grp = await c.request("GET", "/apis/apps")
            assert grp["preferredVersion"]["version"] == "v1"
            assert [v["version"] for v in grp["versions"]] == ["v1", "v1beta2", "v1beta1"]
            res = await c.request("GET", "/apis/extensions/v1beta1")
            names = {r["name"] for r in res["resources"]}
            assert {"deployments", "daemonsets", "replicasets", "ingresses", "podsecuritypolicies", "networkpolicies"} <= names
            # watch through an old version sees old-version objects
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.get(lc.api.url + "/apis/apps/v1beta2/namespaces/default/deployments?watch=1&timeoutSeconds=1") as r:
                    first = json.loads((await r.content.readline()).decode())
            assert first["type"] == "ADDED" and first["object"]["apiVersion"] == "apps/v1beta2"
            # new groups are stored and served
            await c.create({"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
                            "metadata": {"name": "deny", "namespace": "default"}, "spec": {"podSelector": {}}})
            np = await c.request("GET", "/apis/extensions/v1beta1/namespaces/default/networkpolicies/deny")
            assert np["apiVersion"] == "extensions/v1beta1" and np["spec"]["policyTypes"] == ["Ingress"]
            await c.create({"apiVersion": "extensions/v1beta1", "kind": "Ingress", "metadata": {"name": "ing", "namespace": "default"},
                            "spec": {"backend": {"serviceName": "web", "servicePort": 80}}})
            with pytest.raises(m.StatusError) as ei:
                await c.create({"apiVersion": "extensions/v1beta1", "kind": "Ingress",
                                "metadata": {"name": "bad", "namespace": "default"}, "spec": {}})
            assert ei.value.code == 422
    run(go(), 60)


def test_network_policy_validation():
    ok = {"metadata": {"name": "a", "namespace": "d"}, "spec": {
        "podSelector": {"matchLabels": {"a": "b"}},
        "ingress": [{"ports": [{"protocol": "TCP", "port": 80}, {"port": "http"}],
                     "from": [{"podSelector": {}}, {"ipBlock": {"cidr": "10.0.0.0/8", "except": ["10.1.0.0/16"]}}]}],
        "policyTypes": ["Ingress"]}}
    assert validate_network_policy(ok) == []
    bad = json.loads(json.dumps(ok))
    bad["spec"]["ingress"][0]["ports"][0]["protocol"] = "SCTP"
    bad["spec"]["ingress"][0]["from"].append({"podSelector": {}, "namespaceSelector": {}})
    bad["spec"]["ingress"][0]["from"][1]["ipBlock"]["except"] = ["192.168.0.0/16"]
    bad["spec"]["policyTypes"] = ["Ingress", "Sideways"]
    errs = validate_network_policy(bad)
    assert len(errs) == 4, errs


def test_ingress_psp_podpreset_initializer_apiservice_validation():
    ing = {"metadata": {"name": "i", "namespace": "d"}, "spec": {"rules": [
        {"host": "*.example.com", "http": {"paths": [{"path": "/api", "backend": {"serviceName": "s", "servicePort": "http"}}]}}]}}
    assert validate_ingress(ing) == []
    ing["spec"]["rules"][0]["host"] = "1.2.3.4"
    ing["spec"]["rules"][0]["http"]["paths"][0]["path"] = "api"
    assert len(validate_ingress(ing)) == 2
    psp = {"metadata": {"name": "p"}, "spec": {"runAsUser": {"rule": "MustRunAs", "ranges": [{"min": 10, "max": 5}]},
                                               "seLinux": {"rule": "RunAsAny"}, "supplementalGroups": {"rule": "RunAsAny"},
                                               "fsGroup": {"rule": "RunAsAny"}, "volumes": ["secret", "bogus"],
                                               "allowedCapabilities": ["NET_ADMIN"], "requiredDropCapabilities": ["NET_ADMIN"]}}
    assert len(validate_psp(psp)) == 3
    pp = {"metadata": {"name": "pp", "namespace": "d"}, "spec": {"selector": {"matchLabels": {"role": "fe"}},
                                                                  "env": [{"name": "DB", "value": "x"}]}}
    assert validate_pod_preset(pp) == []
    assert validate_pod_preset({"metadata": {"name": "pp", "namespace": "d"}, "spec": {}})
    ic = {"metadata": {"name": "ic"}, "initializers": [{"name": "podimage.initializer.com", "rules": [
        {"apiGroups": [""], "apiVersions": ["v1"], "resources": ["pods"]}]}, {"name": "two.parts"}]}
    errs = validate_initializer_configuration(ic)
    assert len(errs) == 1 and "three segments" in errs[0]
    api = {"metadata": {"name": "v1alpha1.metrics.example.com"}, "spec": {
        "group": "metrics.example.com", "version": "v1alpha1", "groupPriorityMinimum": 100, "versionPriority": 10,
        "service": {"namespace": "kube-system", "name": "metrics"}, "insecureSkipTLSVerify": True}}
    assert validate_apiservice(api) == []
    api["metadata"]["name"] = "v1.metrics.example.com"
    api["spec"]["groupPriorityMinimum"] = 30000
    assert len(validate_apiservice(api)) == 2
