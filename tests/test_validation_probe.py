"""The round-5 verdict's validation probe, through a real apiserver: 13 invalid pods and 12
invalid objects of other kinds are all refused with 422 (each for the reason the reference's
validators give), a valid control object of each kind is accepted, and an invalid
ResourceQuota can no longer be stored to block every pod create in its namespace.

Reference: pkg/apis/core/validation/validation.go (ValidatePodSpec :2879 and its
sub-validators, ValidatePersistentVolume :1453, ValidatePersistentVolumeClaim :1731,
ValidateReplicationController :3727, ValidateLimitRange :4138, ValidateResourceQuota :4492,
ValidateEndpoints :4698), apps/batch/autoscaling/policy/storage/rbac validation.go.
"""
import copy

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import APIServer
from amdkube.client import Client
from tests.conftest import run


def pod(name, **spec_over):
    c = {"name": "c", "image": "busybox"}
    c.update(spec_over.pop("container", {}))
    spec = {"containers": [c]}
    spec.update(spec_over)
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"}, "spec": spec}


BAD_PODS = {
    "dnsPolicy": (pod("p1", dnsPolicy="Bogus"), "spec.dnsPolicy: Unsupported value"),
    "imagePullPolicy": (pod("p2", container={"imagePullPolicy": "Sometimes"}), "imagePullPolicy: Unsupported value"),
    "empty probe": (pod("p3", container={"livenessProbe": {}}), "livenessProbe: Required value: must specify a handler type"),
    "two handlers + negative period": (pod("p4", container={"readinessProbe": {
        "exec": {"command": ["true"]}, "tcpSocket": {"port": 80}, "periodSeconds": -1}}),
        "readinessProbe.tcpSocket: Forbidden: may not specify more than 1 handler type"),
    "runAsUser": (pod("p5", securityContext={"runAsUser": -3}), "securityContext.runAsUser: Invalid value: -3"),
    "port name": (pod("p6", container={"ports": [{"name": "a" * 34, "containerPort": 80}]}),
                  "ports[0].name: Invalid value"),
    "anti-affinity topologyKey": (pod("p7", affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"a": "b"}}}]}}), "topologyKey: Required value: can not be empty"),
    "empty mountPath": (pod("p8", volumes=[{"name": "v", "emptyDir": {}}],
                            container={"volumeMounts": [{"name": "v", "mountPath": ""}]}), "mountPath: Required value"),
    "two volume sources": (pod("p9", volumes=[{"name": "v", "emptyDir": {}, "hostPath": {"path": "/tmp"}}]),
                           "spec.volumes[0].hostPath: Forbidden: may not specify more than 1 volume type"),
    "hostname": (pod("p10", hostname="Not_Valid!"), "spec.hostname: Invalid value"),
    "terminationMessagePolicy": (pod("p11", container={"terminationMessagePolicy": "Whenever"}),
                                 "terminationMessagePolicy: Invalid value"),
    "subPath escape": (pod("p12", volumes=[{"name": "v", "emptyDir": {}}],
                           container={"volumeMounts": [{"name": "v", "mountPath": "/x", "subPath": "../../etc"}]}),
                       "subPath: Invalid value: \"../../etc\": must not contain '..'"),
    "volume without a name": (pod("p13", volumes=[{"name": "", "emptyDir": {}}]), "spec.volumes[0].name: Required value"),
}


def _tpl():
    return {"metadata": {"labels": {"app": "a"}}, "spec": {"containers": [{"name": "c", "image": "busybox"}]}}


BAD_OBJECTS = {
    "statefulset replicas": ({"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "s"},
                              "spec": {"replicas": -5, "selector": {"matchLabels": {"app": "a"}}, "template": _tpl()}},
                             "spec.replicas: Invalid value: -5"),
    "empty pvc": ({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "c"}, "spec": {}},
                  "spec.accessModes: Required value"),
    "empty pv": ({"apiVersion": "v1", "kind": "PersistentVolume", "metadata": {"name": "pv0"}, "spec": {}},
                 "spec.accessModes: Required value"),
    "hpa max < min": ({"apiVersion": "autoscaling/v1", "kind": "HorizontalPodAutoscaler", "metadata": {"name": "h"},
                       "spec": {"scaleTargetRef": {"kind": "Deployment", "name": "d"}, "minReplicas": 5, "maxReplicas": 0}},
                      "spec.maxReplicas: Invalid value: 0: must be greater than 0"),
    "pdb min and max": ({"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget", "metadata": {"name": "b"},
                         "spec": {"minAvailable": 1, "maxUnavailable": 1, "selector": {"matchLabels": {"a": "b"}}}},
                        "minAvailable and maxUnavailable cannot be both set"),
    "cron schedule": ({"apiVersion": "batch/v1beta1", "kind": "CronJob", "metadata": {"name": "cj"},
                       "spec": {"schedule": "not a schedule", "jobTemplate": {"spec": {"template": _tpl()}}}},
                      "spec.schedule: Invalid value"),
    "endpoints": ({"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "e"},
                   "subsets": [{"addresses": [{"ip": "not-an-ip"}], "ports": [{"port": 99999}]}]},
                  "subsets[0].addresses[0].ip: Invalid value"),
    "rc replicas": ({"apiVersion": "v1", "kind": "ReplicationController", "metadata": {"name": "rc"},
                     "spec": {"replicas": -1, "selector": {"app": "a"}, "template": _tpl()}}, "spec.replicas: Invalid value: -1"),
    "quota negative": ({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"}, "spec": {"hard": {"cpu": "-1"}}},
                       "spec.hard[cpu]: Invalid value: \"-1\": must be greater than or equal to 0"),
    "limitrange min > max": ({"apiVersion": "v1", "kind": "LimitRange", "metadata": {"name": "l"},
                              "spec": {"limits": [{"type": "Container", "min": {"cpu": "2"}, "max": {"cpu": "1"}}]}},
                             "min value 2 is greater than max value 1"),
    "storageclass provisioner": ({"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": "sc"}},
                                 "provisioner: Required value"),
    "role without verbs": ({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "r"},
                            "rules": [{"apiGroups": [""], "resources": ["pods"]}]},
                           "rules[0].verbs: Required value: verbs must contain at least one value"),
}


def _fix(obj):
    """The valid twin of a bad object (accepted: the refusals come from the one bad field)."""
    o = copy.deepcopy(obj)
    k = o["kind"]
    if k == "StatefulSet":
        o["spec"]["replicas"] = 1
    elif k == "PersistentVolumeClaim":
        o["spec"] = {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}
    elif k == "PersistentVolume":
        o["spec"] = {"accessModes": ["ReadWriteOnce"], "capacity": {"storage": "1Gi"}, "hostPath": {"path": "/tmp/pv0"}}
    elif k == "HorizontalPodAutoscaler":
        o["spec"]["maxReplicas"] = 6
    elif k == "PodDisruptionBudget":
        del o["spec"]["maxUnavailable"]
    elif k == "CronJob":
        o["spec"]["schedule"] = "*/5 * * * *"
    elif k == "Endpoints":
        o["subsets"] = [{"addresses": [{"ip": "10.1.2.3"}], "ports": [{"port": 8080}]}]
    elif k == "ReplicationController":
        o["spec"]["replicas"] = 1
    elif k == "ResourceQuota":
        o["spec"]["hard"]["cpu"] = "4"
    elif k == "LimitRange":
        o["spec"]["limits"][0]["max"]["cpu"] = "4"
    elif k == "StorageClass":
        o["provisioner"] = "kubernetes.io/no-provisioner"
    elif k == "Role":
        o["rules"][0]["verbs"] = ["get"]
    return o


def test_the_verdict_probe_is_refused_with_422():
    async def go():
        srv = await APIServer().start()
        # the loopback (system:masters) client: an anonymous one may not grant RBAC rules at all
        # (rbacescalation), which would refuse the valid Role twin for a different reason
        c = Client(srv.url, token=srv.loopback_token)
        try:
            for what, (obj, msg) in list(BAD_PODS.items()) + list(BAD_OBJECTS.items()):
                with pytest.raises(m.StatusError) as ei:
                    await c.create(copy.deepcopy(obj), "default")
                assert ei.value.code == 422, (what, ei.value)
                assert msg in str(ei.value), (what, str(ei.value))
            good = pod("ok", volumes=[{"name": "v", "emptyDir": {}}],
                       container={"volumeMounts": [{"name": "v", "mountPath": "/x", "subPath": "data"}],
                                  "livenessProbe": {"httpGet": {"path": "/", "port": "http"}},
                                  "ports": [{"name": "http", "containerPort": 80}]},
                       affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                           {"labelSelector": {"matchLabels": {"a": "b"}}, "topologyKey": "kubernetes.io/hostname"}]}})
            await c.create(good, "default")
            # the valid twins are stored (the refusals above are not blanket ones)
            for what, (obj, _) in BAD_OBJECTS.items():
                await c.create(_fix(obj), "default")
            assert (await c.get("resourcequotas", "q", "default"))["spec"]["hard"] == {"cpu": "4"}
        finally:
            await c.close()
            await srv.stop()
    run(go(), 60)


def test_updates_keep_pod_spec_immutable_and_allow_image_changes():
    async def go():
        srv = await APIServer().start()
        c = Client(srv.url)
        try:
            p = await c.create(pod("u"), "default")
            p["spec"]["containers"][0]["image"] = "busybox:2"
            p = await c.update(p)
            assert p["spec"]["containers"][0]["image"] == "busybox:2"
            p["spec"]["restartPolicy"] = "Never"
            with pytest.raises(m.StatusError) as ei:
                await c.update(p)
            assert ei.value.code == 422 and "pod updates may not change fields" in str(ei.value)
        finally:
            await c.close()
            await srv.stop()
    run(go(), 60)
