"""Defaulting (SetDefaults_*) for the kinds amdkube serves.

Reference: pkg/apis/core/v1/defaults.go:131 (SetDefaults_Pod), :164-179 (fork: copy
ExtendedResources limits into requests), container/pod defaults in the same file,
pkg/apis/apps/v1 defaults for DaemonSet/ReplicaSet/Deployment.
"""
from __future__ import annotations

from .quantity import Quantity, QuantityError
from .scheme import register_hooks


def normalize_resource_list(rl: dict | None):
    """Quantities are strings on the wire ("2", "500m", "288Gi"), whatever the manifest held."""
    if not rl:
        return
    for k, v in list(rl.items()):
        if not isinstance(v, str):
            try:
                rl[k] = str(Quantity(v))
            except (QuantityError, TypeError, ValueError):
                pass


def _default_container(c: dict):
    res = c.get("resources")
    if res:
        normalize_resource_list(res.get("limits"))
        normalize_resource_list(res.get("requests"))
    c.setdefault("terminationMessagePath", "/dev/termination-log")
    c.setdefault("terminationMessagePolicy", "File")
    img = c.get("image") or ""
    if "imagePullPolicy" not in c:
        c["imagePullPolicy"] = "Always" if img.endswith(":latest") or ":" not in img.rsplit("/", 1)[-1] else "IfNotPresent"
    res = c.get("resources")
    if res and res.get("limits"):
        req = res.setdefault("requests", {})
        for k, v in res["limits"].items():
            req.setdefault(k, v)
    for p in c.get("ports") or []:
        p.setdefault("protocol", "TCP")
    for e in c.get("env") or []:               # SetDefaults_ObjectFieldSelector
        fr = (e.get("valueFrom") or {}).get("fieldRef")
        if fr is not None:
            fr.setdefault("apiVersion", "v1")
    for probe in ("livenessProbe", "readinessProbe"):
        pr = c.get(probe)
        if pr:
            pr.setdefault("timeoutSeconds", 1)
            pr.setdefault("periodSeconds", 10)
            pr.setdefault("successThreshold", 1)
            pr.setdefault("failureThreshold", 3)


def default_pod_spec(spec: dict):
    spec.setdefault("restartPolicy", "Always")
    spec.setdefault("dnsPolicy", "ClusterFirst")
    spec.setdefault("terminationGracePeriodSeconds", 30)
    spec.setdefault("schedulerName", "default-scheduler")
    spec.setdefault("securityContext", {})
    for c in spec.get("containers") or []:
        _default_container(c)
        if spec.get("hostNetwork"):
            # SetDefaults_PodSpec: a host-network pod's hostPort is its containerPort
            for port in c.get("ports") or []:
                if not port.get("hostPort"):
                    port["hostPort"] = port.get("containerPort", 0)
    for c in spec.get("initContainers") or []:
        _default_container(c)
    # fork: ExtendedResources requests := limits (defaults.go:164-179)
    for pres in spec.get("extendedResources") or []:
        res = pres.setdefault("resources", {})
        normalize_resource_list(res.get("limits"))
        normalize_resource_list(res.get("requests"))
        lim = res.get("limits") or {}
        if lim and not res.get("requests"):
            res["requests"] = dict(lim)
        pres.setdefault("affinity", {})
    for v in spec.get("volumes") or []:
        if not any(k for k in v if k != "name"):
            v["emptyDir"] = {}
        for it in (v.get("downwardAPI") or {}).get("items") or []:
            if it.get("fieldRef") is not None:
                it["fieldRef"].setdefault("apiVersion", "v1")


def default_pod(pod: dict):
    pod.setdefault("spec", {})
    default_pod_spec(pod["spec"])
    return pod


def default_node(node: dict):
    node.setdefault("spec", {})
    st = node.setdefault("status", {})
    normalize_resource_list(st.get("capacity"))
    normalize_resource_list(st.get("allocatable"))
    if st.get("capacity") and not st.get("allocatable"):
        st["allocatable"] = dict(st["capacity"])
    return node


def default_namespace(ns: dict):
    ns.setdefault("spec", {}).setdefault("finalizers", ["kubernetes"])
    ns.setdefault("status", {}).setdefault("phase", "Active")
    return ns


def _default_template_owner(obj: dict, replicas=True):
    spec = obj.setdefault("spec", {})
    if replicas:
        spec.setdefault("replicas", 1)
    tpl = spec.setdefault("template", {})
    default_pod_spec(tpl.setdefault("spec", {}))
    if "selector" not in spec and (tpl.get("metadata") or {}).get("labels"):
        spec["selector"] = {"matchLabels": dict(tpl["metadata"]["labels"])}
    return obj


def default_daemonset(ds: dict):
    _default_template_owner(ds, replicas=False)
    if ds.get("apiVersion") == "extensions/v1beta1":
        # extensions/v1beta1 keeps the pre-1.6 behaviour (pkg/apis/extensions/v1beta1/defaults.go):
        # OnDelete unless asked, and a templateGeneration
        ds["spec"].setdefault("updateStrategy", {"type": "OnDelete"})
        ds["spec"].setdefault("templateGeneration", 1)
    us = ds["spec"].setdefault("updateStrategy", {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 1}})
    us.setdefault("type", "RollingUpdate")
    if us["type"] == "RollingUpdate":
        us.setdefault("rollingUpdate", {}).setdefault("maxUnavailable", 1)
    ds["spec"].setdefault("revisionHistoryLimit", 10)
    return ds


def default_replicaset(rs: dict):
    return _default_template_owner(rs)


def default_deployment(d: dict):
    _default_template_owner(d)
    st = d["spec"].setdefault("strategy", {"type": "RollingUpdate",
                                           "rollingUpdate": {"maxUnavailable": "25%", "maxSurge": "25%"}})
    st.setdefault("type", "RollingUpdate")
    if st["type"] == "RollingUpdate":
        ru = st.setdefault("rollingUpdate", {})
        ru.setdefault("maxUnavailable", "25%")
        ru.setdefault("maxSurge", "25%")
    d["spec"].setdefault("revisionHistoryLimit", 10)
    d["spec"].setdefault("progressDeadlineSeconds", 600)
    return d


def default_job(j: dict):
    """pkg/apis/batch/v1/defaults.go SetDefaults_Job: a Job with neither completions nor
    parallelism runs one pod to one completion; parallelism alone leaves completions unset
    (a work-queue Job)."""
    spec = j.setdefault("spec", {})
    if spec.get("completions") is None and spec.get("parallelism") is None:
        spec["completions"] = 1
    if spec.get("parallelism") is None:
        spec["parallelism"] = 1
    spec.setdefault("backoffLimit", 6)
    tpl = spec.setdefault("template", {})
    tspec = tpl.setdefault("spec", {})
    tspec.setdefault("restartPolicy", "OnFailure")
    default_pod_spec(tspec)
    return j


def default_service(s: dict):
    spec = s.setdefault("spec", {})
    spec.setdefault("type", "ClusterIP")
    spec.setdefault("sessionAffinity", "None")
    if spec["type"] in ("NodePort", "LoadBalancer"):
        spec.setdefault("externalTrafficPolicy", "Cluster")     # SetDefaults_Service
    for p in spec.get("ports") or []:
        p.setdefault("protocol", "TCP")
        p.setdefault("targetPort", p.get("port"))
    return s


def default_limit_range(lr: dict):
    """SetDefaults_LimitRangeItem (pkg/apis/core/v1/defaults.go:339-369) on every Container item:
    default <- max, defaultRequest <- default, then <- min."""
    for i, item in enumerate((lr.get("spec") or {}).get("limits") or []):
        for k in ("max", "min", "default", "defaultRequest", "maxLimitRequestRatio"):
            normalize_resource_list(item.get(k))
        if item.get("type") == "Container":
            default, dreq = item.setdefault("default", {}), item.setdefault("defaultRequest", {})
            for k, v in (item.get("max") or {}).items():
                default.setdefault(k, v)
            for k, v in default.items():
                dreq.setdefault(k, v)
            for k, v in (item.get("min") or {}).items():
                dreq.setdefault(k, v)
    return lr


register_hooks("Pod", defaulter=default_pod)
register_hooks("LimitRange", defaulter=default_limit_range)
register_hooks("Node", defaulter=default_node)
register_hooks("Namespace", defaulter=default_namespace)
register_hooks("Service", defaulter=default_service)
register_hooks("DaemonSet", "apps/v1", defaulter=default_daemonset)
for _gv in ("apps/v1beta2", "extensions/v1beta1"):
    try:
        register_hooks("DaemonSet", _gv, defaulter=default_daemonset)
    except KeyError:
        pass
register_hooks("ReplicaSet", "apps/v1", defaulter=default_replicaset)
register_hooks("Deployment", "apps/v1", defaulter=default_deployment)
register_hooks("Job", "batch/v1", defaulter=default_job)


def default_cronjob(cj: dict, history_limits: bool = True):
    """SetDefaults_CronJob (batch/v1beta1/defaults.go): concurrency Allow, not suspended, and
    3 successful / 1 failed finished jobs kept (batch/v2alpha1 leaves the limits unset)."""
    spec = cj.setdefault("spec", {})
    spec.setdefault("concurrencyPolicy", "Allow")
    spec.setdefault("suspend", False)
    if history_limits:
        spec.setdefault("successfulJobsHistoryLimit", 3)
        spec.setdefault("failedJobsHistoryLimit", 1)
    return cj


for _gv, _limits in (("batch/v1beta1", True), ("batch/v2alpha1", False)):
    try:
        register_hooks("CronJob", _gv, defaulter=lambda cj, _l=_limits: default_cronjob(cj, _l))
    except KeyError:
        pass


def default_pod_security_policy(psp: dict):
    """SetDefaults_PodSecurityPolicySpec (extensions/v1beta1/defaults.go): privilege escalation
    is allowed unless the policy says otherwise."""
    spec = psp.setdefault("spec", {})
    if spec.get("allowPrivilegeEscalation") is None:
        spec["allowPrivilegeEscalation"] = True
    return psp


for _gv in ("extensions/v1beta1", "policy/v1beta1"):
    try:
        register_hooks("PodSecurityPolicy", _gv, defaulter=default_pod_security_policy)
    except KeyError:
        pass


# ---------------------------------------------------------------- the remaining served kinds
# (pkg/apis/*/v1*/defaults.go): every object is defaulted before it is validated, so each kind
# the validators require defaulted fields of gets its defaulter here
def _default_template(tpl: dict | None):
    if tpl is not None:
        default_pod_spec(tpl.setdefault("spec", {}))


def default_statefulset(sts: dict):
    """apps/v1 SetDefaults_StatefulSet: OrderedReady, RollingUpdate with partition 0, 1 replica,
    10 revisions, selector from the template labels."""
    spec = sts.setdefault("spec", {})
    spec.setdefault("replicas", 1)
    spec.setdefault("podManagementPolicy", "OrderedReady")
    us = spec.setdefault("updateStrategy", {"type": "RollingUpdate"})
    us.setdefault("type", "RollingUpdate")
    if us["type"] == "RollingUpdate":
        us.setdefault("rollingUpdate", {}).setdefault("partition", 0)
    spec.setdefault("revisionHistoryLimit", 10)
    tpl = spec.setdefault("template", {})
    _default_template(tpl)
    if "selector" not in spec and (tpl.get("metadata") or {}).get("labels"):
        spec["selector"] = {"matchLabels": dict(tpl["metadata"]["labels"])}
    return sts


def default_replication_controller(rc: dict):
    """core/v1 SetDefaults_ReplicationController: selector (and labels) from the template,
    one replica."""
    spec = rc.setdefault("spec", {})
    tpl = spec.get("template")
    labels = ((tpl or {}).get("metadata") or {}).get("labels") or {}
    if labels:
        spec.setdefault("selector", dict(labels))
        md = rc.setdefault("metadata", {})
        if not md.get("labels"):
            md["labels"] = dict(labels)
    spec.setdefault("replicas", 1)
    _default_template(tpl)
    return rc


def default_pod_template(pt: dict):
    _default_template(pt.get("template"))
    return pt


def default_cronjob_template(cj: dict, history_limits: bool = True):
    default_cronjob(cj, history_limits)
    jt = cj["spec"].setdefault("jobTemplate", {}).setdefault("spec", {})
    tpl = jt.setdefault("template", {})
    tpl.setdefault("spec", {}).setdefault("restartPolicy", "OnFailure")
    _default_template(tpl)
    return cj


def default_secret(s: dict):
    if not s.get("type"):
        s["type"] = "Opaque"
    return s


def default_endpoints(ep: dict):
    for ss in ep.get("subsets") or []:
        for p in ss.get("ports") or []:
            p.setdefault("protocol", "TCP")
    return ep


def default_persistent_volume(pv: dict):
    pv.setdefault("spec", {}).setdefault("persistentVolumeReclaimPolicy", "Retain")
    pv.setdefault("status", {}).setdefault("phase", "Pending")
    return pv


def default_persistent_volume_claim(pvc: dict):
    pvc.setdefault("status", {}).setdefault("phase", "Pending")
    return pvc


def default_hpa(hpa: dict):
    spec = hpa.setdefault("spec", {})
    if spec.get("minReplicas") is None:
        spec["minReplicas"] = 1
    return hpa


def default_storage_class(sc: dict):
    if not sc.get("reclaimPolicy"):
        sc["reclaimPolicy"] = "Delete"
    return sc


def default_rbac_subjects(obj: dict):
    """rbac/v1 SetDefaults_Subject: users and groups are in the rbac API group."""
    for s in obj.get("subjects") or []:
        if not s.get("apiGroup") and s.get("kind") in ("User", "Group"):
            s["apiGroup"] = "rbac.authorization.k8s.io"
    return obj


register_hooks("StatefulSet", "apps/v1", defaulter=default_statefulset)
register_hooks("ReplicationController", defaulter=default_replication_controller)
register_hooks("PodTemplate", defaulter=default_pod_template)
register_hooks("Secret", defaulter=default_secret)
register_hooks("Endpoints", defaulter=default_endpoints)
register_hooks("PersistentVolume", defaulter=default_persistent_volume)
register_hooks("PersistentVolumeClaim", defaulter=default_persistent_volume_claim)
register_hooks("HorizontalPodAutoscaler", "autoscaling/v1", defaulter=default_hpa)
register_hooks("StorageClass", "storage.k8s.io/v1", defaulter=default_storage_class)
register_hooks("RoleBinding", "rbac.authorization.k8s.io/v1", defaulter=default_rbac_subjects)
register_hooks("ClusterRoleBinding", "rbac.authorization.k8s.io/v1", defaulter=default_rbac_subjects)
for _gv, _limits in (("batch/v1beta1", True), ("batch/v2alpha1", False)):
    try:
        register_hooks("CronJob", _gv, defaulter=lambda cj, _l=_limits: default_cronjob_template(cj, _l))
    except KeyError:
        pass
