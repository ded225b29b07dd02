"""Validation of the non-core API groups' kinds.

Reference:
* pkg/apis/apps/validation/validation.go — ValidateStatefulSetSpec (:72-137), ValidateStatefulSet
  (:140), ValidateStatefulSetUpdate (:147), ValidateStatefulSetStatus (:172);
* pkg/apis/extensions/validation/validation.go — ValidateDaemonSetSpec (:110),
  ValidateDaemonSetUpdateStrategy (:156), ValidateRollingUpdateDaemonSet (:144),
  ValidatePositiveIntOrPercent / IsNotMoreThan100Percent (:182-224),
  ValidateRollingUpdateDeployment / ValidateDeploymentStrategy (:226-258),
  ValidateDeploymentSpec (:268), ValidateReplicaSetSpec (:576),
  ValidatePodTemplateSpecForReplicaSet (:601);
* pkg/apis/batch/validation/validation.go — ValidateJob / validateJobSpec (:64-125),
  ValidateJobSpecUpdate (:156), ValidateCronJob(+Spec) (:170-219), validateConcurrencyPolicy,
  validateScheduleFormat (cron.ParseStandard), ValidateJobTemplateSpec (:246);
* pkg/apis/autoscaling/validation/validation.go — validateHorizontalPodAutoscalerSpec (:41),
  ValidateCrossVersionObjectReference (:60), validateMetricSpec and the three sources (:121-224);
* pkg/apis/policy/validation/validation.go — ValidatePodDisruptionBudget(+Spec, +Update);
* pkg/apis/storage/validation/validation.go — ValidateStorageClass(+Update);
* pkg/apis/rbac/validation/validation.go — ValidateRole / ClusterRole / RoleBinding /
  ClusterRoleBinding and validatePolicyRule / validateRoleBindingSubject;
* pkg/apis/scheduling/validation/validation.go — ValidatePriorityClass(+Update).
"""
from __future__ import annotations

import json

from .corevalidation import (_go, _selector, dns_subdomain, forbidden, invalid, is_int, is_valid_path_segment_name,
                             is_valid_percent, nonneg, not_supported, required, too_long, validate_label_selector,
                             validate_labels, validate_pod_specific_annotations, validate_pod_template_spec,
                             validate_read_only_persistent_disks)
from .labels import is_qualified_name
from .quantity import Quantity, QuantityError

IMMUTABLE = "field is immutable"


def _meta(obj, namespaced=True, name_fn=None):
    from .validation import validate_object_meta
    return validate_object_meta(obj, namespaced, name_fn) if name_fn else validate_object_meta(obj, namespaced)


def _tpl_labels(spec):
    return (((spec.get("template") or {}).get("metadata")) or {}).get("labels") or {}


def _selector_checks(spec, p, kind, required_sel=True) -> tuple[list[str], object]:
    errs = []
    sel = spec.get("selector")
    if sel is None:
        if required_sel:
            errs.append(required(f"{p}.selector"))
    else:
        errs += validate_label_selector(sel, f"{p}.selector")
        if not (sel.get("matchLabels") or {}) and not (sel.get("matchExpressions") or []):
            errs.append(invalid(f"{p}.selector", _go(sel), f"empty selector is not valid for {kind}."))
    return errs, (_selector(sel) if sel is not None else None)


def validate_template_for_replicaset(tpl, selector, replicas, p) -> list[str]:
    if tpl is None:
        return [required(p)]
    errs = []
    labels = ((tpl.get("metadata") or {}).get("labels")) or {}
    if selector is not None and not selector.empty() and not selector.matches(labels):
        errs.append(invalid(f"{p}.metadata.labels", _go(labels), "`selector` does not match template `labels`"))
    errs += validate_pod_template_spec(tpl, p)
    tspec = tpl.get("spec") or {}
    if is_int(replicas) and replicas > 1:
        errs += validate_read_only_persistent_disks(tspec.get("volumes"), f"{p}.spec.volumes")
    if tspec.get("restartPolicy") != "Always":
        errs.append(not_supported(f"{p}.spec.restartPolicy", tspec.get("restartPolicy") or "", ["Always"]))
    if tspec.get("activeDeadlineSeconds") is not None:
        errs.append(invalid(f"{p}.spec.activeDeadlineSeconds", tspec["activeDeadlineSeconds"], "must not be specified"))
    return errs


# ------------------------------------------------------------------ int-or-percent
def _percent(v):
    if isinstance(v, str) and not is_valid_percent(v):
        return int(v[:-1]), True
    return 0, False


def _int_or_percent(v) -> int:
    val, pct = _percent(v)
    if pct:
        return val
    if is_int(v):
        return v
    try:
        return int(v)
    except (TypeError, ValueError):
        return 0


def validate_positive_int_or_percent(v, p) -> list[str]:
    if isinstance(v, str):
        return [invalid(p, v, m) for m in is_valid_percent(v)]
    if is_int(v):
        return nonneg(v, p)
    return [invalid(p, _go(v), "must be an integer or percentage (e.g '5%%')")]


def not_more_than_100_percent(v, p) -> list[str]:
    val, pct = _percent(v)
    return [invalid(p, v, "must not be greater than 100%")] if pct and val > 100 else []


# ------------------------------------------------------------------ apps
def validate_statefulset(sts, old=None) -> list[str]:
    spec = sts.get("spec") or {}
    errs = _meta(sts)
    pmp = spec.get("podManagementPolicy") or ""
    if not pmp:
        errs.append(required("spec.podManagementPolicy"))
    elif pmp not in ("OrderedReady", "Parallel"):
        errs.append(invalid("spec.podManagementPolicy", pmp, "must be 'OrderedReady' or 'Parallel'"))
    us = spec.get("updateStrategy") or {}
    t = us.get("type") or ""
    if not t:
        errs.append(required("spec.updateStrategy"))
    elif t == "OnDelete":
        if us.get("rollingUpdate") is not None:
            errs.append(invalid("spec.updateStrategy.rollingUpdate", _go(us["rollingUpdate"]),
                                "only allowed for updateStrategy 'RollingUpdate'"))
    elif t == "RollingUpdate":
        if us.get("rollingUpdate") is not None:
            errs += nonneg((us["rollingUpdate"] or {}).get("partition", 0), "spec.updateStrategy.rollingUpdate.partition")
    else:
        errs.append(invalid("spec.updateStrategy", _go(us), "must be 'RollingUpdate' or 'OnDelete'"))
    errs += nonneg(spec.get("replicas", 0), "spec.replicas")
    sel = spec.get("selector")
    if sel is None:
        errs.append(required("spec.selector"))
    else:
        errs += validate_label_selector(sel, "spec.selector")
        if not (sel.get("matchLabels") or {}) and not (sel.get("matchExpressions") or []):
            errs.append(invalid("spec.selector", _go(sel), "empty selector is not valid for statefulset."))
    s = _selector(sel) if sel is not None else None
    if s is None and sel is not None:
        errs.append(invalid("spec.selector", _go(sel), ""))
    else:
        tpl = spec.get("template") or {}
        md = tpl.get("metadata") or {}
        if s is not None and not s.empty() and not s.matches(md.get("labels") or {}):
            errs.append(invalid("spec.template.metadata.labels", _go(md.get("labels") or {}),
                                "`selector` does not match template `labels`"))
        errs += validate_labels(md.get("labels"), "spec.template.labels")
        errs += validate_pod_specific_annotations(md.get("annotations"), tpl.get("spec") or {}, "spec.template.annotations")
    tspec = (spec.get("template") or {}).get("spec") or {}
    if tspec.get("restartPolicy") != "Always":
        errs.append(not_supported("spec.template.spec.restartPolicy", tspec.get("restartPolicy") or "", ["Always"]))
    if tspec.get("activeDeadlineSeconds") is not None:
        errs.append(invalid("spec.spec.activeDeadlineSeconds", tspec["activeDeadlineSeconds"], "must not be specified"))
    if old is not None:
        a = {k: v for k, v in spec.items() if k not in ("replicas", "template", "updateStrategy")}
        b = {k: v for k, v in (old.get("spec") or {}).items() if k not in ("replicas", "template", "updateStrategy")}
        if a != b:
            errs.append(forbidden("spec", "updates to statefulset spec for fields other than 'replicas', 'template', "
                                          "and 'updateStrategy' are forbidden."))
    return errs


def validate_statefulset_status(st, p="status") -> list[str]:
    st = st or {}
    errs = []
    for f in ("replicas", "readyReplicas", "currentReplicas", "updatedReplicas", "observedGeneration", "collisionCount"):
        errs += nonneg(st.get(f, 0), f"{p}.{f}")
    for f in ("readyReplicas", "currentReplicas", "updatedReplicas"):
        if st.get(f, 0) > st.get("replicas", 0):
            errs.append(invalid(f"{p}.{f}", st.get(f, 0), "cannot be greater than status.replicas"))
    return errs


def validate_deployment(d, old=None) -> list[str]:
    spec = d.get("spec") or {}
    errs = _meta(d)
    errs += nonneg(spec.get("replicas", 0), "spec.replicas")
    serrs, sel = _selector_checks(spec, "spec", "deployment")
    errs += serrs
    if spec.get("selector") is not None and sel is None:
        errs.append(invalid("spec.selector", _go(spec.get("selector")), "invalid label selector."))
    else:
        errs += validate_template_for_replicaset(spec.get("template"), sel, spec.get("replicas", 1), "spec.template")
    st = spec.get("strategy") or {}
    t = st.get("type")
    if t == "Recreate":
        if st.get("rollingUpdate") is not None:
            errs.append(forbidden("spec.strategy.rollingUpdate", "may not be specified when strategy `type` is 'Recreate'"))
    elif t == "RollingUpdate":
        ru = st.get("rollingUpdate")
        if ru is None:
            errs.append(required("spec.strategy.rollingUpdate", "this should be defaulted and never be nil"))
        else:
            mu, ms = ru.get("maxUnavailable", "25%"), ru.get("maxSurge", "25%")
            errs += validate_positive_int_or_percent(mu, "spec.strategy.rollingUpdate.maxUnavailable")
            errs += validate_positive_int_or_percent(ms, "spec.strategy.rollingUpdate.maxSurge")
            if _int_or_percent(mu) == 0 and _int_or_percent(ms) == 0:
                errs.append(invalid("spec.strategy.rollingUpdate.maxUnavailable", mu, "may not be 0 when `maxSurge` is 0"))
            errs += not_more_than_100_percent(mu, "spec.strategy.rollingUpdate.maxUnavailable")
    else:
        errs.append(not_supported("spec.strategy", _go(st), ["Recreate", "RollingUpdate"]))
    mrs = spec.get("minReadySeconds", 0)
    errs += nonneg(mrs, "spec.minReadySeconds")
    if spec.get("revisionHistoryLimit") is not None:
        errs += nonneg(spec["revisionHistoryLimit"], "spec.revisionHistoryLimit")
    if spec.get("rollbackTo") is not None:
        errs += nonneg((spec["rollbackTo"] or {}).get("revision", 0), "spec.rollback.version")
    pds = spec.get("progressDeadlineSeconds")
    if pds is not None:
        errs += nonneg(pds, "spec.progressDeadlineSeconds")
        if is_int(pds) and is_int(mrs) and pds <= mrs:
            errs.append(invalid("spec.progressDeadlineSeconds", pds, "must be greater than minReadySeconds."))
    return errs


def validate_replicaset(rs, old=None) -> list[str]:
    spec = rs.get("spec") or {}
    errs = _meta(rs)
    errs += nonneg(spec.get("replicas", 0), "spec.replicas")
    errs += nonneg(spec.get("minReadySeconds", 0), "spec.minReadySeconds")
    serrs, sel = _selector_checks(spec, "spec", "deployment")
    errs += serrs
    if spec.get("selector") is not None and sel is None:
        errs.append(invalid("spec.selector", _go(spec.get("selector")), "invalid label selector."))
    else:
        errs += validate_template_for_replicaset(spec.get("template"), sel, spec.get("replicas", 1), "spec.template")
    return errs


def validate_daemonset(ds, old=None) -> list[str]:
    spec = ds.get("spec") or {}
    errs = _meta(ds)
    sel_obj = spec.get("selector")
    errs += validate_label_selector(sel_obj, "spec.selector")
    sel = _selector(sel_obj) if sel_obj is not None else None
    labels = _tpl_labels(spec)
    if sel is not None and not sel.matches(labels):
        errs.append(invalid("spec.template.metadata.labels", _go(labels), "`selector` does not match template `labels`"))
    if sel_obj is not None and not (sel_obj.get("matchLabels") or {}) and not (sel_obj.get("matchExpressions") or []):
        errs.append(invalid("spec.selector", _go(sel_obj), "empty selector is not valid for daemonset."))
    tpl = spec.get("template") or {}
    errs += validate_pod_template_spec(tpl, "spec.template")
    tspec = tpl.get("spec") or {}
    errs += validate_read_only_persistent_disks(tspec.get("volumes"), "spec.template.spec.volumes")
    if tspec.get("restartPolicy") != "Always":
        errs.append(not_supported("spec.template.spec.restartPolicy", tspec.get("restartPolicy") or "", ["Always"]))
    if tspec.get("activeDeadlineSeconds") is not None:
        errs.append(invalid("spec.template.spec.activeDeadlineSeconds", tspec["activeDeadlineSeconds"], "must not be specified"))
    errs += nonneg(spec.get("minReadySeconds", 0), "spec.minReadySeconds")
    errs += nonneg(spec.get("templateGeneration", 0), "spec.templateGeneration")
    us = spec.get("updateStrategy") or {}
    t = us.get("type")
    if t == "RollingUpdate":
        ru = us.get("rollingUpdate")
        if ru is None:
            errs.append(required("spec.updateStrategy.rollingUpdate"))
        else:
            mu = ru.get("maxUnavailable", 1)
            errs += validate_positive_int_or_percent(mu, "spec.updateStrategy.rollingUpdate.maxUnavailable")
            if _int_or_percent(mu) == 0:
                errs.append(invalid("spec.updateStrategy.rollingUpdate.maxUnavailable", mu, "cannot be 0"))
            errs += not_more_than_100_percent(mu, "spec.updateStrategy.rollingUpdate.maxUnavailable")
    elif t != "OnDelete":
        errs.append(not_supported("spec.updateStrategy", _go(us), ["RollingUpdate", "OnDelete"]))
    if spec.get("revisionHistoryLimit") is not None:
        errs += nonneg(spec["revisionHistoryLimit"], "spec.revisionHistoryLimit")
    if old is not None:
        ospec = old.get("spec") or {}
        ng, og = spec.get("templateGeneration", 0), ospec.get("templateGeneration", 0)
        if is_int(ng) and is_int(og) and (spec.get("templateGeneration") is not None or ospec.get("templateGeneration") is not None):
            changed = spec.get("template") != ospec.get("template")
            if ng < og:
                errs.append(invalid("spec.templateGeneration", ng, "must not be decremented"))
            elif ng == og and changed and old.get("apiVersion") == "extensions/v1beta1":
                errs.append(invalid("spec.templateGeneration", ng, "must be incremented upon template update"))
            elif ng > og and not changed:
                errs.append(invalid("spec.templateGeneration", ng, "must not be incremented without template update"))
    return errs


def validate_controller_revision(cr, old=None) -> list[str]:
    errs = _meta(cr)
    if cr.get("data") is None:
        errs.append(required("data"))
    errs += nonneg(cr.get("revision", 0), "revision")
    if old is not None and cr.get("data") != old.get("data"):
        errs.append(invalid("data", "", IMMUTABLE))
    return errs


# ------------------------------------------------------------------ batch
def _validate_job_spec(spec, p) -> list[str]:
    errs = []
    for f in ("parallelism", "completions", "activeDeadlineSeconds", "backoffLimit"):
        if spec.get(f) is not None:
            errs += nonneg(spec[f], f"{p}.{f}")
    tpl = spec.get("template") or {}
    errs += validate_pod_template_spec(tpl, f"{p}.template")
    rp = (tpl.get("spec") or {}).get("restartPolicy")
    if rp not in ("OnFailure", "Never"):
        errs.append(not_supported(f"{p}.template.spec.restartPolicy", rp or "", ["OnFailure", "Never"]))
    return errs


def validate_job(j, old=None) -> list[str]:
    spec = j.get("spec") or {}
    md = j.get("metadata") or {}
    errs = _meta(j)
    if not spec.get("manualSelector") and spec.get("selector") is not None and md.get("uid"):
        # ValidateGeneratedSelector: a generated selector names this job's uid
        tl = _tpl_labels(spec)
        for k, want in (("controller-uid", md["uid"]), ("job-name", md.get("name", ""))):
            if k in tl and tl[k] != want:
                errs.append(invalid(f"spec.template.metadata.labels[{k}]", tl[k], f"must be '{want}'"))
    errs += _validate_job_spec(spec, "spec")
    if spec.get("selector") is not None:
        errs += validate_label_selector(spec["selector"], "spec.selector")
        sel = _selector(spec["selector"])
        if sel is not None and not sel.matches(_tpl_labels(spec)):
            errs.append(invalid("spec.template.metadata.labels", _go(_tpl_labels(spec)),
                                "`selector` does not match template `labels`"))
    if old is not None:
        ospec = old.get("spec") or {}
        for f in ("completions", "selector", "template"):
            if spec.get(f) != ospec.get(f) and ospec.get(f) is not None:
                errs.append(invalid(f"spec.{f}", _go(spec.get(f)), IMMUTABLE))
    return errs


def validate_job_status(st, p="status") -> list[str]:
    st = st or {}
    errs = []
    for f in ("active", "succeeded", "failed"):
        errs += nonneg(st.get(f, 0), f"{p}.{f}")
    return errs


def validate_cronjob(cj, old=None) -> list[str]:
    from ..controllers.apps import CronSchedule
    spec = cj.get("spec") or {}
    errs = _meta(cj)
    sched = spec.get("schedule") or ""
    if not sched:
        errs.append(required("spec.schedule"))
    else:
        try:
            CronSchedule(sched)
        except (ValueError, KeyError) as e:
            errs.append(invalid("spec.schedule", sched, str(e)))
    if spec.get("startingDeadlineSeconds") is not None:
        errs += nonneg(spec["startingDeadlineSeconds"], "spec.startingDeadlineSeconds")
    cp = spec.get("concurrencyPolicy") or ""
    if not cp:
        errs.append(required("spec.concurrencyPolicy"))
    elif cp not in ("Allow", "Forbid", "Replace"):
        errs.append(not_supported("spec.concurrencyPolicy", cp, ["Allow", "Forbid", "Replace"]))
    jt = (spec.get("jobTemplate") or {}).get("spec") or {}
    errs += _validate_job_spec(jt, "spec.jobTemplate.spec")
    if jt.get("selector") is not None:
        errs.append(invalid("spec.jobTemplate.spec.selector", _go(jt["selector"]), "`selector` will be auto-generated"))
    if jt.get("manualSelector"):
        errs.append(not_supported("spec.jobTemplate.spec.manualSelector", True, ["nil", "false"]))
    for f in ("successfulJobsHistoryLimit", "failedJobsHistoryLimit"):
        if spec.get(f) is not None:
            errs += nonneg(spec[f], f"spec.{f}")
    name = (cj.get("metadata") or {}).get("name") or ""
    if len(name) > 52:
        errs.append(invalid("metadata.name", name, "must be no more than 52 characters"))
    return errs


# ------------------------------------------------------------------ autoscaling
def validate_cross_version_object_reference(ref, p) -> list[str]:
    errs = []
    for f in ("kind", "name"):
        v = (ref or {}).get(f) or ""
        if not v:
            errs.append(required(f"{p}.{f}"))
        else:
            errs += [invalid(f"{p}.{f}", v, m) for m in is_valid_path_segment_name(v)]
    return errs


def _sign(v) -> int:
    try:
        f = Quantity(v).as_fraction()
    except (QuantityError, TypeError, ValueError):
        return 0
    return (f > 0) - (f < 0)


def validate_metric_spec(m, p) -> list[str]:
    errs = []
    t = m.get("type") or ""
    if not t:
        errs.append(required(f"{p}.type", "must specify a metric source type"))
    if t not in ("Object", "Pods", "Resource"):
        errs.append(not_supported(f"{p}.type", t, ["Object", "Pods", "Resource"]))
    present = []
    for key in ("object", "pods", "resource"):
        src = m.get(key)
        if src is None:
            continue
        present.append(key)
        if len(present) > 1:
            continue
        sp = f"{p}.{key}"
        if key == "object":
            errs += validate_cross_version_object_reference(src.get("target"), f"{sp}.target")
            if not src.get("metricName"):
                errs.append(required(f"{sp}.metricName", "must specify a metric name"))
            if _sign(src.get("targetValue", "0")) != 1:
                errs.append(required(f"{sp}.targetValue", "must specify a positive target value"))
        elif key == "pods":
            if not src.get("metricName"):
                errs.append(required(f"{sp}.metricName", "must specify a metric name"))
            if _sign(src.get("targetAverageValue", "0")) != 1:
                errs.append(required(f"{sp}.targetAverageValue", "must specify a positive target value"))
        else:
            util, val = src.get("targetAverageUtilization"), src.get("targetAverageValue")
            if not src.get("name"):
                errs.append(required(f"{sp}.name", "must specify a resource name"))
            if util is None and val is None:
                errs.append(required(f"{sp}.targetAverageUtilization", "must set either a target raw value or a target utilization"))
            if util is not None and (not is_int(util) or util < 1):
                errs.append(invalid(f"{sp}.targetAverageUtilization", util, "must be greater than 0"))
            if util is not None and val is not None:
                errs.append(forbidden(f"{sp}.targetAverageValue", "may not set both a target raw value and a target utilization"))
            if val is not None and _sign(val) != 1:
                errs.append(invalid(f"{sp}.targetAverageValue", val, "must be positive"))
    expected = t.lower()
    if expected not in present:
        errs.append(required(f"{p}.{expected}", "must populate information for the given metric source"))
    if len(present) != 1:
        for typ in present:
            if typ != expected:
                errs.append(forbidden(f"{p}.{typ}", "must populate the given metric source only"))
    return errs


def validate_hpa(hpa, old=None) -> list[str]:
    spec = hpa.get("spec") or {}
    errs = _meta(hpa)
    mn, mx = spec.get("minReplicas"), spec.get("maxReplicas", 0)
    if mn is not None and (not is_int(mn) or mn < 1):
        errs.append(invalid("spec.minReplicas", mn, "must be greater than 0"))
    if not is_int(mx) or mx < 1:
        errs.append(invalid("spec.maxReplicas", mx, "must be greater than 0"))
    if mn is not None and is_int(mn) and is_int(mx) and mx < mn:
        errs.append(invalid("spec.maxReplicas", mx, "must be greater than or equal to `minReplicas`"))
    errs += validate_cross_version_object_reference(spec.get("scaleTargetRef"), "spec.scaleTargetRef")
    cpu = spec.get("targetCPUUtilizationPercentage")
    if cpu is not None and (not is_int(cpu) or cpu < 1):
        # autoscaling/v1 → a Resource metric with targetAverageUtilization (conversion)
        errs.append(invalid("spec.metrics[0].resource.targetAverageUtilization", cpu, "must be greater than 0"))
    ann = (hpa.get("metadata") or {}).get("annotations") or {}
    raw = ann.get("autoscaling.alpha.kubernetes.io/metrics")
    if raw:
        try:
            metrics = json.loads(raw)
        except ValueError as e:
            errs.append(invalid("metadata.annotations[autoscaling.alpha.kubernetes.io/metrics]", raw, str(e)))
            metrics = []
        for i, mspec in enumerate(metrics or []):
            errs += validate_metric_spec(mspec or {}, f"spec.metrics[{i}]")
    return errs


# ------------------------------------------------------------------ policy
def validate_pdb(pdb, old=None) -> list[str]:
    spec = pdb.get("spec") or {}
    errs = _meta(pdb)
    mn, mu = spec.get("minAvailable"), spec.get("maxUnavailable")
    if mn is not None and mu is not None:
        errs.append(invalid("spec", _go(spec), "minAvailable and maxUnavailable cannot be both set"))
    for f, v in (("minAvailable", mn), ("maxUnavailable", mu)):
        if v is not None:
            errs += validate_positive_int_or_percent(v, f"spec.{f}") + not_more_than_100_percent(v, f"spec.{f}")
    errs += validate_label_selector(spec.get("selector"), "spec.selector")
    st = pdb.get("status") or {}
    for f in ("disruptionsAllowed", "currentHealthy", "desiredHealthy", "expectedPods"):
        errs += nonneg(st.get(f, 0), f"status.{'podDisruptionsAllowed' if f == 'disruptionsAllowed' else f}")
    if old is not None and spec != (old.get("spec") or {}):
        errs.append(forbidden("spec", "updates to poddisruptionbudget spec are forbidden."))
    return errs


# ------------------------------------------------------------------ storage
def validate_storage_class(sc, old=None) -> list[str]:
    errs = _meta(sc, namespaced=False)
    prov = sc.get("provisioner") or ""
    if not prov:
        errs.append(required("provisioner"))
    else:
        errs += [invalid("provisioner", prov, m) for m in is_qualified_name(prov.lower())]
    params = sc.get("parameters") or {}
    if len(params) > 512:
        errs.append(too_long("parameters", 512))
    else:
        total = 0
        for k, v in params.items():
            if not k:
                errs.append(invalid("parameters", k, "field can not be empty."))
            total += len(k) + len(str(v))
        if total > 256 * 1024:
            errs.append(too_long("parameters", 256 * 1024))
    rp = sc.get("reclaimPolicy") or ""
    if rp and rp not in ("Delete", "Retain"):
        errs.append(not_supported("reclaimPolicy", rp, ["Delete", "Retain"]))
    vbm = sc.get("volumeBindingMode")
    if vbm is not None and vbm not in ("Immediate", "WaitForFirstConsumer"):
        errs.append(not_supported("volumeBindingMode", vbm, ["Immediate", "WaitForFirstConsumer"]))
    if old is not None:
        if (old.get("parameters") or {}) != params:
            errs.append(forbidden("parameters", "updates to parameters are forbidden."))
        if prov != (old.get("provisioner") or ""):
            errs.append(forbidden("provisioner", "updates to provisioner are forbidden."))
        if (sc.get("reclaimPolicy") or "Delete") != (old.get("reclaimPolicy") or "Delete"):
            errs.append(forbidden("reclaimPolicy", "updates to reclaimPolicy are forbidden."))
        if vbm != old.get("volumeBindingMode"):
            errs.append(invalid("volumeBindingMode", vbm, IMMUTABLE))
    return errs


# ------------------------------------------------------------------ rbac
RBAC_GROUP = "rbac.authorization.k8s.io"


def _minimal_name(name: str) -> list[str]:
    return is_valid_path_segment_name(name)


def validate_policy_rule(rule, namespaced, p) -> list[str]:
    errs = []
    if not rule.get("verbs"):
        errs.append(required(f"{p}.verbs", "verbs must contain at least one value"))
    if rule.get("nonResourceURLs"):
        if namespaced:
            errs.append(invalid(f"{p}.nonResourceURLs", _go(rule["nonResourceURLs"]), "namespaced rules cannot apply to non-resource URLs"))
        if rule.get("apiGroups") or rule.get("resources") or rule.get("resourceNames"):
            errs.append(invalid(f"{p}.nonResourceURLs", _go(rule["nonResourceURLs"]),
                                "rules cannot apply to both regular resources and non-resource URLs"))
        return errs
    if not rule.get("apiGroups"):
        errs.append(required(f"{p}.apiGroups", "resource rules must supply at least one api group"))
    if not rule.get("resources"):
        errs.append(required(f"{p}.resources", "resource rules must supply at least one resource"))
    return errs


def _name_fn(name):
    return _minimal_name(name)


def validate_role(role, old=None, namespaced=True) -> list[str]:
    errs = _meta(role, namespaced, _name_fn)
    for i, r in enumerate(role.get("rules") or []):
        errs += validate_policy_rule(r, namespaced, f"rules[{i}]")
    agg = role.get("aggregationRule")
    if not namespaced and agg is not None:
        sels = agg.get("clusterRoleSelectors") or []
        if not sels:
            errs.append(required("aggregationRule.clusterRoleSelectors",
                                 "at least one clusterRoleSelector required if aggregationRule is non-nil"))
        for i, s in enumerate(sels):
            errs += validate_label_selector(s, f"aggregationRule.clusterRoleSelectors[{i}]")
    return errs


def validate_cluster_role(role, old=None) -> list[str]:
    return validate_role(role, old, namespaced=False)


def validate_subject(s, namespaced, p) -> list[str]:
    errs = []
    name, kind, group = s.get("name") or "", s.get("kind") or "", s.get("apiGroup") or ""
    if not name:
        errs.append(required(f"{p}.name"))
    if kind == "ServiceAccount":
        if name:
            errs += dns_subdomain(name, f"{p}.name")
        if group:
            errs.append(not_supported(f"{p}.apiGroup", group, [""]))
        if not namespaced and not s.get("namespace"):
            errs.append(required(f"{p}.namespace"))
    elif kind in ("User", "Group"):
        if not name:
            errs.append(invalid(f"{p}.name", name, f"{kind.lower()} name cannot be empty"))
        if group != RBAC_GROUP:
            errs.append(not_supported(f"{p}.apiGroup", group, [RBAC_GROUP]))
    else:
        errs.append(not_supported(f"{p}.kind", kind, ["ServiceAccount", "User", "Group"]))
    return errs


def validate_role_binding(rb, old=None, namespaced=True) -> list[str]:
    errs = _meta(rb, namespaced, _name_fn)
    ref = rb.get("roleRef") or {}
    if ref.get("apiGroup") != RBAC_GROUP:
        errs.append(not_supported("roleRef.apiGroup", ref.get("apiGroup") or "", [RBAC_GROUP]))
    kinds = ["Role", "ClusterRole"] if namespaced else ["ClusterRole"]
    if ref.get("kind") not in kinds:
        errs.append(not_supported("roleRef.kind", ref.get("kind") or "", kinds))
    if not ref.get("name"):
        errs.append(required("roleRef.name"))
    else:
        errs += [invalid("roleRef.name", ref["name"], m) for m in _minimal_name(ref["name"])]
    for i, s in enumerate(rb.get("subjects") or []):
        errs += validate_subject(s, namespaced, f"subjects[{i}]")
    if old is not None and (old.get("roleRef") or {}) != ref:
        errs.append(invalid("roleRef", _go(ref), "cannot change roleRef"))
    return errs


def validate_cluster_role_binding(rb, old=None) -> list[str]:
    return validate_role_binding(rb, old, namespaced=False)


# ------------------------------------------------------------------ scheduling
def validate_priority_class(pc, old=None) -> list[str]:
    errs = _meta(pc, namespaced=False)
    if old is not None and pc.get("value") != old.get("value"):
        errs.append(forbidden("Value", "may not be changed in an update."))
    return errs


def register():
    from .scheme import register_hooks
    for kind, gv, fn in (("StatefulSet", "apps/v1", validate_statefulset),
                         ("Deployment", "apps/v1", validate_deployment),
                         ("ReplicaSet", "apps/v1", validate_replicaset),
                         ("DaemonSet", "apps/v1", validate_daemonset),
                         ("ControllerRevision", "apps/v1", validate_controller_revision),
                         ("Job", "batch/v1", validate_job),
                         ("CronJob", "batch/v1beta1", validate_cronjob),
                         ("HorizontalPodAutoscaler", "autoscaling/v1", validate_hpa),
                         ("PodDisruptionBudget", "policy/v1beta1", validate_pdb),
                         ("StorageClass", "storage.k8s.io/v1", validate_storage_class),
                         ("Role", "rbac.authorization.k8s.io/v1", validate_role),
                         ("ClusterRole", "rbac.authorization.k8s.io/v1", validate_cluster_role),
                         ("RoleBinding", "rbac.authorization.k8s.io/v1", validate_role_binding),
                         ("ClusterRoleBinding", "rbac.authorization.k8s.io/v1", validate_cluster_role_binding),
                         ("PriorityClass", "scheduling.k8s.io/v1", validate_priority_class)):
        register_hooks(kind, gv, validator=fn)
