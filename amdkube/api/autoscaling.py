"""HorizontalPodAutoscaler autoscaling/v2beta1 ⇄ autoscaling/v1 (the storage version).

Reference: pkg/apis/autoscaling/v1/conversion.go + pkg/apis/autoscaling/annotations.go. v1 has
one metric (targetCPUUtilizationPercentage); everything v2beta1 adds rides in annotations on the
v1 object, exactly as the reference round-trips it:

  autoscaling.alpha.kubernetes.io/metrics          spec.metrics other than the CPU-utilization one
  autoscaling.alpha.kubernetes.io/current-metrics  status.currentMetrics other than CPU utilization
  autoscaling.alpha.kubernetes.io/conditions       status.conditions

The JSON inside the annotations is the v2beta1 MetricSpec / MetricStatus / condition shape.
"""
from __future__ import annotations

import json

METRICS_ANNOTATION = "autoscaling.alpha.kubernetes.io/metrics"
CURRENT_METRICS_ANNOTATION = "autoscaling.alpha.kubernetes.io/current-metrics"
CONDITIONS_ANNOTATION = "autoscaling.alpha.kubernetes.io/conditions"
STATUS_ANNOTATIONS = (CURRENT_METRICS_ANNOTATION, CONDITIONS_ANNOTATION)
DEFAULT_CPU_UTILIZATION = 80


def _is_cpu_util(ms: dict, spec: bool) -> bool:
    r = ms.get("resource") or {}
    key = "targetAverageUtilization" if spec else "currentAverageUtilization"
    return ms.get("type") == "Resource" and r.get("name") == "cpu" and r.get(key) is not None


def v2_to_v1(obj: dict) -> dict:
    """A v2beta1 HPA body → its autoscaling/v1 storage form (in place)."""
    spec = obj.setdefault("spec", {})
    ann = obj.setdefault("metadata", {}).setdefault("annotations", {}) or {}
    obj["metadata"]["annotations"] = ann
    metrics = spec.pop("metrics", None)
    spec.pop("targetCPUUtilizationPercentage", None)
    if metrics is not None:
        cpu = next((ms for ms in metrics if _is_cpu_util(ms, True)), None)
        rest = [ms for ms in metrics if ms is not cpu]
        if cpu is not None:
            spec["targetCPUUtilizationPercentage"] = int(cpu["resource"]["targetAverageUtilization"])
        if rest:
            ann[METRICS_ANNOTATION] = json.dumps(rest, separators=(",", ":"))
        else:
            ann.pop(METRICS_ANNOTATION, None)
    st = obj.get("status")
    if isinstance(st, dict):
        cur = st.pop("currentMetrics", None)
        conds = st.pop("conditions", None)
        if cur is not None:
            cpu = next((ms for ms in cur if _is_cpu_util(ms, False)), None)
            rest = [ms for ms in cur if ms is not cpu]
            if cpu is not None:
                st["currentCPUUtilizationPercentage"] = int(cpu["resource"]["currentAverageUtilization"])
            if rest:
                ann[CURRENT_METRICS_ANNOTATION] = json.dumps(rest, separators=(",", ":"))
            else:
                ann.pop(CURRENT_METRICS_ANNOTATION, None)
        if conds:
            ann[CONDITIONS_ANNOTATION] = json.dumps(conds, separators=(",", ":"))
    if not ann:
        obj["metadata"].pop("annotations", None)
    return obj


def v1_to_v2(obj: dict) -> dict:
    """The stored autoscaling/v1 HPA → the v2beta1 view (in place)."""
    md = obj.setdefault("metadata", {})
    ann = dict(md.get("annotations") or {})
    spec = obj.setdefault("spec", {})
    metrics = []
    cpu = spec.pop("targetCPUUtilizationPercentage", None)
    extra = _load(ann.pop(METRICS_ANNOTATION, None))
    if cpu is not None:
        metrics.append({"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": int(cpu)}})
    elif not extra:       # v1 defaulting: no metric at all means 80 % CPU
        metrics.append({"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": DEFAULT_CPU_UTILIZATION}})
    spec["metrics"] = metrics + extra
    st = obj.get("status")
    cur_extra = _load(ann.pop(CURRENT_METRICS_ANNOTATION, None))
    conds = _load(ann.pop(CONDITIONS_ANNOTATION, None))
    if isinstance(st, dict):
        cur = []
        cpu_now = st.pop("currentCPUUtilizationPercentage", None)
        if cpu_now is not None:
            cur.append({"type": "Resource", "resource": {"name": "cpu", "currentAverageUtilization": int(cpu_now)}})
        st["currentMetrics"] = cur + cur_extra or None
        if st["currentMetrics"] is None:
            st.pop("currentMetrics")
        if conds:
            st["conditions"] = conds
    if ann:
        md["annotations"] = ann
    else:
        md.pop("annotations", None)
    return obj


def metrics_of(hpa_v1: dict) -> list[dict]:
    """spec.metrics of a stored (v1) HPA, for controllers that read the storage version."""
    return v1_to_v2(json.loads(json.dumps(hpa_v1)))["spec"]["metrics"]


def _load(s):
    if not s:
        return []
    try:
        v = json.loads(s)
        return v if isinstance(v, list) else []
    except ValueError:
        return []
