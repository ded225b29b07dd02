"""Controller listers the spreading priorities read: the Services, ReplicationControllers,
ReplicaSets and StatefulSets whose selectors pick a pod.

Reference: plugin/pkg/scheduler/algorithm/priorities/metadata.go:69-96 (getSelectors) over the
client-go listers' GetPodServices / GetPodControllers / GetPodReplicaSets / GetPodStatefulSets
(staging/src/k8s.io/client-go/listers/core/v1/service_expansion.go:36,
replicationcontroller_expansion.go, extensions/v1beta1/replicaset_expansion.go,
apps/v1beta1/statefulset_expansion.go): same namespace only; a Service without a selector, or a
controller whose selector is nil or empty, selects nothing (never everything); a pod without
labels has no controller.

Each lister is a zero-argument callable returning the current objects (an informer's `list`).
The scheduler computes a pod's selectors once per scheduling attempt (PodInfo caches them).
"""
from __future__ import annotations

from ..api import meta as m
from ..api.labels import SelectorError, selector_from_label_selector, selector_from_set


def _ns(obj) -> str:
    return (obj.get("metadata") or {}).get("namespace") or ""


class ControllerListers:
    __slots__ = ("services", "rcs", "rss", "sss")

    def __init__(self, services=None, rcs=None, rss=None, sss=None):
        self.services = services or list
        self.rcs = rcs or list
        self.rss = rss or list
        self.sss = sss or list

    def selectors(self, pod: dict, services_only: bool = False) -> list:
        """The label selectors of every Service/RC/RS/StatefulSet in the pod's namespace that
        selects the pod (metadata.go getSelectors)."""
        ns = _ns(pod)
        labels = m.labels_of(pod)
        out = []
        for s in self.services():
            sel = (s.get("spec") or {}).get("selector")
            if _ns(s) == ns and sel:
                ss = selector_from_set(sel)
                if ss.matches(labels):
                    out.append(ss)
        if services_only or not labels:
            return out
        for rc in self.rcs():
            sel = (rc.get("spec") or {}).get("selector")
            if _ns(rc) == ns and sel:
                ss = selector_from_set(sel)
                if ss.matches(labels):
                    out.append(ss)
        for lister in (self.rss, self.sss):
            for obj in lister():
                if _ns(obj) != ns:
                    continue
                raw = (obj.get("spec") or {}).get("selector")
                if not raw or not (raw.get("matchLabels") or raw.get("matchExpressions")):
                    continue
                try:
                    ss = selector_from_label_selector(raw)
                except SelectorError:
                    continue
                if ss.matches(labels):
                    out.append(ss)
        return out


NO_LISTERS = ControllerListers()
