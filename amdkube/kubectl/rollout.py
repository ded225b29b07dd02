"""kubectl rollout status viewers.

Reference: pkg/kubectl/rollout_status.go — DeploymentStatusViewer (:55-92), DaemonSetStatusViewer
(:95-118) and StatefulSetStatusViewer (:121-156). Each returns (message, done) or raises
StatusError; `kubectl rollout status` prints the message and, with --watch, repeats until done.
Quirks kept: a StatefulSet with a rollingUpdate block (apps/v1beta2 and later default one with
partition 0) reports "partitioned roll out complete" once its pods are ready; the revision
comparison only exists without that block; OnDelete is an error that also ends the watch.
"""
from __future__ import annotations


class StatusError(Exception):
    def __init__(self, msg: str, done: bool = False):
        super().__init__(msg)
        self.done = done


def _revision(obj) -> int:
    v = ((obj.get("metadata") or {}).get("annotations") or {}).get("deployment.kubernetes.io/revision", "0")
    try:
        return int(v)
    except ValueError:
        raise StatusError(f'cannot get the revision of deployment "{(obj.get("metadata") or {}).get("name", "")}": '
                          f'strconv.ParseInt: parsing "{v}": invalid syntax') from None


def deployment_status(d: dict, name: str, revision: int = 0) -> tuple[str, bool]:
    spec, st = d.get("spec") or {}, d.get("status") or {}
    if revision > 0:
        have = _revision(d)
        if revision != have:
            raise StatusError(f"desired revision ({revision}) is different from the running revision ({have})")
    gen = int((d.get("metadata") or {}).get("generation") or 0)
    if gen <= int(st.get("observedGeneration") or 0):
        prog = next((c for c in st.get("conditions") or [] if c.get("type") == "Progressing"), None)
        if prog is not None and prog.get("reason") == "ProgressDeadlineExceeded":
            raise StatusError(f'deployment "{name}" exceeded its progress deadline')
        upd = int(st.get("updatedReplicas") or 0)
        if spec.get("replicas") is not None and upd < int(spec["replicas"]):
            return f"Waiting for rollout to finish: {upd} out of {int(spec['replicas'])} new replicas have been updated...\n", False
        if int(st.get("replicas") or 0) > upd:
            return f"Waiting for rollout to finish: {int(st.get('replicas') or 0) - upd} old replicas are pending termination...\n", False
        av = int(st.get("availableReplicas") or 0)
        if av < upd:
            return f"Waiting for rollout to finish: {av} of {upd} updated replicas are available...\n", False
        return f'deployment "{name}" successfully rolled out\n', True
    return "Waiting for deployment spec update to be observed...\n", False


def daemonset_status(ds: dict, name: str) -> tuple[str, bool]:
    spec, st = ds.get("spec") or {}, ds.get("status") or {}
    if ((spec.get("updateStrategy") or {}).get("type") or "OnDelete") != "RollingUpdate":
        raise StatusError("Status is available only for RollingUpdate strategy type", done=True)
    gen = int((ds.get("metadata") or {}).get("generation") or 0)
    if gen <= int(st.get("observedGeneration") or 0):
        want, upd, av = (int(st.get(k) or 0) for k in ("desiredNumberScheduled", "updatedNumberScheduled", "numberAvailable"))
        if upd < want:
            return f"Waiting for rollout to finish: {upd} out of {want} new pods have been updated...\n", False
        if av < want:
            return f"Waiting for rollout to finish: {av} of {want} updated pods are available...\n", False
        return f'daemon set "{name}" successfully rolled out\n', True
    return "Waiting for daemon set spec update to be observed...\n", False


def statefulset_status(sts: dict, name: str) -> tuple[str, bool]:
    spec, st = sts.get("spec") or {}, sts.get("status") or {}
    strategy = spec.get("updateStrategy") or {}
    if strategy.get("type") == "OnDelete":
        raise StatusError("OnDelete updateStrategy does not have a Status`", done=True)
    gen = int((sts.get("metadata") or {}).get("generation") or 0)
    if st.get("observedGeneration") is None or gen > int(st["observedGeneration"]):
        return "Waiting for statefulset spec update to be observed...\n", False
    replicas = spec.get("replicas")
    ready = int(st.get("readyReplicas") or 0)
    if replicas is not None and ready < int(replicas):
        return f"Waiting for {int(replicas) - ready} pods to be ready...\n", False
    upd = int(st.get("updatedReplicas") or 0)
    if strategy.get("type") == "RollingUpdate" and strategy.get("rollingUpdate") is not None:
        part = strategy["rollingUpdate"].get("partition")
        if replicas is not None and part is not None and upd < int(replicas) - int(part):
            return (f"Waiting for partitioned roll out to finish: {upd} out of {int(replicas) - int(part)} new pods have been "
                    f"updated...\n"), False
        return f"partitioned roll out complete: {upd} new pods have been updated...\n", True
    if st.get("updateRevision") != st.get("currentRevision"):
        return f"waiting for statefulset rolling update to complete {upd} pods at revision {st.get('updateRevision')}...\n", False
    return (f"statefulset rolling update complete {int(st.get('currentReplicas') or 0)} pods at revision "
            f"{st.get('currentRevision')}...\n"), True


VIEWERS = {"Deployment": deployment_status, "DaemonSet": daemonset_status, "StatefulSet": statefulset_status}
