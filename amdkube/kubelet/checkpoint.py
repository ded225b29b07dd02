"""Bootstrap pod checkpoints: the reference's pkg/kubelet/checkpoint (alpha,
--bootstrap-checkpoint-path). Pods annotated `node.kubernetes.io/bootstrap-checkpoint: "true"`
(self-hosted control-plane pods) are written to `<path>/Pod_<uid>.yaml` whenever the kubelet
learns of them from the API server and removed when they are deleted; a kubelet that restarts
without an API server (the apiserver may be one of those pods) loads them as pods to run, and
they are reconciled with the API server's view once it is reachable (kubelet.go
HandlePodAdditions: "pods restored from the checkpoint. Treat them as new").
"""
from __future__ import annotations

import glob
import json
import logging
import os

log = logging.getLogger("amdkube.kubelet.checkpoint")

BOOTSTRAP_CHECKPOINT_ANNOTATION = "node.kubernetes.io/bootstrap-checkpoint"
POD_PREFIX = "Pod_"


class PodCheckpointManager:
    def __init__(self, path: str):
        self.path = path
        os.makedirs(path, exist_ok=True)

    @staticmethod
    def wants(pod: dict) -> bool:
        return ((pod.get("metadata") or {}).get("annotations") or {}).get(BOOTSTRAP_CHECKPOINT_ANNOTATION) == "true"

    def _file(self, pod: dict) -> str:
        return os.path.join(self.path, f"{POD_PREFIX}{pod['metadata']['uid']}.yaml")

    def write_pod(self, pod: dict) -> bool:
        """Checkpoint an annotated pod; a pod that no longer carries the annotation loses its
        checkpoint (it must not be restored from a stale copy). I/O errors are logged, never
        raised into the informer handler."""
        if not self.wants(pod):
            self.delete_pod(pod)
            return False
        p = self._file(pod)
        body = {k: v for k, v in pod.items() if k != "status"}   # the spec is what restarts it
        tmp = p + ".tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(body, f)        # JSON is YAML; the reference writes the same encoding
            os.replace(tmp, p)
        except OSError as e:
            log.error("writing bootstrap checkpoint %s: %s", p, e)
            return False
        return True

    def delete_pod(self, pod: dict):
        try:
            os.unlink(self._file(pod))
        except FileNotFoundError:
            pass
        except OSError as e:
            log.error("removing bootstrap checkpoint %s: %s", self._file(pod), e)

    def load_pods(self) -> list[dict]:
        out = []
        for f in sorted(glob.glob(os.path.join(self.path, POD_PREFIX + "*.yaml"))):
            try:
                with open(f) as fh:
                    pod = json.load(fh)
            except (OSError, ValueError) as e:
                log.warning("skipping unreadable pod checkpoint %s: %s", f, e)
                continue
            if self.wants(pod) and (pod.get("metadata") or {}).get("uid"):
                out.append(pod)
        return out
