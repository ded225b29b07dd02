"""Deployment controller (pkg/controller/deployment/*.go, util/deployment_util.go).

syncDeployment (deployment_controller.go:561-648): claim the ReplicaSets (adopt matching
orphans, release the ones that stop matching), map pods to them by ControllerRef, then
  * being deleted -> status only;
  * checkPausedConditions; paused -> sync (scale only, cleanup, status);
  * spec.rollbackTo -> rollback (rollback.go);
  * a scaling event (an active RS's desired-replicas annotation differs from spec.replicas) ->
    sync: proportional scaling over the active ReplicaSets (sync.go scale: the extra / missing
    replicas are spread by each RS's share of the max-replicas annotation, the rounding
    leftover going to the largest);
  * Recreate (recreate.go): old ReplicaSets to 0, wait for their pods to be gone, then the new
    one to spec.replicas;
  * RollingUpdate (rolling.go): reconcileNewReplicaSet (scale up within maxSurge), then
    reconcileOldReplicaSets (clean up unhealthy old replicas first, then scale old ones down
    while availability stays >= replicas - maxUnavailable).
The new ReplicaSet is the oldest whose template equals the deployment's ignoring
pod-template-hash; creating it takes revision max(old)+1, the deployment's annotations, and the
desired/max-replicas annotations; a name collision with a different template bumps
status.collisionCount. Status and the Progressing / Available / ReplicaFailure conditions with
progressDeadlineSeconds follow progress.go (a stuck rollout is requeued for its deadline);
revisionHistoryLimit old ReplicaSets are kept (cleanupDeployment).

Writes go through `self.client` (update / create / delete / update status); the template hash is
an FNV-32a of the canonical JSON of the template plus the collision count (the reference hashes
its Go struct dump, so hash values differ; names are `<deployment>-<SafeEncodeString(hash)>`).
"""
from __future__ import annotations

import json
import math
import time

from ..api import meta as m
from ..api.labels import selector_from_label_selector
from .base import Controller, split_key
from .controller_utils import (ControllerRefManager, adopt_patch, by_creation_timestamp, filter_active_replica_sets,
                               recheck_deletion, release_patch, rs_replicas, sort_by_size_newer, sort_by_size_older)

REVISION = "deployment.kubernetes.io/revision"
REVISION_HISTORY = "deployment.kubernetes.io/revision-history"
DESIRED = "deployment.kubernetes.io/desired-replicas"
MAX_REPLICAS = "deployment.kubernetes.io/max-replicas"
HASH_LABEL = "pod-template-hash"
LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"

ROLLBACK_REVISION_NOT_FOUND = "DeploymentRollbackRevisionNotFound"
ROLLBACK_TEMPLATE_UNCHANGED = "DeploymentRollbackTemplateUnchanged"
ROLLBACK_DONE = "DeploymentRollback"
RS_UPDATED = "ReplicaSetUpdated"
FAILED_RS_CREATE = "ReplicaSetCreateError"
NEW_RS_CREATED = "NewReplicaSetCreated"
FOUND_NEW_RS = "FoundNewReplicaSet"
NEW_RS_AVAILABLE = "NewReplicaSetAvailable"
TIMED_OUT = "ProgressDeadlineExceeded"
PAUSED = "DeploymentPaused"
RESUMED = "DeploymentResumed"
MIN_AVAILABLE = "MinimumReplicasAvailable"
MIN_UNAVAILABLE = "MinimumReplicasUnavailable"

ANNOTATIONS_TO_SKIP = {LAST_APPLIED, REVISION, REVISION_HISTORY, DESIRED, MAX_REPLICAS}


# ============================================================================ util
def int_or_percent(v, total: int, round_up: bool) -> int:
    """intstr.GetValueFromIntOrPercent."""
    if v is None:
        return 0
    if isinstance(v, bool):
        raise ValueError(f"invalid value {v!r}")
    if isinstance(v, int):
        return v
    s = str(v)
    if not s.endswith("%"):
        raise ValueError(f"invalid value for IntOrString: invalid value {s!r}: must be an integer or percentage")
    try:
        pct = int(s[:-1])
    except ValueError:
        raise ValueError(f"invalid value for IntOrString: invalid value {s!r}") from None
    f = pct * total / 100.0
    return int(math.ceil(f) if round_up else math.floor(f))


def resolve_fenceposts(max_surge, max_unavailable, desired: int) -> tuple[int, int]:
    """ResolveFenceposts: surge rounds up, unavailable down; both zero means one unavailable."""
    surge = int_or_percent(max_surge, desired, True)
    unavailable = int_or_percent(max_unavailable, desired, False)
    if surge == 0 and unavailable == 0:
        unavailable = 1
    return surge, unavailable


def spec_of(o) -> dict:
    return (o or {}).get("spec") or {}


def status_of(o) -> dict:
    return (o or {}).get("status") or {}


def d_replicas(d) -> int:
    return int(spec_of(d).get("replicas", 1))


def is_rolling_update(d) -> bool:
    return ((spec_of(d).get("strategy") or {}).get("type") or "RollingUpdate") == "RollingUpdate"


def _rolling(d) -> dict:
    return (spec_of(d).get("strategy") or {}).get("rollingUpdate") or {}


def max_unavailable(d) -> int:
    if not is_rolling_update(d) or d_replicas(d) == 0:
        return 0
    ru = _rolling(d)
    _, unavailable = resolve_fenceposts(ru.get("maxSurge", "25%"), ru.get("maxUnavailable", "25%"), d_replicas(d))
    return min(unavailable, d_replicas(d))


def min_available(d) -> int:
    if not is_rolling_update(d):
        return 0
    return d_replicas(d) - max_unavailable(d)


def max_surge(d) -> int:
    if not is_rolling_update(d):
        return 0
    ru = _rolling(d)
    return resolve_fenceposts(ru.get("maxSurge", "25%"), ru.get("maxUnavailable", "25%"), d_replicas(d))[0]


def annotations_of(o) -> dict:
    """The object's annotations map, created in place when missing."""
    md = o.setdefault("metadata", {})
    if md.get("annotations") is None:
        md["annotations"] = {}
    return md["annotations"]


def revision(o) -> int:
    v = (((o or {}).get("metadata") or {}).get("annotations") or {}).get(REVISION)
    if v is None:
        return 0
    return int(v)


def _safe_revision(o):
    try:
        return revision(o)
    except ValueError:
        return None


def max_revision(rss) -> int:
    return max([v for v in (_safe_revision(r) for r in rss if r is not None) if v is not None] or [0])


def last_revision(rss) -> int:
    """The second-highest revision (the one a rollback with revision 0 goes to)."""
    mx = sec = 0
    for r in rss:
        if r is None:
            continue
        v = _safe_revision(r)
        if v is None:
            continue
        if v >= mx:
            sec, mx = mx, v
        elif v > sec:
            sec = v
    return sec


def set_deployment_revision(d, rev: str) -> bool:
    ann = annotations_of(d)
    if ann.get(REVISION) != rev:
        ann[REVISION] = rev
        return True
    return False


def copy_deployment_annotations_to_rs(d, rs) -> bool:
    ann = annotations_of(rs)
    changed = False
    for k, v in ((d.get("metadata") or {}).get("annotations") or {}).items():
        if k in ANNOTATIONS_TO_SKIP or ann.get(k) == v:
            continue
        ann[k] = v
        changed = True
    return changed


def set_replicas_annotations(rs, desired: int, maximum: int) -> bool:
    ann = annotations_of(rs)
    changed = False
    for k, v in ((DESIRED, str(desired)), (MAX_REPLICAS, str(maximum))):
        if ann.get(k) != v:
            ann[k] = v
            changed = True
    return changed


def set_new_rs_annotations(d, rs, new_revision: str, exists: bool) -> bool:
    """SetNewReplicaSetAnnotations (deployment_util.go:245-305)."""
    changed = copy_deployment_annotations_to_rs(d, rs)
    ann = annotations_of(rs)
    old = ann.get(REVISION)
    had = REVISION in ann
    try:
        old_int = int(old) if old not in (None, "") else 0
    except ValueError:
        return False
    try:
        new_int = int(new_revision)
    except ValueError:
        return False
    if old_int < new_int:
        ann[REVISION] = new_revision
        changed = True
    if had and changed:
        hist = ann.get(REVISION_HISTORY, "")
        ann[REVISION_HISTORY] = old if not hist else hist + "," + old
    if not exists and set_replicas_annotations(rs, d_replicas(d), d_replicas(d) + max_surge(d)):
        changed = True
    return changed


def set_deployment_annotations_to(d, rollback_rs):
    """The deployment keeps only its skipped annotations and takes the others from the RS."""
    md = d.setdefault("metadata", {})
    kept = {k: v for k, v in (md.get("annotations") or {}).items() if k in ANNOTATIONS_TO_SKIP}
    for k, v in ((rollback_rs.get("metadata") or {}).get("annotations") or {}).items():
        if k not in ANNOTATIONS_TO_SKIP:
            kept[k] = v
    md["annotations"] = kept


def get_int_annotation(rs, key) -> tuple[int, bool]:
    v = (((rs or {}).get("metadata") or {}).get("annotations") or {}).get(key)
    if v is None:
        return 0, False
    try:
        return int(v), True
    except ValueError:
        return 0, False


def find_active_or_latest(new_rs, old_rss):
    if new_rs is None and not old_rss:
        return None
    olds = sorted(old_rss, key=by_creation_timestamp, reverse=True)
    active = filter_active_replica_sets(olds + [new_rs])
    if not active:
        return new_rs if new_rs is not None else olds[0]
    if len(active) == 1:
        return active[0]
    return None


def rs_fraction(rs, d) -> int:
    """getReplicaSetFraction: the change that keeps this RS's share of the annotated total."""
    if d_replicas(d) == 0:
        return -rs_replicas(rs)
    deployment_replicas = d_replicas(d) + max_surge(d)
    annotated, ok = get_int_annotation(rs, MAX_REPLICAS)
    if not ok:
        annotated = int(status_of(d).get("replicas") or 0)
    new_size = float(rs_replicas(rs) * deployment_replicas) / float(annotated) if annotated else 0.0
    rounded = int(new_size - 0.5) if new_size < 0 else int(new_size + 0.5)
    return rounded - rs_replicas(rs)


def get_proportion(rs, d, to_add: int, added: int) -> int:
    if rs is None or rs_replicas(rs) == 0 or to_add == 0 or to_add == added:
        return 0
    fraction = rs_fraction(rs, d)
    allowed = to_add - added
    return min(fraction, allowed) if to_add > 0 else max(fraction, allowed)


def _template_sans_hash(t):
    t = json.loads(json.dumps(t or {}))
    md = t.setdefault("metadata", {})
    (md.get("labels") or {}).pop(HASH_LABEL, None)
    if not md.get("labels"):
        md.pop("labels", None)
    if not md:
        t.pop("metadata", None)
    return t


def _prune(v):
    """Drop null / empty maps and lists: apiequality.Semantic holds nil and empty alike."""
    if isinstance(v, dict):
        out = {k: _prune(x) for k, x in v.items()}
        return {k: x for k, x in out.items() if x is not None and x != {} and x != []}
    if isinstance(v, list):
        return [_prune(x) for x in v]
    return v


def equal_ignore_hash(t1, t2) -> bool:
    """EqualIgnoreHash: the labels agree except pod-template-hash, and the rest is equal."""
    l1 = ((t1 or {}).get("metadata") or {}).get("labels") or {}
    l2 = ((t2 or {}).get("metadata") or {}).get("labels") or {}
    if len(l1) > len(l2):
        l1, l2 = l2, l1
    for k, v in l2.items():
        if l1.get(k) != v and k != HASH_LABEL:
            return False

    def strip(t):
        t = json.loads(json.dumps(t or {}))
        md = t.get("metadata") or {}
        md.pop("labels", None)
        if not md:
            t.pop("metadata", None)
        return _prune(t)
    return strip(t1) == strip(t2)


def find_new_rs(d, rss):
    for rs in sorted([r for r in rss if r is not None], key=by_creation_timestamp):
        if equal_ignore_hash(spec_of(rs).get("template"), spec_of(d).get("template")):
            return rs
    return None


def find_old_rss(d, rss) -> tuple[list, list]:
    new = find_new_rs(d, rss)
    required, all_old = [], []
    for rs in rss:
        if new is not None and m.uid_of(rs) == m.uid_of(new):
            continue
        all_old.append(rs)
        if rs_replicas(rs) != 0:
            required.append(rs)
    return required, all_old


def replica_count(rss) -> int:
    return sum(rs_replicas(r) for r in rss if r is not None)


def _status_sum(rss, k) -> int:
    return sum(int(status_of(r).get(k) or 0) for r in rss if r is not None)


def actual_replica_count(rss) -> int:
    return _status_sum(rss, "replicas")


def ready_replica_count(rss) -> int:
    return _status_sum(rss, "readyReplicas")


def available_replica_count(rss) -> int:
    return _status_sum(rss, "availableReplicas")


def deployment_complete(d, status) -> bool:
    want = d_replicas(d)
    return int(status.get("updatedReplicas") or 0) == want and int(status.get("replicas") or 0) == want and \
        int(status.get("availableReplicas") or 0) == want and \
        int(status.get("observedGeneration") or 0) >= int((d.get("metadata") or {}).get("generation") or 0)


def deployment_progressing(d, new) -> bool:
    old = status_of(d)
    old_old = int(old.get("replicas") or 0) - int(old.get("updatedReplicas") or 0)
    new_old = int(new.get("replicas") or 0) - int(new.get("updatedReplicas") or 0)
    return int(new.get("updatedReplicas") or 0) > int(old.get("updatedReplicas") or 0) or new_old < old_old or \
        int(new.get("readyReplicas") or 0) > int(old.get("readyReplicas") or 0) or \
        int(new.get("availableReplicas") or 0) > int(old.get("availableReplicas") or 0)


def deployment_timed_out(d, status, now: float) -> bool:
    deadline = spec_of(d).get("progressDeadlineSeconds")
    if deadline is None:
        return False
    cond = get_condition(status, "Progressing")
    if cond is None or cond.get("reason") == NEW_RS_AVAILABLE:
        return False
    if cond.get("reason") == TIMED_OUT:
        return True
    frm = m.parse_time(cond.get("lastUpdateTime")) or 0.0
    return frm + int(deadline) < now


def new_rs_new_replicas(d, all_rss, new_rs) -> int:
    strategy = (spec_of(d).get("strategy") or {}).get("type") or "RollingUpdate"
    if strategy == "RollingUpdate":
        surge = int_or_percent(_rolling(d).get("maxSurge", "25%"), d_replicas(d), True)
        current = replica_count(all_rss)
        max_total = d_replicas(d) + surge
        if current >= max_total:
            return rs_replicas(new_rs)
        up = min(max_total - current, d_replicas(d) - rs_replicas(new_rs))
        return rs_replicas(new_rs) + up
    if strategy == "Recreate":
        return d_replicas(d)
    raise ValueError(f"deployment type {strategy} isn't supported")


def is_saturated(d, rs) -> bool:
    if rs is None:
        return False
    desired, ok = get_int_annotation(rs, DESIRED)
    if not ok:
        return False
    return rs_replicas(rs) == d_replicas(d) and desired == d_replicas(d) and \
        int(status_of(rs).get("availableReplicas") or 0) == d_replicas(d)


# ---------------------------------------------------------------------------- conditions
def new_condition(kind, status, reason, message, now: float | None = None) -> dict:
    t = m.format_time(time.time() if now is None else now)
    return {"type": kind, "status": status, "lastUpdateTime": t, "lastTransitionTime": t, "reason": reason,
            "message": message}


def get_condition(status, kind):
    for c in (status or {}).get("conditions") or []:
        if c.get("type") == kind:
            return c
    return None


def set_condition(status, cond):
    cur = get_condition(status, cond["type"])
    if cur is not None and cur.get("status") == cond["status"] and cur.get("reason") == cond.get("reason"):
        return
    if cur is not None and cur.get("status") == cond["status"]:
        cond = dict(cond, lastTransitionTime=cur.get("lastTransitionTime"))
    status["conditions"] = [c for c in status.get("conditions") or [] if c.get("type") != cond["type"]] + [cond]


def remove_condition(status, kind):
    conds = [c for c in status.get("conditions") or [] if c.get("type") != kind]
    if conds:
        status["conditions"] = conds
    else:
        status.pop("conditions", None)


def rs_to_deployment_condition(c) -> dict:
    return {"type": c.get("type"), "status": c.get("status"), "lastTransitionTime": c.get("lastTransitionTime"),
            "lastUpdateTime": c.get("lastTransitionTime"), "reason": c.get("reason"), "message": c.get("message")}


def calculate_status(all_rss, new_rs, d, now: float | None = None) -> dict:
    """calculateStatus (sync.go)."""
    available = available_replica_count(all_rss)
    total = replica_count(all_rss)
    status = {"observedGeneration": (d.get("metadata") or {}).get("generation", 0),
              "replicas": actual_replica_count(all_rss),
              "updatedReplicas": actual_replica_count([new_rs]),
              "readyReplicas": ready_replica_count(all_rss),
              "availableReplicas": available,
              "unavailableReplicas": max(0, total - available)}
    cc = status_of(d).get("collisionCount")
    if cc is not None:
        status["collisionCount"] = cc
    conds = [dict(c) for c in status_of(d).get("conditions") or []]
    if conds:
        status["conditions"] = conds
    if available >= d_replicas(d) - max_unavailable(d):
        set_condition(status, new_condition("Available", "True", MIN_AVAILABLE, "Deployment has minimum availability.", now))
    else:
        set_condition(status, new_condition("Available", "False", MIN_UNAVAILABLE,
                                            "Deployment does not have minimum availability.", now))
    return status


_SAFE = "bcdfghjklmnpqrstvwxz2456789"


def safe_encode(s: str) -> str:
    """rand.SafeEncodeString: every character mapped into an alphabet without vowels."""
    return "".join(_SAFE[ord(c) % len(_SAFE)] for c in s)


def compute_hash(template: dict, collision_count: int | None) -> str:
    """FNV-32a of the canonical JSON of the template (+ the collision count), in decimal."""
    h = 0x811C9DC5
    data = json.dumps(template or {}, sort_keys=True, separators=(",", ":")).encode()
    if collision_count is not None:
        data += int(collision_count).to_bytes(4, "little", signed=False)
    for b in data:
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return str(h)


def status_changed(a: dict, b: dict) -> bool:
    return json.dumps(a or {}, sort_keys=True) != json.dumps(b or {}, sort_keys=True)


# ============================================================================ controller
class DeploymentController(Controller):
    name = "deployment"
    workers = 5

    def __init__(self, mgr, clock=time.time):
        super().__init__(mgr)
        self.clock = clock

    # ------------------------------------------------------------------ informers
    def setup(self):
        f = self.mgr.factory
        self.d_inf = f.informer("deployments")
        self.rs_inf = f.informer("replicasets")
        self.pod_inf = self.mgr.pods
        self.d_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.rs_inf.add_handler(on_add=self.add_rs, on_update=self.update_rs, on_delete=self.delete_rs)
        self.pod_inf.add_handler(on_delete=self.delete_pod)

    def _event(self, obj, etype, reason, msg):
        rec = getattr(self.mgr, "recorder", None)
        if rec is not None:
            rec.event(obj, etype, reason, msg)

    def _resolve(self, ns, ref):
        if ref.get("kind") != "Deployment":
            return None
        d = self.d_inf.get(f"{ns}/{ref.get('name')}")
        if d is None or m.uid_of(d) != ref.get("uid"):
            return None
        return d

    def deployments_for_rs(self, rs) -> list:
        """getDeploymentsForReplicaSet: deployments of the namespace whose selector matches."""
        out = []
        for d in self.d_inf.list():
            if m.namespace_of(d) != m.namespace_of(rs):
                continue
            try:
                sel = selector_from_label_selector(spec_of(d).get("selector"))
            except Exception:
                continue
            if sel.empty() or not sel.matches(m.labels_of(rs)):
                continue
            out.append(d)
        return out

    def add_rs(self, rs):
        if (rs.get("metadata") or {}).get("deletionTimestamp"):
            self.delete_rs(rs)
            return
        ref = m.controller_ref(rs)
        if ref is not None:
            d = self._resolve(m.namespace_of(rs), ref)
            if d is not None:
                self.enqueue(d)
            return
        for d in self.deployments_for_rs(rs):
            self.enqueue(d)

    def update_rs(self, old, cur):
        if (old.get("metadata") or {}).get("resourceVersion") == (cur.get("metadata") or {}).get("resourceVersion"):
            return
        cur_ref, old_ref = m.controller_ref(cur), m.controller_ref(old)
        changed = cur_ref != old_ref
        if changed and old_ref is not None:
            d = self._resolve(m.namespace_of(old), old_ref)
            if d is not None:
                self.enqueue(d)
        if cur_ref is not None:
            d = self._resolve(m.namespace_of(cur), cur_ref)
            if d is not None:
                self.enqueue(d)
            return
        if changed or m.labels_of(old) != m.labels_of(cur):
            for d in self.deployments_for_rs(cur):
                self.enqueue(d)

    def delete_rs(self, rs):
        ref = m.controller_ref(rs)
        if ref is None:
            return
        d = self._resolve(m.namespace_of(rs), ref)
        if d is not None:
            self.enqueue(d)

    def delete_pod(self, pod):
        """A Recreate deployment waits for its old pods; enqueue it when the last is gone."""
        ref = m.controller_ref(pod)
        if ref is None or ref.get("kind") != "ReplicaSet":
            return
        rs = self.rs_inf.get(f"{m.namespace_of(pod)}/{ref.get('name')}")
        if rs is None or m.uid_of(rs) != ref.get("uid"):
            return
        d_ref = m.controller_ref(rs)
        d = self._resolve(m.namespace_of(rs), d_ref) if d_ref else None
        if d is None or (spec_of(d).get("strategy") or {}).get("type") != "Recreate":
            return
        rss = [r for r in self.rs_inf.list() if (m.controller_ref(r) or {}).get("uid") == m.uid_of(d)]
        pod_map = self.pod_map(d, rss)
        if sum(len(v) for v in pod_map.values()) == 0:
            self.enqueue(d)

    # ------------------------------------------------------------------ claiming
    async def replica_sets_for(self, d) -> list:
        """getReplicaSetsForDeployment: claim the namespace's ReplicaSets."""
        sel = selector_from_label_selector(spec_of(d).get("selector"))
        rss = [r for r in self.rs_inf.list() if m.namespace_of(r) == m.namespace_of(d)]
        client = self.client

        async def fresh():
            f = await client.get("deployments", m.name_of(d), m.namespace_of(d))
            if m.uid_of(f) != m.uid_of(d):
                raise RuntimeError(f"original Deployment {m.key_of(d)} is gone")
            return f

        async def adopt(rs):
            await client.patch("replicasets", m.name_of(rs), adopt_patch(d, "apps/v1", "Deployment", rs),
                               m.namespace_of(rs), patch_type="application/strategic-merge-patch+json")

        async def release(rs):
            await client.patch("replicasets", m.name_of(rs), release_patch(d, rs), m.namespace_of(rs),
                               patch_type="application/strategic-merge-patch+json")
        return await ControllerRefManager(d, sel, adopt, release, recheck_deletion(fresh)).claim(rss)

    def pod_map(self, d, rss) -> dict:
        """getPodMapForDeployment: RS uid -> its pods (by ControllerRef), inactive ones included."""
        sel = selector_from_label_selector(spec_of(d).get("selector"))
        out = {m.uid_of(r): [] for r in rss}
        for p in self.pod_inf.list():
            if m.namespace_of(p) != m.namespace_of(d) or not sel.matches(m.labels_of(p)):
                continue
            ref = m.controller_ref(p)
            if ref is not None and ref.get("uid") in out:
                out[ref["uid"]].append(p)
        return out

    # ------------------------------------------------------------------ writes
    @staticmethod
    def _typed(o, api="apps/v1", kind="ReplicaSet"):
        o = dict(o)
        o.setdefault("apiVersion", api)
        o.setdefault("kind", kind)
        return o

    async def update_rs_obj(self, rs):
        return await self.client.update(self._typed(rs))

    async def update_deployment(self, d):
        return await self.client.update(self._typed(d, kind="Deployment"))

    async def update_deployment_status(self, d):
        return await self.client.update(self._typed(d, kind="Deployment"), "status")

    # ------------------------------------------------------------------ syncDeployment
    async def sync(self, key):
        d = self.d_inf.get(key)
        if d is None:
            return
        d = m.deepcopy(d)
        sel = spec_of(d).get("selector")
        if sel is not None and not sel.get("matchLabels") and not sel.get("matchExpressions"):
            self._event(d, "Warning", "SelectingAll",
                        "This deployment is selecting all pods. A non-empty selector is required.")
            st = d.setdefault("status", {})
            gen = (d.get("metadata") or {}).get("generation", 0)
            if int(st.get("observedGeneration") or 0) < gen:
                st["observedGeneration"] = gen
                await self.update_deployment_status(d)
            return
        rss = await self.replica_sets_for(d)
        pod_map = self.pod_map(d, rss)
        if (d.get("metadata") or {}).get("deletionTimestamp"):
            await self.sync_status_only(d, rss, pod_map)
            return
        d = await self.check_paused_conditions(d)
        if spec_of(d).get("paused"):
            await self.sync_scale(d, rss, pod_map)
            return
        if spec_of(d).get("rollbackTo") is not None:
            await self.rollback(d, rss, pod_map)
            return
        if await self.is_scaling_event(d, rss, pod_map):
            await self.sync_scale(d, rss, pod_map)
            return
        strategy = (spec_of(d).get("strategy") or {}).get("type") or "RollingUpdate"
        if strategy == "Recreate":
            await self.rollout_recreate(d, rss, pod_map)
        elif strategy == "RollingUpdate":
            await self.rollout_rolling(d, rss, pod_map)
        else:
            raise ValueError(f"unexpected deployment strategy type: {strategy}")

    async def sync_status_only(self, d, rss, pod_map):
        new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, False)
        await self.sync_deployment_status(olds + [new], new, d)

    async def sync_scale(self, d, rss, pod_map):
        """sync (sync.go): scale, cleanup when paused, status."""
        new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, False)
        await self.scale(d, new, olds)
        if spec_of(d).get("paused") and spec_of(d).get("rollbackTo") is None:
            await self.cleanup_deployment(olds, d)
        await self.sync_deployment_status(olds + [new], new, d)

    async def check_paused_conditions(self, d):
        if spec_of(d).get("progressDeadlineSeconds") is None:
            return d
        st = d.setdefault("status", {})
        cond = get_condition(st, "Progressing")
        if cond is not None and cond.get("reason") == TIMED_OUT:
            return d
        paused_exists = cond is not None and cond.get("reason") == PAUSED
        now = self.clock()
        if spec_of(d).get("paused") and not paused_exists:
            set_condition(st, new_condition("Progressing", "Unknown", PAUSED, "Deployment is paused", now))
        elif not spec_of(d).get("paused") and paused_exists:
            set_condition(st, new_condition("Progressing", "Unknown", RESUMED, "Deployment is resumed", now))
        else:
            return d
        return await self.update_deployment_status(d)

    async def get_all_rss_and_sync_revision(self, d, rss, pod_map, create: bool):
        _, all_old = find_old_rss(d, rss)
        new = await self.get_new_rs(d, rss, all_old, create)
        return new, all_old

    async def get_new_rs(self, d, rss, old_rss, create: bool):
        """getNewReplicaSet (sync.go)."""
        existing = find_new_rs(d, rss)
        new_revision = str(max_revision(old_rss) + 1)
        now = self.clock()
        if existing is not None:
            rs = m.deepcopy(existing)
            ann_changed = set_new_rs_annotations(d, rs, new_revision, True)
            mrs = int(spec_of(d).get("minReadySeconds") or 0)
            if ann_changed or int(spec_of(rs).get("minReadySeconds") or 0) != mrs:
                rs["spec"]["minReadySeconds"] = mrs
                return await self.update_rs_obj(rs)
            needs = set_deployment_revision(d, annotations_of(rs).get(REVISION, ""))
            st = d.setdefault("status", {})
            if spec_of(d).get("progressDeadlineSeconds") is not None and get_condition(st, "Progressing") is None:
                set_condition(st, new_condition("Progressing", "True", FOUND_NEW_RS,
                                                f'Found new replica set "{m.name_of(rs)}"', now))
                needs = True
            if needs:
                updated = await self.update_deployment_status(d)
                d.clear()
                d.update(updated)
            return rs
        if not create:
            return None
        tpl = m.deepcopy(spec_of(d).get("template") or {})
        cc = status_of(d).get("collisionCount")
        h = compute_hash(tpl, cc)
        tpl.setdefault("metadata", {}).setdefault("labels", {})[HASH_LABEL] = h
        sel = m.deepcopy(spec_of(d).get("selector") or {})
        sel.setdefault("matchLabels", {})[HASH_LABEL] = h
        rs = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
              "metadata": {"name": f"{m.name_of(d)}-{safe_encode(h)}", "namespace": m.namespace_of(d),
                           "labels": dict(tpl["metadata"]["labels"]),
                           "ownerReferences": [m.new_controller_ref(d, "apps/v1", "Deployment")]},
              "spec": {"replicas": 0, "minReadySeconds": int(spec_of(d).get("minReadySeconds") or 0),
                       "selector": sel, "template": tpl}}
        count = new_rs_new_replicas(d, old_rss + [rs], rs)
        rs["spec"]["replicas"] = count
        set_new_rs_annotations(d, rs, new_revision, False)
        exists = False
        try:
            created = await self.client.create(rs, m.namespace_of(d))
        except m.StatusError as e:
            if m.is_already_exists(e):
                exists = True
                cur = self.rs_inf.get(f"{m.namespace_of(d)}/{m.name_of(rs)}") or \
                    await self.client.get("replicasets", m.name_of(rs), m.namespace_of(d))
                if not equal_ignore_hash(spec_of(d).get("template"), spec_of(cur).get("template")):
                    st = d.setdefault("status", {})
                    st["collisionCount"] = int(st.get("collisionCount") or 0) + 1
                    await self.update_deployment_status(d)
                    raise
                created = cur
            else:
                msg = f'Failed to create new replica set "{m.name_of(rs)}": {e}'
                if spec_of(d).get("progressDeadlineSeconds") is not None:
                    set_condition(d.setdefault("status", {}),
                                  new_condition("Progressing", "False", FAILED_RS_CREATE, msg, now))
                    try:
                        await self.update_deployment_status(d)
                    except m.StatusError:
                        pass
                self._event(d, "Warning", FAILED_RS_CREATE, msg)
                raise
        if not exists and count > 0:
            self._event(d, "Normal", "ScalingReplicaSet", f"Scaled up replica set {m.name_of(created)} to {count}")
        needs = set_deployment_revision(d, new_revision)
        if not exists and spec_of(d).get("progressDeadlineSeconds") is not None:
            set_condition(d.setdefault("status", {}), new_condition("Progressing", "True", NEW_RS_CREATED,
                                                                    f'Created new replica set "{m.name_of(created)}"', now))
            needs = True
        if needs:
            updated = await self.update_deployment_status(d)
            d.clear()
            d.update(updated)
        return created

    # ------------------------------------------------------------------ scaling
    async def scale(self, d, new, olds):
        """scale (sync.go): the single active (or latest) RS follows spec.replicas; a saturated
        new RS zeroes the old ones; otherwise proportional scaling of a rolling deployment."""
        only = find_active_or_latest(new, olds)
        if only is not None:
            if rs_replicas(only) == d_replicas(d):
                return
            await self.scale_rs_and_record_event(only, d_replicas(d), d)
            return
        if is_saturated(d, new):
            for old in filter_active_replica_sets(olds):
                await self.scale_rs_and_record_event(old, 0, d)
            return
        if not is_rolling_update(d):
            return
        all_rss = filter_active_replica_sets(olds + [new])
        total = replica_count(all_rss)
        allowed = d_replicas(d) + max_surge(d) if d_replicas(d) > 0 else 0
        to_add = allowed - total
        op = ""
        if to_add > 0:
            sort_by_size_newer(all_rss)
            op = "up"
        elif to_add < 0:
            sort_by_size_older(all_rss)
            op = "down"
        added = 0
        sizes = {}
        for rs in all_rss:
            if to_add != 0:
                p = get_proportion(rs, d, to_add, added)
                sizes[m.name_of(rs)] = rs_replicas(rs) + p
                added += p
            else:
                sizes[m.name_of(rs)] = rs_replicas(rs)
        for i, rs in enumerate(all_rss):
            if i == 0 and to_add != 0:
                sizes[m.name_of(rs)] = max(0, sizes[m.name_of(rs)] + to_add - added)
            await self.scale_rs(rs, sizes[m.name_of(rs)], d, op)

    async def scale_rs_and_record_event(self, rs, new_scale: int, d):
        if rs_replicas(rs) == new_scale:
            return False, rs
        op = "up" if rs_replicas(rs) < new_scale else "down"
        return await self.scale_rs(rs, new_scale, d, op)

    async def scale_rs(self, rs, new_scale: int, d, op: str):
        copy = m.deepcopy(rs)
        size_changed = rs_replicas(copy) != new_scale
        ann_changed = set_replicas_annotations(copy, d_replicas(d), d_replicas(d) + max_surge(d))
        scaled = False
        if size_changed or ann_changed:
            copy["spec"]["replicas"] = new_scale
            rs = await self.update_rs_obj(copy)
            if size_changed:
                scaled = True
                self._event(d, "Normal", "ScalingReplicaSet", f"Scaled {op} replica set {m.name_of(rs)} to {new_scale}")
        return scaled, rs

    async def cleanup_deployment(self, olds, d):
        limit = spec_of(d).get("revisionHistoryLimit")
        if limit is None:
            return
        alive = [r for r in olds if r is not None and not (r.get("metadata") or {}).get("deletionTimestamp")]
        diff = len(alive) - int(limit)
        if diff <= 0:
            return
        alive.sort(key=by_creation_timestamp)
        for rs in alive[:diff]:
            st = status_of(rs)
            if int(st.get("replicas") or 0) != 0 or rs_replicas(rs) != 0 or \
                    int((rs.get("metadata") or {}).get("generation") or 0) > int(st.get("observedGeneration") or 0) or \
                    (rs.get("metadata") or {}).get("deletionTimestamp"):
                continue
            try:
                await self.client.delete("replicasets", m.name_of(rs), m.namespace_of(rs))
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise

    async def sync_deployment_status(self, all_rss, new, d):
        status = calculate_status(all_rss, new, d, self.clock())
        if not status_changed(status_of(d), status):
            return
        d["status"] = status
        await self.update_deployment_status(d)

    async def is_scaling_event(self, d, rss, pod_map) -> bool:
        new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, False)
        for rs in filter_active_replica_sets(olds + [new]):
            desired, ok = get_int_annotation(rs, DESIRED)
            if ok and desired != d_replicas(d):
                return True
        return False

    # ------------------------------------------------------------------ rolling update
    async def rollout_rolling(self, d, rss, pod_map):
        new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, True)
        all_rss = olds + [new]
        if await self.reconcile_new_rs(all_rss, new, d):
            await self.sync_rollout_status(all_rss, new, d)
            return
        if await self.reconcile_old_rss(all_rss, filter_active_replica_sets(olds), new, d):
            await self.sync_rollout_status(all_rss, new, d)
            return
        if deployment_complete(d, status_of(d)):
            await self.cleanup_deployment(olds, d)
        await self.sync_rollout_status(all_rss, new, d)

    async def reconcile_new_rs(self, all_rss, new, d) -> bool:
        if rs_replicas(new) == d_replicas(d):
            return False
        if rs_replicas(new) > d_replicas(d):
            scaled, _ = await self.scale_rs_and_record_event(new, d_replicas(d), d)
            return scaled
        count = new_rs_new_replicas(d, all_rss, new)
        scaled, _ = await self.scale_rs_and_record_event(new, count, d)
        return scaled

    async def reconcile_old_rss(self, all_rss, olds, new, d) -> bool:
        if replica_count(olds) == 0:
            return False
        all_count = replica_count(all_rss)
        min_avail = d_replicas(d) - max_unavailable(d)
        new_unavailable = rs_replicas(new) - int(status_of(new).get("availableReplicas") or 0)
        max_scaled_down = all_count - min_avail - new_unavailable
        if max_scaled_down <= 0:
            return False
        try:
            olds, cleaned = await self.cleanup_unhealthy_replicas(olds, d, max_scaled_down)
        except Exception:
            return False
        all_rss = olds + [new]
        try:
            scaled_down = await self.scale_down_old_rss_for_rolling_update(all_rss, olds, d)
        except Exception:
            return False
        return cleaned + scaled_down > 0

    async def cleanup_unhealthy_replicas(self, olds, d, max_cleanup: int):
        olds = sorted(olds, key=by_creation_timestamp)
        total = 0
        for i, rs in enumerate(olds):
            if total >= max_cleanup:
                break
            if rs_replicas(rs) == 0:
                continue
            avail = int(status_of(rs).get("availableReplicas") or 0)
            if rs_replicas(rs) == avail:
                continue
            n = min(max_cleanup - total, rs_replicas(rs) - avail)
            new_count = rs_replicas(rs) - n
            if new_count > rs_replicas(rs):
                raise ValueError(f"when cleaning up unhealthy replicas, got invalid request to scale down "
                                 f"{m.key_of(rs)} {rs_replicas(rs)} -> {new_count}")
            _, updated = await self.scale_rs_and_record_event(rs, new_count, d)
            total += n
            olds[i] = updated
        return olds, total

    async def scale_down_old_rss_for_rolling_update(self, all_rss, olds, d) -> int:
        min_avail = d_replicas(d) - max_unavailable(d)
        available = available_replica_count(all_rss)
        if available <= min_avail:
            return 0
        total, to_scale = 0, available - min_avail
        for rs in sorted(olds, key=by_creation_timestamp):
            if total >= to_scale:
                break
            if rs_replicas(rs) == 0:
                continue
            n = min(rs_replicas(rs), to_scale - total)
            await self.scale_rs_and_record_event(rs, rs_replicas(rs) - n, d)
            total += n
        return total

    # ------------------------------------------------------------------ recreate
    async def rollout_recreate(self, d, rss, pod_map):
        new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, False)
        all_rss = olds + [new]
        active_olds = filter_active_replica_sets(olds)
        if await self.scale_down_old_rss_for_recreate(active_olds, d):
            await self.sync_rollout_status(all_rss, new, d)
            return
        if old_pods_running(new, olds, pod_map):
            await self.sync_rollout_status(all_rss, new, d)
            return
        if new is None:
            new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, True)
            all_rss = olds + [new]
        await self.scale_rs_and_record_event(new, d_replicas(d), d)
        if deployment_complete(d, status_of(d)):
            await self.cleanup_deployment(olds, d)
        await self.sync_rollout_status(all_rss, new, d)

    async def scale_down_old_rss_for_recreate(self, olds, d) -> bool:
        scaled = False
        for i, rs in enumerate(olds):
            if rs_replicas(rs) == 0:
                continue
            s, updated = await self.scale_rs_and_record_event(rs, 0, d)
            if s:
                olds[i] = updated
                scaled = True
        return scaled

    # ------------------------------------------------------------------ progress
    async def sync_rollout_status(self, all_rss, new, d):
        """syncRolloutStatus (progress.go:34-107)."""
        now = self.clock()
        status = calculate_status(all_rss, new, d, now)
        deadline = spec_of(d).get("progressDeadlineSeconds")
        if deadline is None:
            remove_condition(status, "Progressing")
        cur = get_condition(status_of(d), "Progressing")
        complete = status.get("replicas") == status.get("updatedReplicas") and cur is not None and \
            cur.get("reason") == NEW_RS_AVAILABLE
        name = m.name_of(new) if new is not None else ""
        if deadline is not None and not complete:
            if deployment_complete(d, status):
                msg = f'ReplicaSet "{name}" has successfully progressed.' if new is not None else \
                    f'Deployment "{m.name_of(d)}" has successfully progressed.'
                set_condition(status, new_condition("Progressing", "True", NEW_RS_AVAILABLE, msg, now))
            elif deployment_progressing(d, status):
                msg = f'ReplicaSet "{name}" is progressing.' if new is not None else \
                    f'Deployment "{m.name_of(d)}" is progressing.'
                cond = new_condition("Progressing", "True", RS_UPDATED, msg, now)
                if cur is not None:
                    if cur.get("status") == "True":
                        cond["lastTransitionTime"] = cur.get("lastTransitionTime")
                    remove_condition(status, "Progressing")
                set_condition(status, cond)
            elif deployment_timed_out(d, status, now):
                msg = f'ReplicaSet "{name}" has timed out progressing.' if new is not None else \
                    f'Deployment "{m.name_of(d)}" has timed out progressing.'
                set_condition(status, new_condition("Progressing", "False", TIMED_OUT, msg, now))
        failures = self.replica_failures(all_rss, new)
        if failures:
            set_condition(status, failures[0])
        else:
            remove_condition(status, "ReplicaFailure")
        if not status_changed(status_of(d), status):
            self.requeue_stuck_deployment(d, status)
            return
        d["status"] = status
        await self.update_deployment_status(d)

    @staticmethod
    def replica_failures(all_rss, new) -> list:
        out = []
        if new is not None:
            out = [rs_to_deployment_condition(c) for c in status_of(new).get("conditions") or []
                   if c.get("type") == "ReplicaFailure"]
        if out:
            return out
        for rs in all_rss:
            if rs is None:
                continue
            out += [rs_to_deployment_condition(c) for c in status_of(rs).get("conditions") or []
                    if c.get("type") == "ReplicaFailure"]
        return out

    def requeue_stuck_deployment(self, d, status) -> float:
        """requeueStuckDeployment (progress.go:148-181): -1 (no requeue), 0 (rate limited now)
        or the seconds until the progress deadline."""
        cur = get_condition(status_of(d), "Progressing")
        deadline = spec_of(d).get("progressDeadlineSeconds")
        if deadline is None or cur is None:
            return -1
        if deployment_complete(d, status) or cur.get("reason") == TIMED_OUT:
            return -1
        after = (m.parse_time(cur.get("lastUpdateTime")) or 0.0) + int(deadline) - self.clock()
        if after < 1.0:
            self.queue.add_rate_limited(m.key_of(d))
            return 0
        self.queue.add_after(m.key_of(d), after + 1.0)
        return after

    # ------------------------------------------------------------------ rollback
    async def rollback(self, d, rss, pod_map):
        """rollback.go: to spec.rollbackTo.revision (0: the previous revision)."""
        new, olds = await self.get_all_rss_and_sync_revision(d, rss, pod_map, True)
        all_rss = olds + [new]
        to = int((spec_of(d).get("rollbackTo") or {}).get("revision") or 0)
        if to == 0:
            to = last_revision(all_rss)
            if to == 0:
                self._event(d, "Warning", ROLLBACK_REVISION_NOT_FOUND, "Unable to find last revision.")
                await self.update_deployment_and_clear_rollback_to(d)
                return
        for rs in all_rss:
            if rs is None:
                continue
            v = _safe_revision(rs)
            if v is None or v != to:
                continue
            if await self.rollback_to_template(d, rs):
                self._event(d, "Normal", ROLLBACK_DONE, f'Rolled back deployment "{m.name_of(d)}" to revision {to}')
            return
        self._event(d, "Warning", ROLLBACK_REVISION_NOT_FOUND, "Unable to find the revision to rollback to.")
        await self.update_deployment_and_clear_rollback_to(d)

    async def rollback_to_template(self, d, rs) -> bool:
        performed = False
        if not equal_ignore_hash(spec_of(d).get("template"), spec_of(rs).get("template")):
            tpl = m.deepcopy(spec_of(rs).get("template") or {})
            labels = (tpl.get("metadata") or {}).get("labels")
            if labels is not None:
                labels.pop(HASH_LABEL, None)
            d["spec"]["template"] = tpl
            set_deployment_annotations_to(d, rs)
            performed = True
        else:
            self._event(d, "Warning", ROLLBACK_TEMPLATE_UNCHANGED,
                        f'The rollback revision contains the same template as current deployment "{m.name_of(d)}"')
        await self.update_deployment_and_clear_rollback_to(d)
        return performed

    async def update_deployment_and_clear_rollback_to(self, d):
        d["spec"].pop("rollbackTo", None)
        return await self.update_deployment(d)


def old_pods_running(new, olds, pod_map) -> bool:
    """oldPodsRunning (recreate.go): an old RS reports pods, or a pod of an old RS is neither
    Succeeded nor Failed."""
    if actual_replica_count(olds) > 0:
        return True
    for uid, pods in pod_map.items():
        if new is not None and m.uid_of(new) == uid:
            continue
        for p in pods:
            if (p.get("status") or {}).get("phase") not in ("Failed", "Succeeded"):
                return True
    return False
