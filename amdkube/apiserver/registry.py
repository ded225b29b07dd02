"""Resource registries: generic REST store + per-kind strategies + subresources.

Reference: staging/src/k8s.io/apiserver/pkg/registry/generic/registry/store.go:308
(Create: BeforeCreate → Storage.Create), :507 (Update), :664 (Get), :262 (List), :1133
(Watch); per-kind strategies in pkg/registry/core/{pod,node,...}/strategy.go; the fork's
pods/binding path pkg/registry/core/pod/storage/storage.go:138-211 (assignPod →
setPodHostAndAnnotations writes NodeName and every ExtendedResources[i].Assigned in one
GuaranteedUpdate).

Deliberate fix: binding validates the extendedResourceBinding
against the node's advertised healthy devices and against the device IDs already
assigned to other non-terminal pods on that node (an index maintained from the commit
stream), inside the same atomic update — so two racing schedulers can never hand out
one GPU twice.
"""
from __future__ import annotations

import copy
import json
import time

from ..api import meta as m
from ..utils.trace import POD_TRACE
from ..api.helpers import (HEALTHY, pod_assigned_devices, pod_extended_resource_count, pod_extended_resource_name,
                           ExtendedResourceError, set_condition, is_pod_terminal)
from ..api.labels import parse_field_selector, parse_selector
from ..api.scheme import SCHEME, ResourceInfo
from ..api.validation import validate_binding
from ..store import Filter, MVCCStore, Storage, event_object, PUT
from ..store.storage import decode_kv
from . import rbacescalation
from . import admission as adm
from .service import ServiceAllocator
from ..api.field import go_value


def _json_merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = _json_merge_patch(target.get(k), v)
    return out


def _json_pointer(path):
    return [p.replace("~1", "/").replace("~0", "~") for p in path.lstrip("/").split("/")] if path else []


def _json_patch(doc, ops):
    doc = copy.deepcopy(doc)
    for op in ops:
        parts = _json_pointer(op["path"])
        parent = doc
        for p in parts[:-1]:
            parent = parent[int(p)] if isinstance(parent, list) else parent[p]
        last = parts[-1] if parts else None
        kind = op["op"]
        if kind in ("add", "replace"):
            if isinstance(parent, list):
                if last == "-":
                    parent.append(op["value"])
                elif kind == "add":
                    parent.insert(int(last), op["value"])
                else:
                    parent[int(last)] = op["value"]
            else:
                if kind == "replace" and last not in parent:
                    raise m.invalid("Patch", "", [f"replace of missing path {op['path']}"])
                parent[last] = op["value"]
        elif kind == "remove":
            if isinstance(parent, list):
                parent.pop(int(last))
            else:
                parent.pop(last)
        elif kind == "test":
            cur = parent[int(last)] if isinstance(parent, list) else parent.get(last)
            if cur != op["value"]:
                raise m.invalid("Patch", "", [f"test failed at {op['path']}"])
        else:
            raise m.bad_request(f"unsupported json patch op {kind}")
    return doc


def apply_patch(cur: dict, patch_body: bytes, content_type: str) -> dict:
    """PATCH (staging/src/k8s.io/apiserver/pkg/endpoints/handlers/patch.go): JSON patch, JSON
    merge patch, or strategic merge patch interpreted against the kind's schema (the patch
    strategy and merge key of every nested field, api/strategicpatch.py). Custom resources have
    no strategic schema: the reference answers 415 for them."""
    try:
        patch = json.loads(patch_body)
    except ValueError as e:
        raise m.bad_request(f"invalid patch: {e}")
    if "json-patch" in content_type:
        return _json_patch(cur, patch)
    if "strategic-merge" in content_type:
        from ..api import strategicpatch as smp
        node = smp.schema_for(cur.get("apiVersion"), cur.get("kind"))
        if node is None:        # every built-in kind has a schema: this is a custom resource
            raise m.StatusError(415, "UnsupportedMediaType",
                                f"the body of the request was in an unknown format - accepted media types include: "
                                f"application/json-patch+json, application/merge-patch+json")
        try:
            return smp.apply(cur, patch, node)
        except smp.PatchError as e:
            raise m.bad_request(str(e))
    if not isinstance(patch, dict):
        raise m.bad_request("a merge patch must be a JSON object")
    return _json_merge_patch(cur, patch)


# ---------------------------------------------------------------------------- fields
def pod_fields(o):
    sp, st, md = o.get("spec") or {}, o.get("status") or {}, o.get("metadata") or {}
    return {"metadata.name": md.get("name", ""), "metadata.namespace": md.get("namespace", ""),
            "spec.nodeName": sp.get("nodeName", ""), "spec.restartPolicy": sp.get("restartPolicy", ""),
            "spec.schedulerName": sp.get("schedulerName", ""), "status.phase": st.get("phase", ""),
            "status.podIP": st.get("podIP", "")}


def node_fields(o):
    return {"metadata.name": m.name_of(o), "spec.unschedulable": str(bool((o.get("spec") or {}).get("unschedulable"))).lower()}


def event_fields(o):
    io = o.get("involvedObject") or {}
    f = {"metadata.name": m.name_of(o), "metadata.namespace": m.namespace_of(o), "reason": o.get("reason", ""),
         "type": o.get("type", ""), "source": (o.get("source") or {}).get("component", "")}
    for k in ("kind", "namespace", "name", "uid", "apiVersion", "resourceVersion", "fieldPath"):
        f["involvedObject." + k] = io.get(k, "")
    return f


def ns_fields(o):
    return {"metadata.name": m.name_of(o), "status.phase": (o.get("status") or {}).get("phase", "")}


def default_fields(o):
    return {"metadata.name": m.name_of(o), "metadata.namespace": m.namespace_of(o)}


FIELDS = {"pods": pod_fields, "nodes": node_fields, "events": event_fields, "namespaces": ns_fields}

_STATUS_KINDS = {"pods", "nodes", "namespaces", "services", "daemonsets", "replicasets", "deployments", "jobs",
                 "resourcequotas", "persistentvolumes", "persistentvolumeclaims", "statefulsets", "replicationcontrollers",
                 "cronjobs", "horizontalpodautoscalers", "poddisruptionbudgets", "certificatesigningrequests",
                 "volumeattachments"}
_GENERATION_KINDS = {"daemonsets", "replicasets", "deployments", "jobs", "statefulsets", "replicationcontrollers",
                     "poddisruptionbudgets", "horizontalpodautoscalers"}


def pod_qos(pod) -> str:
    reqs, lims, any_set, guaranteed = {}, {}, False, True
    for c in (pod.get("spec") or {}).get("containers") or []:
        r = (c.get("resources") or {})
        rq, li = r.get("requests") or {}, r.get("limits") or {}
        if rq or li:
            any_set = True
        for k in ("cpu", "memory"):
            if k not in li or (k in rq and rq[k] != li[k]):
                guaranteed = False
    if not any_set:
        return "BestEffort"
    return "Guaranteed" if guaranteed else "Burstable"


def _generate_job_selector(job: dict):
    """pkg/registry/batch/job/strategy.go generateSelector: unless spec.manualSelector, the Job
    selects its pods by its own uid (controller-uid), set on the template with job-name."""
    spec = job.setdefault("spec", {})
    if spec.get("manualSelector"):
        return
    uid, name = job["metadata"]["uid"], job["metadata"].get("name", "")
    tmd = spec.setdefault("template", {}).setdefault("metadata", {})
    labels = tmd.setdefault("labels", {})
    labels["controller-uid"] = uid
    labels["job-name"] = name
    sel = spec.get("selector") or {}
    sel.setdefault("matchLabels", {})["controller-uid"] = uid
    spec["selector"] = sel


class ResourceStore:
    def __init__(self, api: "Registry", ri: ResourceInfo):
        self.api, self.ri = api, ri
        self.storage = Storage(api.store, ri.plural, getattr(api, "media_type", "application/json"))
        self.fields_fn = FIELDS.get(ri.plural, default_fields)
        self.has_status = ri.plural in _STATUS_KINDS or ri.plural == "customresourcedefinitions"
        self.generation = ri.plural in _GENERATION_KINDS
        self.storage_prefix = f"/registry/{ri.plural}"   # custom resources: /registry/crd/<group>/<plural>

    # ----------------------------------------------------------------- keys
    def key(self, ns, name):
        p = self.storage_prefix
        return f"{p}/{ns}/{name}" if self.ri.namespaced else f"{p}/{name}"

    def prefix(self, ns=""):
        if self.ri.namespaced and ns:
            return f"{self.storage_prefix}/{ns}/"
        return f"{self.storage_prefix}/"

    def filter(self, label_selector=None, field_selector=None) -> Filter | None:
        ls = parse_selector(label_selector) if label_selector else None
        fs = parse_field_selector(field_selector) if field_selector else None
        if ls is None and fs is None:
            return None
        return Filter(ls, fs, self.fields_fn)

    # --------------------------------------------------------------- verbs
    def get(self, ns, name):
        return self.storage.get(self.key(ns, name))

    def list(self, ns="", label_selector=None, field_selector=None, limit=0, cont=None):
        flt = self.filter(label_selector, field_selector)
        return self.storage.list(self.prefix(ns), flt, limit, cont)

    def watch(self, ns="", rv=None, label_selector=None, field_selector=None, name=None):
        flt = self.filter(label_selector, field_selector)
        if name:
            return self.storage.watch(self.key(ns, name), rv, flt, exact=True)
        return self.storage.watch(self.prefix(ns), rv, flt)

    def _admission_ctx(self):
        return self.api

    def create(self, ns, obj, user=None, dry_run=False):
        ri = self.ri
        SCHEME.to_storage(obj)   # a served-only version's body (extensions/v1beta1 …) → storage version
        md = obj.setdefault("metadata", {})
        obj["apiVersion"], obj["kind"] = ri.api_version, ri.kind
        if ri.namespaced:
            if md.get("namespace") and ns and md["namespace"] != ns:
                raise m.bad_request("the namespace of the provided object does not match the namespace sent on the request")
            md["namespace"] = ns or md.get("namespace") or "default"
        else:
            md.pop("namespace", None)
        if not md.get("name") and md.get("generateName"):
            md["name"] = md["generateName"] + m.new_uid().replace("-", "")[:5]
        md["uid"] = m.new_uid()
        md["creationTimestamp"] = m.now_rfc3339()
        md.pop("resourceVersion", None)
        md.pop("deletionTimestamp", None)
        if self.generation:
            md["generation"] = 1
        SCHEME.default(obj)
        key = self.key(md.get("namespace", ""), md["name"])
        try:
            out = self._create_checked(key, obj, md, user, dry_run)
        finally:
            if ri.plural == "services":      # allocations of a create that did not commit go back
                self.api.services.release_pending(key)
        if dry_run:
            return out
        if self.ri.plural == "pods":
            POD_TRACE(md.get("uid", ""), "api_created")
        return out

    def _create_checked(self, key, obj, md, user, dry_run):
        ri = self.ri
        self.prepare_for_create(obj)
        if ri.plural == "certificatesigningrequests" and user is not None:
            # certificates/strategy.go PrepareForCreate: the requester is who authenticated, not
            # what the body claims
            spec = obj.setdefault("spec", {})
            spec["username"], spec["uid"] = user.get("name", ""), user.get("uid", "")
            spec["groups"] = list(user.get("groups") or [])
        attrs = adm.Attributes(adm.CREATE, ri.plural, "", md.get("namespace", ""), md.get("name", ""), obj, None, user, ri.kind,
                               ri.group, dry_run=dry_run)
        self.api.admission.admit(attrs, self.api)
        SCHEME.default(obj)  # admission may add fields (e.g. ResourceV2) that need defaults
        if ri.group == rbacescalation.GROUP:
            rbacescalation.check(self.api, ri.plural, md.get("namespace", ""), obj, user)
        errs = SCHEME.validate(obj)
        if errs:
            raise m.invalid(ri.kind, md.get("name", ""), errs)
        self.api.admission.validate(attrs, self.api)
        if dry_run:
            return obj
        return self.storage.create(key, obj)

    def prepare_for_create(self, obj):
        p = self.ri.plural
        if p == "pods":
            st = obj.setdefault("status", {})
            st.clear()
            st.update({"phase": "Pending", "qosClass": pod_qos(obj)})
        elif p == "namespaces":
            obj["status"] = {"phase": "Active"}
        elif p in _STATUS_KINDS and p not in ("nodes",):
            obj["status"] = {}
        if p == "jobs":
            _generate_job_selector(obj)
        if p == "services":
            md = obj["metadata"]
            self.api.services.prepare_create(self.key(md.get("namespace", ""), md.get("name", "")), obj)

    def _prepare_update(self, new, cur, subresource):
        md, cmd = new.setdefault("metadata", {}), cur.get("metadata") or {}
        for k in ("uid", "creationTimestamp", "namespace", "name", "deletionTimestamp", "deletionGracePeriodSeconds",
                  "generateName"):
            if k in cmd:
                md[k] = cmd[k]
            else:
                md.pop(k, None)
        new["apiVersion"], new["kind"] = self.ri.api_version, self.ri.kind
        if subresource == "status":
            new["spec"] = m.deepcopy(cur.get("spec"))
            keep = m.deepcopy(cmd)
            keep["resourceVersion"] = md.get("resourceVersion", cmd.get("resourceVersion"))
            if self.ri.plural == "horizontalpodautoscalers":
                # v2beta1 status (current metrics, conditions) lives in annotations of the v1 object
                from ..api.autoscaling import METRICS_ANNOTATION, STATUS_ANNOTATIONS
                na, ka = md.get("annotations") or {}, dict(keep.get("annotations") or {})
                for k in STATUS_ANNOTATIONS:
                    if k in na:
                        ka[k] = na[k]
                    else:
                        ka.pop(k, None)
                if METRICS_ANNOTATION in (cmd.get("annotations") or {}):
                    ka[METRICS_ANNOTATION] = cmd["annotations"][METRICS_ANNOTATION]
                keep["annotations"] = ka or None
            if self.ri.plural == "deployments":
                # deploymentStatusStrategy keeps spec and labels only: the controller records
                # the revision annotation through /status (registry/extensions/deployment)
                keep["annotations"] = m.deepcopy(md.get("annotations"))
                if keep["annotations"] is None:
                    keep.pop("annotations")
            new["metadata"] = keep
        elif self.has_status:
            if "status" in cur:
                new["status"] = m.deepcopy(cur["status"])
            else:
                new.pop("status", None)
            if self.ri.plural == "horizontalpodautoscalers":   # status annotations change only via status
                from ..api.autoscaling import STATUS_ANNOTATIONS
                ca, na = cmd.get("annotations") or {}, dict(md.get("annotations") or {})
                for k in STATUS_ANNOTATIONS:
                    if k in ca:
                        na[k] = ca[k]
                    else:
                        na.pop(k, None)
                md["annotations"] = na or None
        if self.ri.plural == "daemonsets" and subresource != "status":
            # daemonSetStrategy.PrepareForUpdate: a changed template bumps spec.templateGeneration
            # (the extensions/v1beta1 field; apps/v1 objects do not carry it)
            cs, ns_ = cur.get("spec") or {}, new.get("spec") or {}
            if "templateGeneration" in cs:
                if cs.get("template") != ns_.get("template"):
                    ns_["templateGeneration"] = int(cs["templateGeneration"] or 0) + 1
                else:
                    ns_["templateGeneration"] = cs["templateGeneration"]
        if self.generation:
            md["generation"] = cmd.get("generation", 1) + (1 if new.get("spec") != cur.get("spec") else 0)
        if self.ri.plural == "services" and subresource != "status":
            self.api.services.prepare_update(self.key(md.get("namespace", ""), md.get("name", "")), new, cur)
        if self.ri.plural == "pods" and subresource != "status":
            # only pods/binding may write spec.nodeName and extendedResources[].assigned
            cur_spec = cur.get("spec") or {}
            new.setdefault("spec", {})
            if cur_spec.get("nodeName"):
                new["spec"]["nodeName"] = cur_spec["nodeName"]
            cur_assigned = {r.get("name"): r.get("assigned") for r in cur_spec.get("extendedResources") or []}
            for r in new["spec"].get("extendedResources") or []:
                if cur_assigned.get(r.get("name")):
                    r["assigned"] = cur_assigned[r.get("name")]
                else:
                    r.pop("assigned", None)

    def update(self, ns, name, obj, subresource="", user=None, patch=None, content_type="", create_on_update=False,
               served=None):
        """PUT (obj) or PATCH (patch bytes). Returns (obj, created)."""
        key = self.key(ns, name)
        precond_rv = None if patch is not None else ((obj.get("metadata") or {}).get("resourceVersion") or None)
        created = [False]
        delete_after = [False]

        def try_update(cur):
            if cur is None:
                if patch is None and create_on_update:
                    created[0] = True
                    return None
                raise m.not_found(self.ri.plural, name)
            if patch is not None and served is not None and served.from_storage is not None:
                # a patch written against a served version with its own shape (autoscaling/v2beta1):
                # apply it to that view of the object, then convert back
                view = m.deepcopy(cur)
                view["apiVersion"], view["kind"] = served.api_version, served.kind
                served.from_storage(view)
                new = SCHEME.to_storage(apply_patch(view, patch, content_type))
            elif patch is not None:
                new = apply_patch(cur, patch, content_type)
            else:
                new = SCHEME.to_storage(m.deepcopy(obj))
            nmd = new.setdefault("metadata", {})
            if nmd.get("name", name) != name:
                raise m.bad_request("the name of the object does not match the name on the URL")
            if patch is not None and nmd.get("resourceVersion") and \
                    nmd["resourceVersion"] != (cur.get("metadata") or {}).get("resourceVersion"):
                # a patch that sets metadata.resourceVersion is a precondition (the patched object
                # goes through Store.Update, which compares it: `kubectl label --resource-version`)
                raise m.conflict(self.ri.plural, name, "the object has been modified; please apply your changes to "
                                 "the latest version and try again")
            self._prepare_update(new, cur, subresource)
            SCHEME.default(new)
            if self.ri.group == rbacescalation.GROUP:
                rbacescalation.check(self.api, self.ri.plural, ns, new, user, cur)
            attrs = adm.Attributes(adm.UPDATE, self.ri.plural, subresource, ns, name, new, cur, user, self.ri.kind,
                                   self.ri.group)
            self.api.admission.admit(attrs, self.api)
            errs = SCHEME.validate(new, cur) if not subresource else []
            if self.ri.plural == "pods" and subresource == "status":
                errs = _validate_pod_status(new)
            if errs:
                raise m.invalid(self.ri.kind, name, errs)
            self.api.admission.validate(attrs, self.api)
            a, b = dict(new), dict(cur)
            a["metadata"] = {k: v for k, v in new["metadata"].items() if k != "resourceVersion"}
            b["metadata"] = {k: v for k, v in (cur.get("metadata") or {}).items() if k != "resourceVersion"}
            if a == b:
                return None
            if nmd.get("deletionTimestamp") and not nmd.get("finalizers") and not (
                    self.ri.plural == "namespaces" and ((new.get("spec") or {}).get("finalizers"))):
                if self.ri.plural != "pods" or nmd.get("deletionGracePeriodSeconds") == 0:
                    delete_after[0] = True
            return new

        try:
            res = self.storage.guaranteed_update(key, try_update, precond_rv=precond_rv, ignore_not_found=create_on_update)
        finally:
            if self.ri.plural == "services":
                self.api.services.release_pending(key)
        if created[0]:
            return self.create(ns, obj, user), True
        if res is None:
            raise m.not_found(self.ri.plural, name)
        if delete_after[0]:
            try:
                self.storage.delete(key)
            except m.StatusError:
                pass
        return res, False

    def delete(self, ns, name, grace=None, precond_uid=None, user=None, propagation=None):
        """Returns (obj, deleted_now)."""
        key = self.key(ns, name)
        cur = self.storage.get(key)
        attrs = adm.Attributes(adm.DELETE, self.ri.plural, "", ns, name, None, cur, user, self.ri.kind, self.ri.group)
        self.api.admission.admit(attrs, self.api)
        self.api.admission.validate(attrs, self.api)
        md = cur.get("metadata") or {}
        graceful = self._grace_period(cur, grace)
        finalizers = list(md.get("finalizers") or [])
        if propagation == "Orphan" and "orphan" not in finalizers:
            finalizers.append("orphan")
        elif propagation == "Foreground" and "foregroundDeletion" not in finalizers:
            finalizers.append("foregroundDeletion")
        ns_finalizers = self.ri.plural == "namespaces" and ((cur.get("spec") or {}).get("finalizers"))
        if graceful or finalizers or ns_finalizers:
            def mark(c):
                cm = c.setdefault("metadata", {})  # c is a fresh decode: mutate in place
                if precond_uid and cm.get("uid") != precond_uid:
                    raise m.conflict(self.ri.plural, name, "Precondition failed: UID mismatch")
                if not cm.get("deletionTimestamp"):
                    cm["deletionTimestamp"] = m.now_rfc3339() if not graceful else \
                        time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(time.time() + graceful))
                if graceful:
                    prev = cm.get("deletionGracePeriodSeconds")
                    cm["deletionGracePeriodSeconds"] = graceful if prev is None else min(prev, graceful)
                elif self.ri.plural == "pods":
                    # a final (grace 0) delete held only by finalizers: removing the last one deletes it
                    cm["deletionGracePeriodSeconds"] = 0
                if finalizers:
                    cm["finalizers"] = sorted(set((cm.get("finalizers") or []) + finalizers))
                if self.ri.plural == "namespaces":
                    c.setdefault("status", {})["phase"] = "Terminating"
                return c
            obj = self.storage.guaranteed_update(key, mark)
            return obj, False
        obj = self.storage.delete(key, precond_uid=precond_uid)
        return obj, True

    def _grace_period(self, cur, grace):
        if self.ri.plural != "pods":
            return 0
        spec = cur.get("spec") or {}
        if not spec.get("nodeName") or is_pod_terminal(cur):
            return 0
        if grace is None:
            grace = spec.get("terminationGracePeriodSeconds", 30)
        md = cur.get("metadata") or {}
        if md.get("deletionTimestamp") and grace and md.get("deletionGracePeriodSeconds") is not None:
            grace = min(grace, md["deletionGracePeriodSeconds"])
        return max(0, int(grace or 0))


def _validate_pod_status(pod):
    errs = []
    ph = (pod.get("status") or {}).get("phase")
    if ph and ph not in ("Pending", "Running", "Succeeded", "Failed", "Unknown"):
        errs.append(f"status.phase: Unsupported value: {go_value(ph)}")
    return errs


class Registry:
    """All resource stores + admission context + the node device-assignment index."""

    def __init__(self, store: MVCCStore, admission: adm.Chain, services: ServiceAllocator | None = None,
                 media_type: str = "application/json"):
        self.store = store
        self.media_type = media_type     # --storage-media-type: how objects are encoded in the store
        self.admission = admission
        self.services = services or ServiceAllocator()
        self.resources: dict[tuple[str, str], ResourceStore] = {}
        for ri in SCHEME.storage_versions():
            if ri.plural == "bindings":
                continue
            self.resources[(ri.group, ri.plural)] = ResourceStore(self, ri)
        # node -> rname -> device id -> pod key ; pod key -> list[(node, rname, id)]
        self.device_index: dict[str, dict[str, dict[str, str]]] = {}
        self._device_claims: dict[tuple[str, str, str], str] = {}   # (node, resource, id) -> binding pod (in flight)
        self._claims_by_pod: dict[str, list] = {}
        self._pod_devices: dict[str, list[tuple[str, str, str]]] = {}
        store.commit_hooks.append(self._on_commit)
        self._rebuild_index()

    def rs(self, plural: str, group: str = "") -> ResourceStore:
        return self.resources[(group, plural)]

    # ------------------------------------------------------ admission context
    def get_namespace(self, name):
        return self.rs("namespaces").storage.get(f"/registry/namespaces/{name}", ignore_not_found=True)

    def create_namespace(self, name):
        try:
            self.rs("namespaces").create("", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name}})
        except m.StatusError as e:
            if not m.is_already_exists(e):
                raise

    def list_objects(self, plural, ns, group=""):
        for (g, p), r in self.resources.items():
            if p == plural:
                return r.list(ns)[0]
        return []

    authorizer = None   # set by the APIServer (admission plugins that check permissions)
    cloud = None        # cloud provider (PersistentVolumeLabel)

    def authorize(self, user, verb, group, resource, sub="", ns="", name="") -> bool:
        if self.authorizer is None:
            return True
        from .auth import Attributes as AuthzAttributes
        ok, _ = self.authorizer.authorize(AuthzAttributes(user or {}, verb, group, resource, sub, ns, name))
        return ok

    def plural_for_kind(self, api_version, kind):
        ri = SCHEME.for_kind(api_version, kind)
        return ri.plural if ri is not None else None

    def guaranteed_update_object(self, plural, ns, name, try_update, group=""):
        """Read-modify-CAS an object straight in storage (no admission, no validation): the
        ResourceQuota admission's status reservation (controller.go UpdateQuotaStatus)."""
        for (g, p), r in self.resources.items():
            if p == plural and (not group or g == group):
                return r.storage.guaranteed_update(r.key(ns, name), try_update)
        raise m.not_found(plural, name)

    def get_object(self, plural, ns, name):
        for (g, p), r in self.resources.items():
            if p == plural:
                return r.storage.get(r.key(ns, name), ignore_not_found=True)
        return None

    # --------------------------------------------------------- device index
    def _index_pod(self, key: str, pod: dict | None):
        for node, rname, did in self._pod_devices.pop(key, []):
            d = self.device_index.get(node, {}).get(rname, {})
            if d.get(did) == key:
                del d[did]
        if pod is None or is_pod_terminal(pod):
            return
        node = (pod.get("spec") or {}).get("nodeName")
        if not node:
            return
        entries = []
        for rname, ids in pod_assigned_devices(pod).items():
            slot = self.device_index.setdefault(node, {}).setdefault(rname, {})
            for did in ids:
                slot[did] = key
                entries.append((node, rname, did))
        if entries:
            self._pod_devices[key] = entries

    def _on_commit(self, ev):
        k = ev.kv.key
        if k.startswith("/registry/pods/"):
            self._index_pod(k, event_object(ev) if ev.type == PUT else None)
        elif k.startswith("/registry/services/"):
            self.services.index(k, event_object(ev) if ev.type == PUT else None)

    def _rebuild_index(self):
        kvs, _, _ = self.store.range("/registry/pods/")
        for kv in kvs:
            self._index_pod(kv.key, decode_kv(kv.value))
        self.services.rebuild(self.store.range("/registry/services/")[0])  # ipallocator/portallocator repair

    # ------------------------------------------------------------ eviction
    def evict(self, ns: str, name: str, body: dict, user=None):
        """POST pods/<name>/eviction (pkg/registry/core/pod/storage/eviction.go): a pod covered by
        a PodDisruptionBudget is deleted only while the budget allows a disruption; the budget's
        disruptionsAllowed is decremented and the pod recorded in status.disruptedPods in the same
        CAS update, so concurrent evictions cannot overdraw it (429 otherwise)."""
        from ..api.labels import selector_from_label_selector
        pods = self.rs("pods")
        pod = pods.get(ns, name)
        grace = (body.get("deleteOptions") or {}).get("gracePeriodSeconds")
        if not is_pod_terminal(pod) and (pod.get("status") or {}).get("phase") != "Pending":
            labels = (pod.get("metadata") or {}).get("labels") or {}
            pdbs = [p for p in self.rs("poddisruptionbudgets", "policy").list(ns)[0]
                    if (p.get("spec") or {}).get("selector") and
                    selector_from_label_selector(p["spec"]["selector"]).matches(labels)]
            if len(pdbs) > 1:
                raise m.StatusError(500, "InternalError", "This pod has more than one PodDisruptionBudget, which the eviction "
                                                          "subresource does not support.")
            if pdbs:
                pdb = pdbs[0]
                prs = self.rs("poddisruptionbudgets", "policy")

                def take(cur):
                    st = cur.setdefault("status", {})
                    if st.get("observedGeneration", 0) < (cur.get("metadata") or {}).get("generation", 1):
                        raise m.too_many_requests("Cannot evict pod as it would violate the pod's disruption budget: "
                                                  "the budget's status is out of date")
                    if int(st.get("disruptionsAllowed", st.get("podDisruptionsAllowed", 0)) or 0) <= 0:
                        raise m.too_many_requests("Cannot evict pod as it would violate the pod's disruption budget.")
                    st["disruptionsAllowed"] = int(st.get("disruptionsAllowed", 0)) - 1
                    st.setdefault("disruptedPods", {})[name] = m.now_rfc3339()
                    return cur
                prs.storage.guaranteed_update(prs.key(ns, m.name_of(pdb)), take)
        return pods.delete(ns, name, grace=grace, user=user)

    # ------------------------------------------------------------- binding
    def bind(self, ns: str, binding: dict, user=None) -> dict:
        """POST pods/<name>/binding (storage.go:138-211 + SURVEY fix #1/#10)."""
        name = m.name_of(binding)
        errs = validate_binding(binding)
        if errs:
            raise m.invalid("Binding", name, errs)
        tgt = binding["target"]
        node_name = tgt["name"]
        ext = tgt.get("extendedResourceBinding") or {}
        pods = self.rs("pods")
        key = pods.key(ns, name)
        node = None
        attrs = adm.Attributes(adm.CREATE, "pods", "binding", ns, name, binding, None, user, "Binding")
        self.admission.admit(attrs, self)
        self.admission.validate(attrs, self)

        def assign(cur):
            nonlocal node
            pod = cur  # freshly decoded from the store by guaranteed_update: safe to mutate
            md = pod.setdefault("metadata", {})
            if md.get("deletionTimestamp"):
                raise m.conflict("pods", name, "pod is being deleted, cannot be assigned to a host")
            spec = pod.setdefault("spec", {})
            if spec.get("nodeName"):
                raise m.conflict("pods", name, f"pod {name} is already assigned to node {spec['nodeName']!r}")
            pres_list = spec.get("extendedResources") or []
            if pres_list or ext:
                node = node or self.rs("nodes").storage.get(f"/registry/nodes/{node_name}", ignore_not_found=True)
                self._check_device_binding(pod, pres_list, ext, node, node_name, key)
            spec["nodeName"] = node_name
            for pres in pres_list:
                if pres.get("name") in ext:
                    pres["assigned"] = list(ext[pres["name"]].get("resources") or [])
            ann = m.annotations_of(binding)
            if ann:
                md.setdefault("annotations", {}).update(ann)
            set_condition(pod, {"type": "PodScheduled", "status": "True"}, m.now_rfc3339())
            return pod

        try:
            pods.storage.guaranteed_update(key, assign, precond_uid=(binding.get("metadata") or {}).get("uid"))
        finally:
            self._release_device_claims(key)
        return m.success_status()

    def _release_device_claims(self, pod_key: str):
        for slot in self._claims_by_pod.pop(pod_key, ()):
            if self._device_claims.get(slot) == pod_key:
                del self._device_claims[slot]

    def _check_device_binding(self, pod, pres_list, ext, node, node_name, pod_key):
        name = m.name_of(pod)
        known = {p.get("name"): p for p in pres_list}
        for k in ext:
            if k not in known:
                raise m.invalid("Binding", name, [f"target.extendedResourceBinding[{k}]: Not found: pod has no such extended resource"])
        if node is None:
            raise m.invalid("Binding", name, [f"target.name: Not found: node {node_name!r} (needed to validate device binding)"])
        node_ext = (node.get("status") or {}).get("extendedResources") or {}
        in_use = self.device_index.get(node_name, {})
        claimed: set[tuple[str, str]] = set()
        for pres in pres_list:
            pname = pres.get("name")
            if pname not in ext:
                raise m.invalid("Binding", name, [f"target.extendedResourceBinding[{pname}]: Required value: every pod extended resource must be bound"])
            try:
                rname = pod_extended_resource_name(pres)
                want = pod_extended_resource_count(pres)
            except ExtendedResourceError as e:
                raise m.invalid("Binding", name, [str(e)])
            ids = ext[pname].get("resources") or []
            if len(ids) != want:
                raise m.invalid("Binding", name, [f"target.extendedResourceBinding[{pname}]: Invalid value: {len(ids)} devices bound, {want} requested"])
            devs = ((node_ext.get(rname) or {}).get("resources") or {})
            used = in_use.get(rname, {})
            for did in ids:
                dev = devs.get(did)
                if dev is None:
                    raise m.invalid("Binding", name, [f"target.extendedResourceBinding[{pname}]: Invalid value: device {did!r} of {rname} does not exist on node {node_name}"])
                if (dev.get("health") or HEALTHY) != HEALTHY:
                    raise m.conflict("pods", name, f"device {did} of {rname} on node {node_name} is Unhealthy")
                owner = used.get(did) or self._device_claims.get((node_name, rname, did))
                if owner and owner != pod_key:
                    raise m.conflict("pods", name, f"device {did} of {rname} on node {node_name} is already assigned to pod {owner.split('/', 3)[-1]}")
                if (rname, did) in claimed:
                    raise m.invalid("Binding", name, [f"device {did} bound twice in one binding"])
                claimed.add((rname, did))
        # claim the devices until this bind's write settles: over a bridged store other binds
        # run while it is in flight, and the device index moves only on commit
        slots = self._claims_by_pod.setdefault(pod_key, [])
        for rname, did in claimed:
            slot = (node_name, rname, did)
            if self._device_claims.setdefault(slot, pod_key) == pod_key and slot not in slots:
                slots.append(slot)
