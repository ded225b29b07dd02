"""ObjectMeta helpers, API errors (metav1.Status) and the watch event vocabulary.

Objects are plain JSON-shaped dicts everywhere in amdkube (wire format == in-memory
format), which keeps codecs trivial and lets the apiserver pass stored bytes through.
Parity: apimachinery pkg/apis/meta/v1 types, pkg/api/errors/errors.go (reason strings,
HTTP codes), pkg/watch/watch.go (event types; reference SURVEY U4).
"""
from __future__ import annotations

import copy
import datetime as _dt
import json
import uuid

ADDED, MODIFIED, DELETED, ERROR, BOOKMARK = "ADDED", "MODIFIED", "DELETED", "ERROR", "BOOKMARK"


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def format_time(t: float) -> str:
    return _dt.datetime.fromtimestamp(t, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def now_rfc3339_micro() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_time(s: str | None) -> float | None:
    if not s:
        return None
    s = s.rstrip("Z")
    fmt = "%Y-%m-%dT%H:%M:%S.%f" if "." in s else "%Y-%m-%dT%H:%M:%S"
    return _dt.datetime.strptime(s, fmt).replace(tzinfo=_dt.timezone.utc).timestamp()


def new_uid() -> str:
    return str(uuid.uuid4())


def meta(obj: dict) -> dict:
    return obj.setdefault("metadata", {})


def name_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("name", "")


def namespace_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("namespace", "")


def key_of(obj: dict) -> str:
    ns = namespace_of(obj)
    return f"{ns}/{name_of(obj)}" if ns else name_of(obj)


def labels_of(obj: dict) -> dict:
    return (obj.get("metadata") or {}).get("labels") or {}


def annotations_of(obj: dict) -> dict:
    return (obj.get("metadata") or {}).get("annotations") or {}


def uid_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("uid", "")


def rv_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("resourceVersion", "")


def deepcopy(obj):
    # json round-trip is ~2x faster than copy.deepcopy for JSON-shaped data
    try:
        return json.loads(json.dumps(obj))
    except (TypeError, ValueError):
        return copy.deepcopy(obj)


def controller_ref(obj: dict) -> dict | None:
    for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
        if r.get("controller"):
            return r
    return None


def new_controller_ref(owner: dict, api_version: str, kind: str) -> dict:
    return {"apiVersion": api_version, "kind": kind, "name": name_of(owner), "uid": uid_of(owner),
            "controller": True, "blockOwnerDeletion": True}


# ------------------------------------------------------------------------- errors
class StatusError(Exception):
    """An API error carrying a metav1.Status body (errors.StatusError)."""

    def __init__(self, code: int, reason: str, message: str, details: dict | None = None):
        super().__init__(message)
        self.code, self.reason, self.message, self.details = code, reason, message, details or {}

    def status(self) -> dict:
        st = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
              "message": self.message, "reason": self.reason, "code": self.code}
        if self.details:
            st["details"] = self.details
        return st

    @classmethod
    def from_status(cls, st: dict) -> "StatusError":
        return cls(int(st.get("code", 500)), st.get("reason", ""), st.get("message", ""), st.get("details"))

    def __repr__(self):
        return f"StatusError({self.code}, {self.reason!r}, {self.message!r})"


def _details(resource, name):
    group, _, res = resource.rpartition("/") if "/" in resource else ("", "", resource)
    return {"name": name, "group": group, "kind": res}


def not_found(resource: str, name: str) -> StatusError:
    return StatusError(404, "NotFound", f'{resource} "{name}" not found', _details(resource, name))


def already_exists(resource: str, name: str) -> StatusError:
    return StatusError(409, "AlreadyExists", f'{resource} "{name}" already exists', _details(resource, name))


def conflict(resource: str, name: str, msg: str) -> StatusError:
    return StatusError(409, "Conflict", f'Operation cannot be fulfilled on {resource} "{name}": {msg}',
                       _details(resource, name))


def invalid(kind: str, name: str, errs: list[str]) -> StatusError:
    return StatusError(422, "Invalid", f'{kind} "{name}" is invalid: ' + "; ".join(errs),
                       {"name": name, "kind": kind, "causes": [{"message": e} for e in errs]})


def bad_request(msg: str) -> StatusError:
    return StatusError(400, "BadRequest", msg)


def forbidden(msg: str) -> StatusError:
    return StatusError(403, "Forbidden", msg)


def unauthorized(msg: str = "Unauthorized") -> StatusError:
    return StatusError(401, "Unauthorized", msg)


def gone(msg: str) -> StatusError:
    return StatusError(410, "Expired", msg)


def too_many_requests(msg: str = "Too many requests, please try again later.") -> StatusError:
    return StatusError(429, "TooManyRequests", msg)


def internal(msg: str) -> StatusError:
    return StatusError(500, "InternalError", msg)


def method_not_allowed(msg: str) -> StatusError:
    return StatusError(405, "MethodNotAllowed", msg)


def is_not_found(e) -> bool:
    return isinstance(e, StatusError) and e.code == 404


def is_conflict(e) -> bool:
    return isinstance(e, StatusError) and e.code == 409 and e.reason == "Conflict"


def is_already_exists(e) -> bool:
    return isinstance(e, StatusError) and e.reason == "AlreadyExists"


def is_gone(e) -> bool:
    return isinstance(e, StatusError) and e.code == 410


def success_status(details: dict | None = None) -> dict:
    st = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success"}
    if details:
        st["details"] = details
    return st
