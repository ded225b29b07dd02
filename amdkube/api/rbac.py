"""RBAC rule coverage and role / binding reconciliation.

Reference: pkg/registry/rbac/validation/policy_comparator.go (Covers, BreakdownRule,
ruleCovers — a servant rule set is covered when every atomic (group, resource, verb[, name])
or (non-resource URL, verb) tuple it grants is granted by some owner rule) and
pkg/registry/rbac/reconciliation/reconcile_role.go, reconcile_rolebindings.go (what
`kubectl auth reconcile` applies, pkg/kubectl/cmd/auth/reconcile.go:59,153): an existing role
keeps what it has, gains the missing rules (union) and the expected labels/annotations; a
binding gains the missing subjects; a binding whose roleRef changed is deleted and re-created;
an object annotated `rbac.authorization.kubernetes.io/autoupdate: "false"` is left alone.
"""
from __future__ import annotations

import copy

AUTOUPDATE = "rbac.authorization.kubernetes.io/autoupdate"
NONE, CREATE, UPDATE, RECREATE = "none", "create", "update", "recreate"


def breakdown(rule: dict) -> list[dict]:
    """BreakdownRule: one rule per (group, resource, verb[, resourceName]) and (URL, verb)."""
    out = []
    names = rule.get("resourceNames") or []
    for g in rule.get("apiGroups") or []:
        for r in rule.get("resources") or []:
            for v in rule.get("verbs") or []:
                if names:
                    out += [{"apiGroups": [g], "resources": [r], "verbs": [v], "resourceNames": [n]} for n in names]
                else:
                    out.append({"apiGroups": [g], "resources": [r], "verbs": [v]})
    for u in rule.get("nonResourceURLs") or []:
        for v in rule.get("verbs") or []:
            out.append({"nonResourceURLs": [u], "verbs": [v]})
    return out


def _resource_covers(owner: list, sub: list) -> bool:
    if "*" in owner or set(sub) <= set(owner):
        return True
    for path in sub:
        if path in owner:
            continue
        if "/" not in path:
            return False
        if "*/" + path.split("/", 1)[1] not in owner:
            return False
    return True


def _url_covers(owner: str, sub: str) -> bool:
    return owner == sub or (owner.endswith("*") and sub.startswith(owner.rstrip("*")))


def rule_covers(owner: dict, sub: dict) -> bool:
    ov, og = owner.get("verbs") or [], owner.get("apiGroups") or []
    verbs = "*" in ov or set(sub.get("verbs") or []) <= set(ov)
    groups = "*" in og or set(sub.get("apiGroups") or []) <= set(og)
    resources = _resource_covers(owner.get("resources") or [], sub.get("resources") or [])
    urls = all(any(_url_covers(o, p) for o in owner.get("nonResourceURLs") or []) for p in sub.get("nonResourceURLs") or [])
    on, sn = owner.get("resourceNames") or [], sub.get("resourceNames") or []
    names = (not on) if not sn else (not on or set(sn) <= set(on))
    return verbs and groups and resources and names and urls


def covers(owner_rules: list[dict], servant_rules: list[dict]) -> tuple[bool, list[dict]]:
    """(covered, the atomic servant rules no owner rule covers)."""
    missing = [s for r in servant_rules for s in breakdown(r) if not any(rule_covers(o, s) for o in owner_rules)]
    return not missing, missing


def _merged(expected: dict | None, have: dict | None) -> dict | None:
    """merge(): the later map wins; None when both are empty."""
    if not expected and not have:
        return have
    out = dict(expected or {})
    out.update(have or {})
    return out


def _meta_merge(result: dict, existing: dict, expected: dict) -> bool:
    md, emd = result.setdefault("metadata", {}), expected.get("metadata") or {}
    changed = False
    for k in ("annotations", "labels"):
        m = _merged(emd.get(k), md.get(k))
        if m is not None:
            md[k] = m
        if (md.get(k) or {}) != ((existing.get("metadata") or {}).get(k) or {}):
            changed = True
    return changed


def _protected(obj: dict) -> bool:
    return ((obj.get("metadata") or {}).get("annotations") or {}).get(AUTOUPDATE) == "false"


def reconcile_role(existing: dict | None, expected: dict, remove_extra: bool = False) -> dict:
    """computeReconciledRole: {"object", "operation", "protected", "missing_rules", "extra_rules"}."""
    if existing is None:
        agg = (expected.get("aggregationRule") or {}).get("clusterRoleSelectors") or []
        return {"object": expected, "operation": CREATE, "protected": False,
                "missing_rules": expected.get("rules") or [], "extra_rules": [], "missing_selectors": agg}
    res = copy.deepcopy(existing)
    op = UPDATE if _meta_merge(res, existing, expected) else NONE
    _, extra = covers(expected.get("rules") or [], existing.get("rules") or [])
    _, missing = covers(existing.get("rules") or [], expected.get("rules") or [])
    if not remove_extra and missing:
        res["rules"] = list(res.get("rules") or []) + missing
        op = UPDATE
    elif remove_extra and (missing or extra):
        res["rules"] = expected.get("rules") or []
        op = UPDATE
    have_sel = ((existing.get("aggregationRule") or {}).get("clusterRoleSelectors") or [])
    want_sel = ((expected.get("aggregationRule") or {}).get("clusterRoleSelectors") or [])
    miss_sel = [s for s in want_sel if s not in have_sel]
    extra_sel = [s for s in have_sel if s not in want_sel] if expected.get("aggregationRule") is not None else []
    if not remove_extra and miss_sel:
        res.setdefault("aggregationRule", {}).setdefault("clusterRoleSelectors", [])
        res["aggregationRule"]["clusterRoleSelectors"] = list(have_sel) + miss_sel
        op = UPDATE
    elif remove_extra and (miss_sel or extra_sel):
        res["aggregationRule"] = expected.get("aggregationRule")
        op = UPDATE
    return {"object": res, "operation": op, "protected": _protected(existing), "missing_rules": missing,
            "extra_rules": extra, "missing_selectors": miss_sel}


def _subject_key(s: dict) -> tuple:
    return (s.get("kind", ""), s.get("apiGroup", ""), s.get("name", ""), s.get("namespace", ""))


def reconcile_binding(existing: dict | None, expected: dict, remove_extra: bool = False) -> dict:
    """computeReconciledRoleBinding: {"object", "operation", "protected", "missing_subjects", "extra_subjects"}."""
    if existing is None:
        return {"object": expected, "operation": CREATE, "protected": False,
                "missing_subjects": expected.get("subjects") or [], "extra_subjects": []}
    prot = _protected(existing)
    if (expected.get("roleRef") or {}) != (existing.get("roleRef") or {}):
        return {"object": expected, "operation": RECREATE, "protected": prot, "missing_subjects": [], "extra_subjects": []}
    res = copy.deepcopy(existing)
    op = UPDATE if _meta_merge(res, existing, expected) else NONE
    have = {_subject_key(s): s for s in existing.get("subjects") or []}
    want = {_subject_key(s): s for s in expected.get("subjects") or []}
    missing = [s for k, s in want.items() if k not in have]
    extra = [s for k, s in have.items() if k not in want]
    if not remove_extra and missing:
        res["subjects"] = list(existing.get("subjects") or []) + missing
        op = UPDATE
    elif remove_extra and (missing or extra):
        res["subjects"] = expected.get("subjects") or []
        op = UPDATE
    return {"object": res, "operation": op, "protected": prot, "missing_subjects": missing, "extra_subjects": extra}
