"""Label / field selectors and qualified-name validation.

Semantics follow apimachinery labels (reference:
staging/src/k8s.io/apimachinery/pkg/labels/selector.go:134-160 NewRequirement validation,
:193-240 Matches incl. Gt/Lt integer parsing; selector string grammar in the same file's
Lexer/Parser). The fork converts device-attribute requirements (NodeSelectorRequirement
shape) into these selectors (pkg/apis/core/v1/helper/helpers.go:465-498).

Implementation note: requirements are compiled once into closures so that the device
allocator's hot loop (devices x selectors) does no string parsing.
"""
from __future__ import annotations

import re
from typing import Callable, Iterable, Mapping

IN, NOT_IN, EQUALS, DOUBLE_EQUALS, NOT_EQUALS = "in", "notin", "=", "==", "!="
EXISTS, DOES_NOT_EXIST, GT, LT = "exists", "!", "gt", "lt"

_NODE_OPS = {"In": IN, "NotIn": NOT_IN, "Exists": EXISTS, "DoesNotExist": DOES_NOT_EXIST, "Gt": GT, "Lt": LT}

_DNS1123_LABEL = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")
_DNS1123_SUBDOMAIN = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")
_QUALIFIED_NAME = re.compile(r"^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$")
_LABEL_VALUE = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")


class SelectorError(ValueError):
    pass


def is_dns1123_label(s: str) -> list[str]:
    errs = []
    if len(s) > 63:
        errs.append("must be no more than 63 characters")
    if not _DNS1123_LABEL.match(s or ""):
        errs.append("a DNS-1123 label must consist of lower case alphanumeric characters or '-', and must start and end with an alphanumeric character")
    return errs


def is_dns1123_subdomain(s: str) -> list[str]:
    errs = []
    if len(s) > 253:
        errs.append("must be no more than 253 characters")
    if not _DNS1123_SUBDOMAIN.match(s or ""):
        errs.append("a DNS-1123 subdomain must consist of lower case alphanumeric characters, '-' or '.', and must start and end with an alphanumeric character")
    return errs


def is_qualified_name(s: str) -> list[str]:
    """`[prefix/]name`; exactly zero or one slash (selector.go:135 quirk #13 in SURVEY §7.6)."""
    parts = s.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if not prefix:
            return ["prefix part must be non-empty"]
        errs = is_dns1123_subdomain(prefix)
        if errs:
            return ["prefix part " + e for e in errs]
    else:
        return ["a qualified name must consist of alphanumeric characters, '-', '_' or '.', with an optional DNS subdomain prefix and '/' (e.g. 'example.com/MyName')"]
    if not name:
        return ["name part must be non-empty"]
    if len(name) > 63:
        return ["name part must be no more than 63 characters"]
    if not _QUALIFIED_NAME.match(name):
        return ["name part must consist of alphanumeric characters, '-', '_' or '.', and must start and end with an alphanumeric character"]
    return []


def is_valid_label_value(v: str) -> list[str]:
    if len(v) > 63:
        return ["must be no more than 63 characters"]
    if not _LABEL_VALUE.match(v):
        return ["a valid label must be an empty string or consist of alphanumeric characters, '-', '_' or '.'"]
    return []


class Requirement:
    __slots__ = ("key", "op", "values", "_match")

    def __init__(self, key: str, op: str, values: Iterable[str] = ()):
        errs = is_qualified_name(key)
        if errs:
            raise SelectorError(f"invalid label key {key!r}: {'; '.join(errs)}")
        values = [str(v) for v in values]
        if op in (IN, NOT_IN):
            if not values:
                raise SelectorError("for 'in', 'notin' operators, values set can't be empty")
        elif op in (EQUALS, DOUBLE_EQUALS, NOT_EQUALS):
            if len(values) != 1:
                raise SelectorError("exact-match compatibility requires one single value")
        elif op in (EXISTS, DOES_NOT_EXIST):
            if values:
                raise SelectorError("values set must be empty for exists and does not exist")
        elif op in (GT, LT):
            if len(values) != 1:
                raise SelectorError("for 'Gt', 'Lt' operators, exactly one value is required")
            try:
                int(values[0])
            except ValueError:
                raise SelectorError("for 'Gt', 'Lt' operators, the value must be an integer")
        else:
            raise SelectorError(f"operator {op!r} is not recognized")
        for v in values:
            if op not in (GT, LT):
                errs = is_valid_label_value(v)
                if errs:
                    raise SelectorError(f"invalid label value {v!r}: {'; '.join(errs)}")
        self.key, self.op, self.values = key, op, values
        self._match = self._compile()

    def _compile(self) -> Callable[[Mapping[str, str]], bool]:
        k, vals = self.key, frozenset(self.values)
        op = self.op
        if op in (IN, EQUALS, DOUBLE_EQUALS):
            return lambda ls: k in ls and ls[k] in vals
        if op in (NOT_IN, NOT_EQUALS):
            return lambda ls: k not in ls or ls[k] not in vals
        if op == EXISTS:
            return lambda ls: k in ls
        if op == DOES_NOT_EXIST:
            return lambda ls: k not in ls
        bound = int(self.values[0])

        def cmp(ls, gt=(op == GT)):
            if k not in ls:
                return False
            try:
                v = int(ls[k])
            except (TypeError, ValueError):
                return False
            return v > bound if gt else v < bound
        return cmp

    def matches(self, ls: Mapping[str, str]) -> bool:
        return self._match(ls)

    def __str__(self):
        if self.op == EXISTS:
            return self.key
        if self.op == DOES_NOT_EXIST:
            return "!" + self.key
        if self.op in (IN, NOT_IN):
            return f"{self.key} {self.op} ({','.join(sorted(self.values))})"
        if self.op in (GT, LT):
            return f"{self.key}{'>' if self.op == GT else '<'}{self.values[0]}"
        return f"{self.key}{self.op}{self.values[0]}"


class Selector:
    __slots__ = ("reqs",)

    def __init__(self, reqs: Iterable[Requirement] = ()):
        self.reqs = list(reqs)

    def matches(self, ls: Mapping[str, str] | None) -> bool:
        ls = ls or {}
        for r in self.reqs:
            if not r._match(ls):
                return False
        return True

    def empty(self) -> bool:
        return not self.reqs

    def __str__(self):
        return ",".join(str(r) for r in self.reqs)


EVERYTHING = Selector()

_TOKEN = re.compile(r"\s*(\(|\)|,|!=|==|=|!|>|<|[^\s(),!=<>]+)")


def parse_selector(s: str | None) -> Selector:
    """Parse the label-selector string grammar (`a=b,c!=d,e in (x,y),!f,g,h>3`)."""
    if not s or not s.strip():
        return Selector()
    toks = [t for t in _TOKEN.findall(s)]
    i, reqs = 0, []

    def peek(j=0):
        return toks[i + j] if i + j < len(toks) else None

    while i < len(toks):
        t = toks[i]
        if t == "!":
            reqs.append(Requirement(toks[i + 1], DOES_NOT_EXIST))
            i += 2
        else:
            key = t
            nxt = peek(1)
            if nxt in (None, ","):
                reqs.append(Requirement(key, EXISTS))
                i += 1
            elif nxt in ("=", "==", "!="):
                val = peek(2)
                if val in (None, ","):
                    reqs.append(Requirement(key, nxt, [""]))
                    i += 2
                else:
                    reqs.append(Requirement(key, nxt, [val]))
                    i += 3
            elif nxt in (">", "<"):
                reqs.append(Requirement(key, GT if nxt == ">" else LT, [peek(2)]))
                i += 3
            elif nxt in (IN, NOT_IN):
                if peek(2) != "(":
                    raise SelectorError(f"found {peek(2)!r}, expected: '('")
                j, vals = i + 3, []
                while j < len(toks) and toks[j] != ")":
                    if toks[j] != ",":
                        vals.append(toks[j])
                    j += 1
                if j >= len(toks):
                    raise SelectorError("found end of string, expected: ')'")
                reqs.append(Requirement(key, nxt, vals))
                i = j + 1
            else:
                raise SelectorError(f"unable to parse requirement: found {nxt!r}")
        if i < len(toks):
            if toks[i] != ",":
                raise SelectorError(f"found {toks[i]!r}, expected: ','")
            i += 1
    return Selector(reqs)


def selector_from_set(ls: Mapping[str, str] | None) -> Selector:
    return Selector(Requirement(k, EQUALS, [v]) for k, v in sorted((ls or {}).items()))


def selector_from_label_selector(ls: dict | None) -> Selector:
    """metav1.LabelSelector {matchLabels, matchExpressions} -> Selector."""
    if ls is None:
        return Selector([Requirement("__nothing__", EXISTS), Requirement("__nothing__", DOES_NOT_EXIST)])
    reqs = [Requirement(k, EQUALS, [v]) for k, v in sorted((ls.get("matchLabels") or {}).items())]
    for e in ls.get("matchExpressions") or []:
        op = _NODE_OPS.get(e.get("operator"))
        if op is None or op in (GT, LT):
            raise SelectorError(f"{e.get('operator')!r} is not a valid pod selector operator")
        reqs.append(Requirement(e["key"], op, e.get("values") or []))
    return Selector(reqs)


def node_requirements_as_selector(reqs: list[dict] | None) -> Selector:
    """NodeSelectorRequirement list (also the fork's ResourceSelector) -> Selector.

    Parity: pkg/apis/core/v1/helper/helpers.go:465-498 (ExtendedRequirementsAsSelector /
    NodeSelectorRequirementsAsSelector). Empty list -> matches everything.
    """
    if not reqs:
        return Selector()
    out = []
    for r in reqs:
        op = _NODE_OPS.get(r.get("operator"))
        if op is None:
            raise SelectorError(f"{r.get('operator')!r} is not a valid selector operator")
        out.append(Requirement(r.get("key", ""), op, r.get("values") or []))
    return Selector(out)


# ----------------------------------------------------------------- field selectors
class FieldSelector:
    """`metadata.name=x,spec.nodeName!=,status.phase!=Succeeded` over a flattened field map."""
    __slots__ = ("terms",)

    def __init__(self, terms):
        self.terms = terms  # list of (field, op, value)

    def matches(self, fields: Mapping[str, str]) -> bool:
        for f, op, v in self.terms:
            have = fields.get(f, "")
            if op == "!=":
                if have == v:
                    return False
            elif have != v:
                return False
        return True

    def empty(self):
        return not self.terms

    def fields(self):
        return [t[0] for t in self.terms]

    def __str__(self):
        return ",".join(f"{f}{op}{v}" for f, op, v in self.terms)


def parse_field_selector(s: str | None) -> FieldSelector:
    if not s:
        return FieldSelector([])
    terms = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        for op in ("!=", "==", "="):
            if op in part:
                f, v = part.split(op, 1)
                terms.append((f.strip(), "!=" if op == "!=" else "=", v.strip()))
                break
        else:
            raise SelectorError(f"invalid field selector term {part!r}")
    return FieldSelector(terms)
