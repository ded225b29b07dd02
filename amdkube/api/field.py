"""Validation error rendering shared by every validator.

Reference: apimachinery pkg/util/validation/field/errors.go — Error.ErrorBody. A string bad value
prints %q-quoted, numbers and bools with %v, nil and nil pointers as the quoted string "null",
anything else with %#v. `go_slice` builds the %#v form of a typed Go slice.
"""
from __future__ import annotations

import json


class GoRepr(str):
    """A value already rendered the way Go's %#v prints it."""


def go_slice(type_name: str, items) -> GoRepr:
    if items is None:
        return GoRepr(f"[]{type_name}(nil)")
    return GoRepr(f"[]{type_name}{{" + ", ".join(go_quote(x) if isinstance(x, str) else str(x) for x in items) + "}")


def go_quote(s: str) -> str:
    """strconv.Quote for the characters validation messages meet (printable Unicode kept)."""
    return json.dumps(s, ensure_ascii=False)


def go_value(v) -> str:
    """A field.Error's bad value as ErrorBody prints it."""
    if isinstance(v, GoRepr):
        return str(v)
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return '"null"'
    if isinstance(v, str):
        return go_quote(v)
    return str(v)


class FieldError:
    REQUIRED, FORBIDDEN, INVALID = "Required value", "Forbidden", "Invalid value"

    def __init__(self, kind: str, field: str, value=None, detail: str = ""):
        self.type, self.field, self.value, self.detail = kind, field, value, detail

    def __str__(self):
        body = self.type if self.type in (self.REQUIRED, self.FORBIDDEN) else f"{self.type}: {go_value(self.value)}"
        if self.detail:
            body += f": {self.detail}"
        return f"{self.field}: {body}"

    __repr__ = __str__


def invalid(path, value, detail):
    return FieldError(FieldError.INVALID, path, value, detail)


def required(path, detail=""):
    return FieldError(FieldError.REQUIRED, path, None, detail)


def forbidden(path, detail):
    return FieldError(FieldError.FORBIDDEN, path, None, detail)
