"""A small evaluator for the Go expressions table-driven reference tests are written in.

The reference's `_test.go` tables are composite literals built from a handful of local helper
calls (`validPod("x", 2, getResourceRequirements(getComputeResourceList("100m", ""), ...))`).
`hack/extract_*_cases.py` scripts feed a test file's table through this evaluator with Python
versions of those helpers, and write the result as a JSON fixture that amdkube's tests replay;
no case is retyped by hand.

Supported: string/int/float/bool literals, identifiers (qualified: `api.LimitTypePod`), calls,
`&T{...}` / `T{...}` / `[]T{...}` / `map[K]V{...}` composite literals (keyed -> dict, positional
-> list), `nil`, comments. Anything else raises, so a table the evaluator cannot read fails
the extraction loudly instead of being skipped.
"""
from __future__ import annotations

import re

_TOKEN = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<str>"(?:[^"\\]|\\.)*"|`[^`]*`)
  | (?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z_][A-Za-z0-9_]*)*)
  | (?P<punct>\[\]|[(){}\[\],:&*=+])
""", re.S | re.X)


def tokenize(src: str) -> list[tuple[str, str]]:
    out, pos = [], 0
    while pos < len(src):
        mt = _TOKEN.match(src, pos)
        if mt is None:
            raise SyntaxError(f"goexpr: cannot tokenize at {src[pos:pos + 40]!r}")
        pos = mt.end()
        kind = mt.lastgroup
        if kind != "ws":
            out.append((kind, mt.group(kind)))
    return out


class _Unhashable:
    """A map key that is an object; the literal becomes a list of [key, value] pairs."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v


class GoField(str):
    """A composite-literal key written as a bare Go identifier (a struct field name), as opposed
    to a string / named-constant map key; `hook`s rename only these."""


class Evaluator:
    def __init__(self, funcs: dict | None = None, names: dict | None = None, hook=None):
        self.funcs = dict(funcs or {})
        self.names = {"nil": None, "true": True, "false": False, **(names or {})}
        # hook(type_name | None, value) post-processes every keyed struct literal (type_name None
        # for an element whose type Go lets the source elide); map literals are left alone.
        self.hook = hook

    # ------------------------------------------------------------------ driver
    def eval(self, src: str):
        self.toks, self.i = tokenize(src), 0
        v = self.expr()
        if self.i != len(self.toks):
            raise SyntaxError(f"goexpr: trailing tokens {self.toks[self.i:self.i + 5]}")
        return v

    def peek(self, k=0):
        j = self.i + k
        return self.toks[j] if j < len(self.toks) else ("eof", "")

    def take(self, val=None):
        t = self.peek()
        if val is not None and t[1] != val:
            raise SyntaxError(f"goexpr: expected {val!r}, got {t}")
        self.i += 1
        return t

    # ------------------------------------------------------------------ grammar
    def expr(self):
        v = self.unary()
        while self.peek()[1] == "+":              # string concatenation / integer sum
            self.take()
            v = v + self.unary()
        return v

    def unary(self):
        kind, val = self.peek()
        if val in ("&", "*"):
            self.take()
            return self.unary()
        if kind == "str":
            self.take()
            return _unquote(val)
        if kind == "num":
            self.take()
            if any(c in val for c in ".eE"):
                return float(val)
            if len(val.lstrip("-")) > 1 and val.lstrip("-").startswith("0"):
                return int(val, 8)            # Go octal literal (file modes: 0644)
            return int(val)
        if val == "[]":
            self.take()
            self.type_name()
            return self.literal_body()
        if val == "{":
            return self._hooked(None, self.literal_body())
        if kind == "ident":
            if val == "map" and self.peek(1)[1] == "[":
                self.type_name()
                return self.literal_body(is_map=True)
            self.take()
            nxt = self.peek()[1]
            if nxt == "(":
                args = self.args()
                fn = self.funcs.get(val)
                if fn is None:
                    raise NameError(f"goexpr: no helper for {val}()")
                return fn(*args)
            if nxt == "{":
                return self._hooked(val, self.literal_body(is_map=val in self.map_types))
            if val in self.names:
                v = self.names[val]
                while self.peek()[1] == "[" and self.peek(1)[0] == "num" and self.peek(2)[1] == "]":
                    self.take()
                    v = v[int(self.take()[1])]          # indexing a table variable: xs[1]
                    self.take("]")
                return v
            raise NameError(f"goexpr: unknown name {val}")
        raise SyntaxError(f"goexpr: unexpected {kind} {val!r}")

    map_types: frozenset = frozenset()

    def _hooked(self, type_name, v):
        if v == [] and self.hook is not None:
            v = {}                      # `T{}`: an empty struct (empty slices are written []T{})
        if self.hook is not None and isinstance(v, dict) and any(isinstance(k, GoField) for k in v):
            return self.hook(type_name, v)
        return v

    def type_name(self):
        """Skip a type: *pkg.T, []T, map[K]V."""
        while True:
            kind, val = self.peek()
            if val in ("*", "[]"):
                self.take()
                continue
            if val == "map":
                self.take()
                self.take("[")
                self.type_name()
                self.take("]")
                continue
            if val == "struct" and self.peek(1)[1] == "{":
                # an anonymous struct type: skip its field list
                self.take()
                depth = 0
                while True:
                    v = self.take()[1]
                    depth += (v == "{") - (v == "}")
                    if depth == 0:
                        return
            if kind == "ident":
                self.take()
                return
            raise SyntaxError(f"goexpr: bad type at {val!r}")

    def args(self):
        self.take("(")
        out = []
        while self.peek()[1] != ")":
            out.append(self.expr())
            if self.peek()[1] == ",":
                self.take()
        self.take(")")
        return out

    def literal_body(self, is_map=False):
        self.take("{")
        keyed, items = None, []
        while self.peek()[1] != "}":
            if self.peek(1)[1] == ":" and self.peek()[0] in ("ident", "str", "num"):
                kind, k = self.take()
                if kind == "str":
                    k = _unquote(k)
                elif kind == "num":
                    k = int(k)
                elif k in self.names and (is_map or "." in k):
                    k = self.names[k]
                    if isinstance(k, (dict, list)):     # a map keyed by objects (map[*v1.Pod]T): keep pairs
                        k = _Unhashable(k)
                elif not is_map:
                    k = GoField(k)
                self.take(":")
                keyed = keyed if keyed is not None else {}
                keyed[k] = self.expr()
            else:
                e = self.expr()
                if self.peek()[1] == ":":          # a computed map key: core.ResourceName(x): v
                    self.take(":")
                    keyed = keyed if keyed is not None else {}
                    keyed[e if not isinstance(e, (dict, list)) else _Unhashable(e)] = self.expr()
                else:
                    items.append(e)
            if self.peek()[1] == ",":
                self.take()
        self.take("}")
        if keyed is not None:
            if any(isinstance(k, _Unhashable) for k in keyed):
                return [[k.v if isinstance(k, _Unhashable) else k, v] for k, v in keyed.items()]
            return keyed
        return items


def _unquote(s: str) -> str:
    if s.startswith("`"):
        return s[1:-1]
    return bytes(s[1:-1], "utf-8").decode("unicode_escape")


def block_after(src: str, anchor: str, start: int = 0) -> tuple[str, int]:
    """The balanced `{...}` literal that starts at the first `{` after `anchor` (inclusive), and
    the offset just past it. String literals and comments are skipped while balancing."""
    i = src.index(anchor, start)
    j = src.index("{", i + len(anchor) - 1)
    depth, k = 0, j
    while k < len(src):
        c = src[k]
        if c == '"':
            k += 1
            while src[k] != '"':
                k += 2 if src[k] == "\\" else 1
        elif c == "`":
            k = src.index("`", k + 1)
        elif src.startswith("//", k):
            k = src.index("\n", k)
        elif c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return src[j:k + 1], k + 1
        k += 1
    raise SyntaxError(f"unbalanced literal after {anchor!r}")


def line_of(src: str, offset: int) -> int:
    return src.count("\n", 0, offset) + 1


# ---------------------------------------------------------------------------- reading test files
def func_body(src: str, name: str) -> tuple[int, int]:
    start = src.index(f"func {name}(")
    _, end = block_after(src, "{", src.index(")", start))
    return start, end


def statement_extent(src: str, i: int) -> int:
    """End offset of the Go expression starting at i (to the end of its line, brackets balanced)."""
    depth = 0
    while i < len(src):
        c = src[i]
        if c == '"':
            i += 1
            while src[i] != '"':
                i += 2 if src[i] == "\\" else 1
        elif c == "`":
            i = src.index("`", i + 1)
        elif src.startswith("//", i):
            if depth == 0:
                return i
            i = src.index("\n", i)
            continue
        elif c in "({[":
            depth += 1
        elif c in ")}]":
            depth -= 1
        elif c == "\n" and depth == 0:
            return i
        i += 1
    return i


def eval_locals(src: str, ev: Evaluator, start: int, end: int):
    """Evaluate every `\\tname := <expr>` (and `name = <expr>` of a `var (...)` block) at the top
    level of a function body, in order; a statement the evaluator cannot read is skipped (it is
    harness, not data)."""
    for mt in re.finditer(r"^\t(\w+) := |^\t\t(\w+)\s+= ", src[start:end], re.M):
        i = start + mt.end()
        j = statement_extent(src, i)
        try:
            ev.names[mt.group(1) or mt.group(2)] = ev.eval(src[i:j])
        except (SyntaxError, NameError, KeyError, ValueError, TypeError):
            pass


def struct_fields(type_body: str) -> list[str]:
    return [m.group(1) for m in re.finditer(r"^\s*(\w+)\s+[\w.*\[\]]", type_body.strip("{}"), re.M)]


def table(src: str, ev: Evaluator, var: str, start: int) -> tuple[list, int]:
    """The cases of `var := []struct{...}{...}` (or `map[string]struct{...}{...}`, each case
    gaining its key as "name") after `start`, positional cases keyed by the struct's fields."""
    mt = re.compile(rf"\b{re.escape(var)} := (\[\]struct|map\[string\]struct)").search(src, start)
    if mt is None:
        raise ValueError(f"no table {var!r}")
    at = mt.start()
    type_body, k = block_after(src, "struct {", at)
    body, _ = block_after(src, "{", k)
    fields = struct_fields(type_body)
    raw = ev.eval(body)
    if mt.group(1).startswith("map"):
        raw = [{**v, "name": name} if isinstance(v, dict) else {**dict(zip(fields, v)), "name": name}
               for name, v in ((ev_key, val) for ev_key, val in raw.items())]
    out = []
    for c in raw:
        if isinstance(c, list):
            c = dict(zip(fields, c))
        out.append(c)
    return out, line_of(src, at)



# ---------------------------------------------------------------------------- k8s API objects
# Go struct field -> JSON name where the json tag is not the field name with its leading
# acronym lower-cased; None = an embedded struct whose fields are inlined.
JSON_FIELD = {"ObjectMeta": "metadata", "ListMeta": "metadata", "RBDImage": "image", "RBDPool": "pool",
              "CephMonitors": "monitors", "TypeMeta": None, "VolumeSource": None, "PersistentVolumeSource": None,
              "LocalObjectReference": None, "Handler": None, "PodSecurityPolicySpec": "spec"}


def json_key(field: str) -> str:
    if field in JSON_FIELD:
        return JSON_FIELD[field]
    i = 0
    while i < len(field) and field[i].isupper():
        i += 1
    if i == len(field):
        return field.lower()                      # UID, IQN, RBD
    if i > 1:
        i -= 1                                    # PDName -> pdName, HostIP -> hostIP
    return field[:i].lower() + field[i:]


def k8s_hook(type_name, v: dict) -> dict:
    """A keyed Go struct literal -> the JSON object the apiserver would serve."""
    out = {}
    for k, val in v.items():
        if not isinstance(k, GoField):
            out[k] = val
            continue
        jk = json_key(k)
        if jk is None:
            if isinstance(val, dict):
                out.update(val)
            continue
        if val is None:
            continue
        out[jk] = val
    return out


_CONST = re.compile(r'^\s+([A-Z]\w*)\s+(?:[\w.]+\s+)?=\s+"((?:[^"\\]|\\.)*)"', re.M)


def go_string_constants(path: str, prefix: str) -> dict:
    """`Name Type = "value"` constants of a Go file as {prefix + Name: value}."""
    return {prefix + n: val for n, val in _CONST.findall(open(path).read())}


def k8s_names(ref: str) -> dict:
    """The core/v1 and meta/v1 string constants tables refer to (v1.ResourceCPU, metav1.LabelSelectorOpIn)."""
    import os
    names = {}
    names.update(go_string_constants(os.path.join(ref, "staging/src/k8s.io/api/core/v1/types.go"), "v1."))
    names.update(go_string_constants(os.path.join(ref, "staging/src/k8s.io/apimachinery/pkg/apis/meta/v1/types.go"),
                                     "metav1."))
    names.update(go_string_constants(os.path.join(ref, "staging/src/k8s.io/api/storage/v1/types.go"), "storagev1."))
    names.update(go_string_constants(os.path.join(ref, "pkg/kubelet/apis/well_known_labels.go"), "kubeletapis."))
    return names
