"""Go text/template for `kubectl -o go-template=…` / `go-template-file=…`.

Reference: pkg/printers/template.go (the printer: the object as decoded JSON, the `exists`
function, `missingkey=default` unless --allow-missing-template-keys=false) over Go's
text/template. This is the subset kubectl templates use, with Go's semantics:

  * actions `{{ }}` with `{{-`/`-}}` whitespace trimming and `{{/* comments */}}`;
  * pipelines `a | b | c` (the previous value is the last argument), variable declaration
    and assignment (`$x := …`, `$x = …`), parenthesised pipelines, `$` and `$var.Field`;
  * `if`/`else if`/`else`, `range` (lists, maps in sorted key order, `$i, $v :=`, `else`),
    `with`/`else`, `end`; `define`/`template` for named templates;
  * functions and, or, not, len, index, print, printf, println, eq (with several operands), ne,
    lt, le, gt, ge, html, js, urlquery, and kubectl's `exists`;
  * values print as fmt's %v (maps `map[k:v]`, missing keys `<no value>`).
"""
from __future__ import annotations

import html as _html
import json
import re
import urllib.parse

from .jsonpath import go_fmt

__all__ = ["Template", "TemplateError", "render"]


class TemplateError(Exception):
    pass


class _NoValue:
    """A missing map key under missingkey=default (prints "<no value>")."""

    def __repr__(self):
        return "<no value>"

    def go_string(self):
        return "<no value>"

    def __bool__(self):
        return False


NO_VALUE = _NoValue()


# ---------------------------------------------------------------------------- lexing
_ACTION = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)
_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<raw>`[^`]*`)
  | (?P<char>'(?:[^'\\]|\\.)+')
  | (?P<num>[+-]?(?:0[xX][0-9a-fA-F]+|\d+\.\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?|\d+(?:[eE][+-]?\d+)?))
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
  | (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<pipe>\|)
  | (?P<lp>\()
  | (?P<rp>\)(?:\.[A-Za-z0-9_]+)*)
  | (?P<comma>,)
""", re.X | re.S)


def _tokens(src: str) -> list[tuple[str, str]]:
    out, i = [], 0
    while i < len(src):
        mt = _TOKEN.match(src, i)
        if mt is None:
            raise TemplateError(f"unexpected {src[i]!r} in command")
        if mt.lastgroup != "ws":
            out.append((mt.lastgroup, mt.group()))
        i = mt.end()
    return out


def _go_unquote(s: str) -> str:
    if s[0] == "`":
        return s[1:-1]
    return json.loads(s) if s[0] == '"' else s[1:-1]


# ---------------------------------------------------------------------------- parse tree
class _Text:
    def __init__(self, text):
        self.text = text


class _Action:
    def __init__(self, pipe):
        self.pipe = pipe


class _If:
    def __init__(self, kind, pipe):
        self.kind, self.pipe, self.body, self.else_ = kind, pipe, [], None


class _Template:
    def __init__(self, name, pipe):
        self.name, self.pipe = name, pipe


class _Pipe:
    """decl: ([variable names], is_declaration) or None; cmds: list of command token lists."""

    def __init__(self, decl, cmds):
        self.decl, self.cmds = decl, cmds


def _parse_pipe(toks: list) -> _Pipe:
    decl = None
    for j, (k, _v) in enumerate(toks):
        if k in ("decl", "assign"):
            names = [v for kk, v in toks[:j] if kk == "var"]
            decl = (names, k == "decl")
            toks = toks[j + 1:]
            break
        if k not in ("var", "comma"):
            break
    cmds, cur, depth = [], [], 0
    for t in toks:
        if t[0] == "lp":
            depth += 1
        elif t[0] == "rp":
            depth -= 1
        if t[0] == "pipe" and depth == 0:
            cmds.append(cur)
            cur = []
        else:
            cur.append(t)
    cmds.append(cur)
    if any(not c for c in cmds):
        raise TemplateError("missing command")
    return _Pipe(decl, cmds)


class Template:
    def __init__(self, text: str, name: str = "output", funcs: dict | None = None, missingkey: str = "default"):
        self.name = name
        self.missingkey = missingkey
        self.defines: dict[str, list] = {}
        self.funcs = dict(BUILTINS)
        self.funcs.update(funcs or {})
        self.root = self._parse(text)

    # ------------------------------------------------------------- parsing
    def _lex(self, text: str) -> list:
        items, pos = [], 0
        for mt in _ACTION.finditer(text):
            chunk = text[pos:mt.start()]
            if mt.group(1):
                chunk = chunk.rstrip()
            items.append(("text", chunk))
            items.append(("action", mt.group(2).strip(), bool(mt.group(3))))
            pos = mt.end()
        items.append(("text", text[pos:]))
        out, trim_next = [], False
        for it in items:
            if it[0] == "text":
                t = it[1].lstrip() if trim_next else it[1]
                trim_next = False
                if t:
                    out.append(("text", t))
            else:
                out.append(("action", it[1]))
                trim_next = it[2]
        return out

    def _parse(self, text: str) -> list:
        items = self._lex(text)
        stack = [[]]
        blocks: list = []
        for it in items:
            if it[0] == "text":
                stack[-1].append(_Text(it[1]))
                continue
            src = it[1]
            if src.startswith("/*"):
                if not src.endswith("*/"):
                    raise TemplateError("unclosed comment")
                continue
            toks = _tokens(src)
            if not toks:
                raise TemplateError("missing value for command")
            head = toks[0]
            kw = head[1] if head[0] == "ident" else None
            if kw in ("if", "range", "with"):
                node = _If(kw, _parse_pipe(toks[1:]))
                stack[-1].append(node)
                blocks.append(node)
                stack.append(node.body)
            elif kw == "else":
                if not blocks:
                    raise TemplateError("unexpected {{else}}")
                node = blocks[-1]
                stack.pop()
                if len(toks) > 1 and toks[1] == ("ident", "if"):
                    # else if: a nested if in the else branch, closed by the same {{end}}
                    inner = _If("if", _parse_pipe(toks[2:]))
                    node.else_ = [inner]
                    inner.chained = True
                    blocks.append(inner)
                    stack.append(inner.body)
                else:
                    node.else_ = []
                    stack.append(node.else_)
            elif kw == "end":
                if not blocks:
                    raise TemplateError("unexpected {{end}}")
                stack.pop()
                node = blocks.pop()
                while getattr(node, "chained", False):
                    node = blocks.pop()
                if isinstance(node, tuple):          # define
                    self.defines[node[1]] = node[2]
            elif kw == "define":
                name = _go_unquote(toks[1][1])
                body: list = []
                blocks.append(("define", name, body))
                stack.append(body)
            elif kw == "template":
                name = _go_unquote(toks[1][1])
                stack[-1].append(_Template(name, _parse_pipe(toks[2:]) if len(toks) > 2 else None))
            else:
                stack[-1].append(_Action(_parse_pipe(toks)))
        if blocks:
            raise TemplateError("unexpected EOF")
        return stack[0]

    # ------------------------------------------------------------- execution
    def execute(self, data) -> str:
        out: list[str] = []
        self._run(self.root, data, [{"$": data}], out)
        return "".join(out)

    def _run(self, nodes, dot, scopes, out):
        for n in nodes:
            if isinstance(n, _Text):
                out.append(n.text)
            elif isinstance(n, _Action):
                v = self._pipe(n.pipe, dot, scopes)
                if n.pipe.decl is None:
                    out.append(_print(v))
            elif isinstance(n, _If):
                self._block(n, dot, scopes, out)
            elif isinstance(n, _Template):
                body = self.defines.get(n.name)
                if body is None:
                    raise TemplateError(f'template: no template "{n.name}" associated with template "{self.name}"')
                d = self._pipe(n.pipe, dot, scopes) if n.pipe else None
                self._run(body, d, [{"$": d}], out)

    def _block(self, n: _If, dot, scopes, out):
        scopes.append({})
        try:
            v = self._pipe(n.pipe, dot, scopes, declare_only=(n.kind == "range"))
            if n.kind == "if":
                if truth(v):
                    self._run(n.body, dot, scopes, out)
                elif n.else_ is not None:
                    self._run(n.else_, dot, scopes, out)
            elif n.kind == "with":
                if truth(v):
                    self._run(n.body, v, scopes, out)
                elif n.else_ is not None:
                    self._run(n.else_, dot, scopes, out)
            else:
                items = _range_items(v)
                if not items:
                    if n.else_ is not None:
                        self._run(n.else_, dot, scopes, out)
                    return
                names = n.pipe.decl[0] if n.pipe.decl else []
                for k, item in items:
                    scopes.append({})
                    if len(names) == 1:
                        scopes[-1][names[0]] = item
                    elif len(names) == 2:
                        scopes[-1][names[0]], scopes[-1][names[1]] = k, item
                    self._run(n.body, item, scopes, out)
                    scopes.pop()
        finally:
            scopes.pop()

    def _pipe(self, pipe: _Pipe, dot, scopes, declare_only=False):
        val = None
        first = True
        for cmd in pipe.cmds:
            val = self._command(cmd, dot, scopes, None if first else val, not first)
            first = False
        if pipe.decl is not None and not declare_only:
            names, is_decl = pipe.decl
            if is_decl:
                scopes[-1][names[0]] = val
            else:
                for s in reversed(scopes):
                    if names[0] in s:
                        s[names[0]] = val
                        break
                else:
                    raise TemplateError(f"undefined variable: {names[0]}")
        return val

    def _command(self, toks, dot, scopes, piped, has_piped):
        head = toks[0]
        if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
            fn = self.funcs.get(head[1])
            if fn is None:
                raise TemplateError(f'function "{head[1]}" not defined')
            args = self._args(toks[1:], dot, scopes)
            if has_piped:
                args.append(piped)
            return fn(*args)
        args = self._args(toks, dot, scopes)
        if has_piped:
            raise TemplateError(f"can't give argument to non-function {toks[0][1]}")
        if len(args) != 1:
            raise TemplateError(f"can't give argument to non-function {toks[0][1]}")
        return args[0]

    def _args(self, toks, dot, scopes) -> list:
        out, i = [], 0
        while i < len(toks):
            k, v = toks[i]
            if k == "lp":
                depth, j = 1, i + 1
                while j < len(toks) and depth:
                    if toks[j][0] == "lp":
                        depth += 1
                    elif toks[j][0] == "rp":
                        depth -= 1
                    j += 1
                inner = toks[i + 1:j - 1]
                val = self._pipe(_parse_pipe(inner), dot, scopes)
                rp = toks[j - 1][1]
                for f in rp[1:].split(".")[1:] if "." in rp else []:
                    val = self._field(val, f)
                out.append(val)
                i = j
                continue
            out.append(self._operand(k, v, dot, scopes))
            i += 1
        return out

    def _operand(self, k, v, dot, scopes):
        if k in ("str", "raw"):
            return _go_unquote(v)
        if k == "char":
            return ord(_go_unquote(v)) if len(v) == 3 else ord(json.loads('"' + v[1:-1] + '"'))
        if k == "num":
            try:
                return int(v, 0)
            except ValueError:
                return float(v)
        if k == "ident":
            if v == "true":
                return True
            if v == "false":
                return False
            if v == "nil":
                return None
            fn = self.funcs.get(v)
            if fn is None:
                raise TemplateError(f'function "{v}" not defined')
            return fn()
        if k == "var":
            name, *path = v.split(".")
            for s in reversed(scopes):
                if name in s:
                    val = s[name]
                    break
            else:
                raise TemplateError(f"undefined variable: {name}")
            for f in path:
                val = self._field(val, f)
            return val
        if k == "field":
            val = dot
            for f in v.split(".")[1:]:
                if f:
                    val = self._field(val, f)
            return val
        raise TemplateError(f"unexpected {v} in operand")

    def _field(self, val, name):
        if val is NO_VALUE or val is None:
            if self.missingkey == "error":
                raise TemplateError(f"nil data; no entry for key {json.dumps(name)}")
            return NO_VALUE
        if isinstance(val, dict):
            if name in val:
                return val[name]
            if self.missingkey == "error":
                raise TemplateError(f"map has no entry for key {json.dumps(name)}")
            return NO_VALUE
        raise TemplateError(f"can't evaluate field {name} in type {_go_kind(val)}")


def _go_kind(v) -> str:
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int64"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "[]interface {}"
    return "interface {}"


def _print(v) -> str:
    if v is None:
        return "<no value>"
    return go_fmt(v)


def truth(v) -> bool:
    if v is None or v is NO_VALUE:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _range_items(v) -> list:
    if v is None or v is NO_VALUE:
        return []
    if isinstance(v, dict):
        return [(k, v[k]) for k in sorted(v, key=str)]
    if isinstance(v, (list, tuple)):
        return list(enumerate(v))
    raise TemplateError(f"range can't iterate over {go_fmt(v)}")


# ---------------------------------------------------------------------------- functions (funcs.go)
def _and(*args):
    for a in args:
        if not truth(a):
            return a
    return args[-1]


def _or(*args):
    for a in args:
        if truth(a):
            return a
    return args[-1]


def _len(x):
    if isinstance(x, (str, list, dict, tuple)):
        return len(x)
    raise TemplateError(f"len of type {_go_kind(x)}")


def _index(item, *idx):
    v = item
    for i in idx:
        if isinstance(v, dict):
            v = v.get(i, NO_VALUE)
        elif isinstance(v, (list, tuple, str)):
            if not isinstance(i, int) or not 0 <= i < len(v):
                raise TemplateError(f"index out of range: {i}")
            v = v[i]
        elif v is NO_VALUE or v is None:
            raise TemplateError("index of untyped nil")
        else:
            raise TemplateError(f"can't index item of type {_go_kind(v)}")
    return v


def _num(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool)


def _basic_cmp(a, b):
    if _num(a) and _num(b):
        return a, b
    if type(a) is not type(b):
        raise TemplateError("incompatible types for comparison")
    if not isinstance(a, (str, bool, int, float)):
        raise TemplateError("invalid type for comparison")
    return a, b


def _eq(a, *bs):
    for b in bs:
        x, y = _basic_cmp(a, b)
        if x == y:
            return True
    return False


def _lt(a, b):
    x, y = _basic_cmp(a, b)
    if isinstance(x, bool):
        raise TemplateError("invalid type for comparison")
    return x < y


def _sprint(*args) -> str:
    """fmt.Sprint: spaces between operands when neither is a string."""
    out = []
    for i, a in enumerate(args):
        if i and not isinstance(a, str) and not isinstance(args[i - 1], str):
            out.append(" ")
        out.append(_print(a))
    return "".join(out)


_VERB = re.compile(r"%([-+# 0]*)(\d+|\*)?(?:\.(\d+|\*))?([a-zA-Z%])")


def sprintf(fmt: str, *args) -> str:
    """fmt.Sprintf for the verbs templates use: %v %s %d %q %f %e %g %x %X %t %c %%."""
    out, ai, pos = [], 0, 0
    for mt in _VERB.finditer(fmt):
        out.append(fmt[pos:mt.start()])
        pos = mt.end()
        flags, width, prec, verb = mt.groups()
        if verb == "%":
            out.append("%")
            continue
        if ai >= len(args):
            out.append(f"%!{verb}(MISSING)")
            continue
        a = args[ai]
        ai += 1
        if verb in ("v", "s"):
            s = _print(a)
            if prec is not None and verb == "s":
                s = s[:int(prec)]
        elif verb == "d":
            s = str(int(a)) if _num(a) else f"%!d({_go_kind(a)}={_print(a)})"
        elif verb == "q":
            s = json.dumps(a) if isinstance(a, str) else _print(a)
        elif verb in "feEgG":
            p = int(prec) if prec is not None else (6 if verb in "feE" else -1)
            if verb in "gG" and p < 0:
                s = go_fmt(float(a))
            else:
                s = format(float(a), f".{p}{verb}")
        elif verb in "xX":
            s = format(a, verb) if isinstance(a, int) else (a.encode().hex() if isinstance(a, str) else _print(a))
            s = s.upper() if verb == "X" else s
        elif verb == "t":
            s = "true" if a is True else ("false" if a is False else f"%!t({_print(a)})")
        elif verb == "c":
            s = chr(a)
        else:
            s = f"%!{verb}({_print(a)})"
        if width is not None and width != "*":
            w = int(width)
            s = s.ljust(w) if "-" in (flags or "") else (s.rjust(w, "0") if "0" in (flags or "") and verb in "dfeg"
                                                         else s.rjust(w))
        out.append(s)
    out.append(fmt[pos:])
    if ai < len(args):
        out.append("%!(EXTRA " + ", ".join(f"{_go_kind(a)}={_print(a)}" for a in args[ai:]) + ")")
    return "".join(out)


def exists(item, *indices) -> bool:
    """template.go exists: whether the chain of keys / indices leads somewhere."""
    v = item
    for i in indices:
        if isinstance(v, dict):
            if i not in v:
                return False
            v = v[i]
        elif isinstance(v, (list, tuple)) and isinstance(i, int):
            if not 0 <= i < len(v):
                return False
            v = v[i]
        else:
            return False
    return True


BUILTINS = {
    "and": _and, "or": _or, "not": lambda x: not truth(x), "len": _len, "index": _index,
    "print": _sprint, "printf": sprintf, "println": lambda *a: " ".join(_print(x) for x in a) + "\n",
    "eq": _eq, "ne": lambda a, b: not _eq(a, b), "lt": _lt, "le": lambda a, b: _lt(a, b) or _eq(a, b),
    "gt": lambda a, b: not (_lt(a, b) or _eq(a, b)), "ge": lambda a, b: not _lt(a, b),
    "html": lambda *a: _html.escape(_sprint(*a), quote=True).replace("&#x27;", "&#39;"),
    "js": lambda *a: json.dumps(_sprint(*a))[1:-1].replace("'", "\\'"),
    "urlquery": lambda *a: urllib.parse.quote_plus(_sprint(*a)),
    "exists": exists,
}


def render(text: str, data, allow_missing_keys: bool = True) -> str:
    return Template(text, missingkey="default" if allow_missing_keys else "error").execute(data)
