"""JSONPath templates for `kubectl -o jsonpath=…`, `custom-columns` and `--sort-by`.

Reference: staging/src/k8s.io/client-go/util/jsonpath/ — parser.go (the text / action lexer:
fields with `\\.` escapes, `..` recursive descent, `[start:end:step]` slices, `[*]`, unions
`[a,b]`, `['key']`, filters `[?(@.x == "y")]`, quoted strings, numbers, booleans and the
`range`/`end` identifiers), node.go (the node types and their String forms, which the parser
tests compare), jsonpath.go (FindResults: range blocks re-run the rest of the template once
per element; evaluation of every node kind; AllowMissingKeys; PrintResults joining a result
list with spaces).

Values print as Go's fmt `%v` prints the decoded JSON the reference walks: maps as
`map[k:v …]` with sorted keys, lists as `[a b]`, floats in strconv's shortest `%g` form.
Filters compare numbers numerically whatever their JSON type (the reference's text/template
comparison refuses float64 against an int literal, so `[?(@.spec.replicas>1)]` errors there).
"""
from __future__ import annotations

import dataclasses
import re
from decimal import Decimal

__all__ = ["JSONPath", "JSONPathError", "parse", "go_fmt", "relaxed_expression"]


class JSONPathError(Exception):
    pass


# ---------------------------------------------------------------------------- nodes (node.go)
class Node:
    type_name = ""

    def __str__(self):
        return self.type_name


class ListNode(Node):
    type_name = "NodeList"

    def __init__(self):
        self.nodes: list = []


class TextNode(Node):
    type_name = "NodeText"

    def __init__(self, text):
        self.text = text

    def __str__(self):
        return f"{self.type_name}: {self.text}"


class FieldNode(Node):
    type_name = "NodeField"

    def __init__(self, value):
        self.value = value

    def __str__(self):
        return f"{self.type_name}: {self.value}"


class IdentifierNode(Node):
    type_name = "NodeIdentifier"

    def __init__(self, name):
        self.name = name

    def __str__(self):
        return f"{self.type_name}: {self.name}"


class ArrayNode(Node):
    type_name = "NodeArray"

    def __init__(self, params):
        self.params = params        # [(value, known)] * 3: start, end, step

    def __str__(self):
        return f"{self.type_name}: [" + " ".join(f"{{{v} {'true' if k else 'false'}}}" for v, k in self.params) + "]"


class FilterNode(Node):
    type_name = "NodeFilter"

    def __init__(self, left, right, op):
        self.left, self.right, self.op = left, right, op

    def __str__(self):
        return f"{self.type_name}: {self.left} {self.op} {self.right}"


class IntNode(Node):
    type_name = "NodeInt"

    def __init__(self, value):
        self.value = value

    def __str__(self):
        return f"{self.type_name}: {self.value}"


class FloatNode(Node):
    type_name = "NodeFloat"

    def __init__(self, value):
        self.value = value

    def __str__(self):
        return f"{self.type_name}: {self.value:f}"


class WildcardNode(Node):
    type_name = "NodeWildcard"


class RecursiveNode(Node):
    type_name = "NodeRecursive"


class UnionNode(Node):
    type_name = "NodeUnion"

    def __init__(self, nodes):
        self.nodes = nodes


class BoolNode(Node):
    type_name = "NodeBool"

    def __init__(self, value):
        self.value = value

    def __str__(self):
        return f"{self.type_name}: {'true' if self.value else 'false'}"


# ---------------------------------------------------------------------------- parser (parser.go)
_DICT_KEY = re.compile(r"^'([^']*)'$")
_SLICE = re.compile(r"^(-?[\d]*)(:-?[\d]*)?(:[\d]*)?$")
_FILTER = re.compile(r"^([^!<>=]+)([!<>=]+)(.+?)$", re.S)
EOF = ""


def _is_terminator(r: str) -> bool:
    return r in (EOF, " ", "\t", "\r", "\n", ".", ",", "[", "]", "$", "@", "{", "}")


def _is_alnum(r: str) -> bool:
    return r == "_" or r.isalpha() or r.isdigit()


def _unquote_extend(s: str) -> str:
    """UnquoteExtend: a single- or double-quoted string with Go escapes."""
    if len(s) < 2 or s[0] != s[-1] or s[0] not in "\"'":
        raise JSONPathError("invalid syntax")
    body, q = s[1:-1], s[0]
    if "\\" not in body and q not in body:
        return body
    out, i = [], 0
    simple = {"a": "\a", "b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v", "\\": "\\", "'": "'",
              '"': '"'}
    while i < len(body):
        c = body[i]
        if c == q:
            raise JSONPathError("invalid syntax")
        if c != "\\":
            out.append(c)
            i += 1
            continue
        if i + 1 >= len(body):
            raise JSONPathError("invalid syntax")
        e = body[i + 1]
        if e in simple:
            if (e == "'" and q == '"') or (e == '"' and q == "'"):
                raise JSONPathError("invalid syntax")
            out.append(simple[e])
            i += 2
        elif e in "xuU":
            n = {"x": 2, "u": 4, "U": 8}[e]
            out.append(chr(int(body[i + 2:i + 2 + n], 16)))
            i += 2 + n
        elif e in "01234567":
            out.append(chr(int(body[i + 1:i + 4], 8)))
            i += 4
        else:
            raise JSONPathError("invalid syntax")
    return "".join(out)


class Parser:
    def __init__(self, name=""):
        self.name = name
        self.root = ListNode()
        self.input = ""
        self.pos = self.start = self.width = 0

    def parse(self, text: str):
        self.input, self.root, self.pos, self.start = text, ListNode(), 0, 0
        self._parse_text(self.root)
        return self

    # ------------------------------------------------------------- lexer
    def _consume(self) -> str:
        v = self.input[self.start:self.pos]
        self.start = self.pos
        return v

    def _next(self) -> str:
        if self.pos >= len(self.input):
            self.width = 0
            return EOF
        self.width = 1
        self.pos += 1
        return self.input[self.pos - 1]

    def _peek(self) -> str:
        r = self._next()
        self._backup()
        return r

    def _backup(self):
        self.pos -= self.width

    # ------------------------------------------------------------- grammar
    def _parse_text(self, cur: ListNode):
        while True:
            if self.input.startswith("{", self.pos):
                if self.pos > self.start:
                    cur.nodes.append(TextNode(self._consume()))
                return self._parse_left_delim(cur)
            if self._next() == EOF:
                break
        if self.pos > self.start:
            cur.nodes.append(TextNode(self._consume()))

    def _parse_left_delim(self, cur):
        self.pos += 1
        self._consume()
        node = ListNode()
        cur.nodes.append(node)
        return self._parse_inside_action(node)

    def _parse_inside_action(self, cur):
        while True:
            rest = self.input[self.pos:]
            if rest.startswith("}"):
                self.pos += 1
                self._consume()
                return self._parse_text(self.root)
            if rest.startswith("[?("):
                cur = self._parse_filter(cur)
                continue
            if rest.startswith(".."):
                self.pos += 2
                self._consume()
                cur.nodes.append(RecursiveNode())
                if _is_alnum(self._peek()):
                    self._parse_field(cur)
                continue
            r = self._next()
            if r == EOF or r in "\r\n":
                raise JSONPathError("unclosed action")
            if r == " ":
                self._consume()
            elif r in "@$":
                self._consume()
            elif r == "[":
                self._parse_array(cur)
            elif r in "\"'":
                self._parse_quote(cur, r)
            elif r == ".":
                self._parse_field(cur)
            elif r in "+-" or r.isdigit():
                self._backup()
                self._parse_number(cur)
            elif _is_alnum(r):
                self._backup()
                self._parse_identifier(cur)
            else:
                raise JSONPathError(f"unrecognized character in action: U+{ord(r):04X} {_go_quote_rune(r)}")

    def _parse_identifier(self, cur):
        while True:
            r = self._next()
            if _is_terminator(r):
                self._backup() if r != EOF else None
                break
        value = self._consume()
        if value in ("true", "false"):
            cur.nodes.append(BoolNode(value == "true"))
        else:
            cur.nodes.append(IdentifierNode(value))

    def _parse_number(self, cur):
        r = self._peek()
        if r in "+-":
            self._next()
        while True:
            r = self._next()
            if r != "." and not r.isdigit():
                if r != EOF:
                    self._backup()
                break
        value = self._consume()
        try:
            cur.nodes.append(IntNode(int(value)))
            return
        except ValueError:
            pass
        try:
            if value.count(".") <= 1:
                cur.nodes.append(FloatNode(float(value)))
                return
        except ValueError:
            pass
        raise JSONPathError(f"cannot parse number {value}")

    def _parse_array(self, cur):
        while True:
            r = self._next()
            if r in (EOF, "\n"):
                raise JSONPathError("unterminated array")
            if r == "]":
                break
        text = self._consume()[1:-1]
        if text == "*":
            text = ":"
        parts = text.split(",")
        if len(parts) > 1:
            union = []
            for s in parts:
                union.append(_parse_action("union", f"[{s.strip(' ')}]"))
            cur.nodes.append(UnionNode(union))
            return
        mt = _DICT_KEY.match(text)
        if mt:
            cur.nodes.extend(_parse_action("arraydict", f".{mt.group(1)}").nodes)
            return
        mt = _SLICE.match(text)
        if mt is None:
            raise JSONPathError(f"invalid array index {text}")
        vals = list(mt.groups())
        params = [(0, False)] * 3
        for i in range(3):
            v = vals[i] or ""
            if v != "":
                if i > 0:
                    v = v[1:]
                if i > 0 and v == "":
                    params[i] = (0, False)
                else:
                    try:
                        params[i] = (int(v), True)
                    except ValueError:
                        raise JSONPathError(f"array index {v} is not a number") from None
            elif i == 1:
                params[i] = (params[0][0] + 1, True)
            else:
                params[i] = (0, False)
        cur.nodes.append(ArrayNode(params))

    def _parse_filter(self, cur):
        self.pos += 3
        self._consume()
        begin = end = False
        pair = ""
        while True:
            r = self._next()
            if r in (EOF, "\n"):
                raise JSONPathError("unterminated filter")
            if r in "\"'":
                if not begin:
                    begin, pair = True, r
                    continue
                if self.input[self.pos - 2] != "\\" and r == pair:
                    end = True
            elif r == ")":
                if begin == end:
                    break
        if self._next() != "]":
            raise JSONPathError("unclosed array expect ]")
        text = self._consume()[:-2]
        mt = _FILTER.match(text)
        if mt is None:
            cur.nodes.append(FilterNode(_parse_action("text", text), ListNode(), "exists"))
        else:
            cur.nodes.append(FilterNode(_parse_action("left", mt.group(1)), _parse_action("right", mt.group(3)),
                                        mt.group(2)))
        return cur

    def _parse_quote(self, cur, end):
        while True:
            r = self._next()
            if r in (EOF, "\n"):
                raise JSONPathError("unterminated quoted string")
            if r == end and self.input[self.pos - 2] != "\\":
                break
        value = self._consume()
        try:
            cur.nodes.append(TextNode(_unquote_extend(value)))
        except (JSONPathError, ValueError) as e:
            raise JSONPathError(f"unquote string {value} error {e}") from None

    def _parse_field(self, cur):
        self._consume()
        while True:
            r = self._next()
            if r == "\\":
                self._next()
            elif _is_terminator(r):
                if r != EOF:
                    self._backup()
                break
        value = self._consume()
        if value == "*":
            cur.nodes.append(WildcardNode())
        else:
            cur.nodes.append(FieldNode(value.replace("\\", "")))


def _go_quote_rune(r: str) -> str:
    return "'" + r + "'" if r.isprintable() else repr(r)


def _parse_action(name, text) -> ListNode:
    p = Parser(name).parse("{" + text + "}")
    return p.root.nodes[0]


def parse(text: str, name: str = "") -> Parser:
    return Parser(name).parse(text)


def collect_nodes(root: ListNode) -> list:
    """parser_test.go collectNode: the tree in pre-order (root excluded by callers)."""
    out = []

    def walk(n):
        out.append(n)
        if isinstance(n, ListNode):
            for c in n.nodes:
                walk(c)
        elif isinstance(n, FilterNode):
            walk(n.left)
            walk(n.right)
        elif isinstance(n, UnionNode):
            for c in n.nodes:
                walk(c)
    walk(root)
    return out


# ---------------------------------------------------------------------------- values
class _Missing:
    pass


def _is_struct(v) -> bool:
    return dataclasses.is_dataclass(v) and not isinstance(v, type)


def go_type(v) -> str:
    """The Go type a decoded value would have (error messages)."""
    t = getattr(v, "go_type", None)
    if t:
        return t
    if isinstance(v, dict):
        return "map[string]interface {}"
    if isinstance(v, (list, tuple)):
        return "[]interface {}"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int64"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if v is None:
        return "<nil>"
    return type(v).__name__


def go_float(f: float) -> str:
    """fmt's %v for a float64, strconv.FormatFloat(f, 'g', -1, 64): the shortest digits, in
    exponent form when the exponent is below -4 or at least 6 (1e+06)."""
    if f != f:
        return "NaN"
    if f in (float("inf"), float("-inf")):
        return "+Inf" if f > 0 else "-Inf"
    if f == 0:
        return "-0" if str(f).startswith("-") else "0"
    sign, digits, exp = Decimal(repr(f)).normalize().as_tuple()
    ds = "".join(map(str, digits))
    dp = len(ds) + exp              # decimal point position
    x = dp - 1
    s = "-" if sign else ""
    if x < -4 or x >= 6:
        mant = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
        return f"{s}{mant}e{'-' if x < 0 else '+'}{abs(x):02d}"
    if dp <= 0:
        return f"{s}0.{'0' * -dp}{ds}"
    if dp >= len(ds):
        return s + ds + "0" * (dp - len(ds))
    return f"{s}{ds[:dp]}.{ds[dp:]}"


def go_fmt(v) -> str:
    """fmt.Sprint(v) for decoded JSON values (and the dataclass stand-ins of Go structs)."""
    if hasattr(v, "go_string"):
        return v.go_string()
    if v is None:
        return "<nil>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return go_float(v)
    if isinstance(v, str):
        return v
    if isinstance(v, dict):
        return "map[" + " ".join(f"{go_fmt(k)}:{go_fmt(v[k])}" for k in sorted(v, key=str)) + "]"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(go_fmt(x) for x in v) + "]"
    if _is_struct(v):
        return "{" + " ".join(go_fmt(getattr(v, f.name)) for f in dataclasses.fields(v)) + "}"
    return str(v)


def _num(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _compare(op, a, b) -> bool:
    """text/template eq/ne/lt/le/gt/ge over basic kinds (numbers compared numerically)."""
    if _num(a) and _num(b):
        pass
    elif type(a) is not type(b) or not isinstance(a, (str, bool, int, float)):
        if op in ("==", "!="):
            if isinstance(a, bool) != isinstance(b, bool) or isinstance(a, str) != isinstance(b, str):
                raise JSONPathError("incompatible types for comparison")
        else:
            raise JSONPathError("incompatible types for comparison")
    if isinstance(a, bool) and op not in ("==", "!="):
        raise JSONPathError("invalid type for comparison")
    if op == "==":
        return a == b
    if op == "!=":
        return a != b
    if op == "<":
        return a < b
    if op == ">":
        return a > b
    if op == "<=":
        return a <= b
    if op == ">=":
        return a >= b
    raise JSONPathError(f"unrecognized filter operator {op}")


# ---------------------------------------------------------------------------- evaluator (jsonpath.go)
class JSONPath:
    def __init__(self, name: str = "", allow_missing_keys: bool = False):
        self.name = name
        self.allow_missing_keys = allow_missing_keys
        self.parser: Parser | None = None
        self.stack: list = []
        self.cur: list = []
        self.begin_range = self.in_range = self.end_range = 0

    def parse(self, text: str):
        self.parser = parse(text, self.name)
        return self

    def execute(self, data) -> str:
        out = []
        for results in self.find_results(data):
            out.append(" ".join(go_fmt(r) for r in results))
        return "".join(out)

    def find_results(self, data) -> list[list]:
        if self.parser is None:
            raise JSONPathError(f"{self.name} is an incomplete jsonpath template")
        return self._find(data, self.parser.root.nodes)

    def _find(self, data, nodes) -> list[list]:
        self.cur = [data]
        full = []
        for i, node in enumerate(nodes):
            results = self._walk(self.cur, node)
            if 0 < self.end_range <= self.in_range:
                self.end_range -= 1
                break
            if self.begin_range > 0:
                self.begin_range -= 1
                self.in_range += 1
                for k, value in enumerate(results):
                    if k == len(results) - 1:
                        self.in_range -= 1
                    full.extend(self._find(value, nodes[i + 1:]))
                break
            full.append(results)
        return full

    def _walk(self, value: list, node) -> list:
        if isinstance(node, ListNode):
            cur = value
            for n in node.nodes:
                cur = self._walk(cur, n)
            return cur
        if isinstance(node, TextNode):
            return [node.text]
        if isinstance(node, FieldNode):
            return self._eval_field(value, node)
        if isinstance(node, ArrayNode):
            return self._eval_array(value, node)
        if isinstance(node, FilterNode):
            return self._eval_filter(value, node)
        if isinstance(node, (IntNode, FloatNode, BoolNode)):
            return [node.value for _ in value]
        if isinstance(node, WildcardNode):
            return self._eval_wildcard(value)
        if isinstance(node, RecursiveNode):
            return self._eval_recursive(value)
        if isinstance(node, UnionNode):
            out = []
            for ln in node.nodes:
                out.extend(self._walk(value, ln))
            return out
        if isinstance(node, IdentifierNode):
            return self._eval_identifier(value, node)
        raise JSONPathError(f"unexpected Node {node}")

    def _eval_identifier(self, value, node):
        if node.name == "range":
            self.stack.append(self.cur)
            self.begin_range += 1
            return value
        if node.name == "end":
            if self.end_range < self.in_range:
                self.end_range += 1
                return []
            if self.stack:
                self.cur = self.stack.pop()
                return []
            raise JSONPathError("not in range, nothing to end")
        raise JSONPathError(f"unrecognized identifier {node.name}")

    def _eval_field(self, value, node):
        results = []
        if not value:
            return results
        for v in value:
            if v is None:
                continue
            if isinstance(v, dict):
                if node.value in v:
                    results.append(v[node.value])
            elif _is_struct(v):
                if hasattr(v, node.value):
                    results.append(getattr(v, node.value))
        if not results:
            if self.allow_missing_keys:
                return results
            raise JSONPathError(f"{node.value} is not found")
        return results

    def _eval_array(self, value, node):
        out = []
        for v in value:
            if v is None:
                continue
            if not isinstance(v, (list, tuple)):
                raise JSONPathError(f"{go_type(v)} is not array or slice")
            (s, sk), (e, ek), (st, stk) = node.params
            n = len(v)
            if not sk:
                s = 0
            if s < 0:
                s += n
            if not ek:
                e = n
            if e < 0:
                e += n
            if e != s:
                if s >= n or s < 0:
                    raise JSONPathError(f"array index out of bounds: index {s}, length {n}")
                if e > n or e < 0:
                    raise JSONPathError(f"array index out of bounds: index {e - 1}, length {n}")
            out.extend(v[s:e] if not stk else v[s:e:st if st else None])
        return out

    @staticmethod
    def _children(v) -> list:
        if isinstance(v, dict):
            return list(v.values())
        if isinstance(v, (list, tuple)):
            return list(v)
        if isinstance(v, str):
            return list(v)
        if _is_struct(v):
            return [getattr(v, f.name) for f in dataclasses.fields(v)]
        return []

    def _eval_wildcard(self, value):
        out = []
        for v in value:
            if v is not None:
                out.extend(self._children(v))
        return out

    def _eval_recursive(self, value):
        out = []
        for v in value:
            if v is None:
                continue
            kids = [] if isinstance(v, str) else self._children(v)
            if kids:
                out.append(v)
                out.extend(self._eval_recursive(kids))
        return out

    def _eval_filter(self, value, node):
        out = []
        for v in value:
            if not isinstance(v, (list, tuple)):
                raise JSONPathError(f"{go_fmt(v)} is not array or slice and cannot be filtered")
            for item in v:
                try:
                    lefts = self._walk([item], node.left)
                    err = None
                except JSONPathError as e:
                    lefts, err = [], e
                if node.op == "exists":
                    if lefts:
                        out.append(item)
                    continue
                if err is not None:
                    raise err
                if not lefts:
                    continue
                if len(lefts) > 1:
                    raise JSONPathError("can only compare one element at a time")
                rights = self._walk([item], node.right)
                if not rights:
                    continue
                if len(rights) > 1:
                    raise JSONPathError("can only compare one element at a time")
                if node.op not in ("<", ">", "==", "!=", "<=", ">="):
                    raise JSONPathError(f"unrecognized filter operator {node.op}")
                if _compare(node.op, lefts[0], rights[0]):
                    out.append(item)
        return out


def execute(template: str, data, allow_missing_keys: bool = True) -> str:
    return JSONPath("", allow_missing_keys).parse(template).execute(data)


_RELAXED = re.compile(r"^\{\.?([^{}]+)\}$|^\.?([^{}]+)$")


def relaxed_expression(path: str) -> str:
    """customcolumn.go RelaxedJSONPathExpression: 'a.b', '.a.b', '{a.b}' → '{.a.b}'."""
    if not path:
        return path
    mt = _RELAXED.match(path)
    if mt is None:
        raise JSONPathError("unexpected path string, expected a 'name1.name2' or '.name1.name2' or '{name1.name2}' "
                            "or '{.name1.name2}'")
    return "{." + (mt.group(1) or mt.group(2)) + "}"
