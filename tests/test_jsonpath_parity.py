"""kubectl's JSONPath held to client-go util/jsonpath's tests, transcribed:

* parser_test.go TestParser (:29-75, every case's node list compared by String()) and
  TestFailParser (:127);
* jsonpath_test.go TestStructInput (:119, Go structs stood in by dataclasses with the same
  fields and String methods), TestJSONInput (:185), TestKubernetes (:207, incl. the sorted
  recursive-name case), TestFilterPartialMatchesSometimesMissingAnnotations (:290);
* the verdict's probe: `{range .items[*]}…{end}`, `[?(@.status.phase=="Running")]` and escaped
  keys such as `amd\\.com/gpu-type`.
"""
import dataclasses
import json

import pytest

from amdkube.kubectl import jsonpath as jp


# ---------------------------------------------------------------------------- parser
def nodes_of(text):
    return [str(n) for n in jp.collect_nodes(jp.parse(text).root)[1:]]


L = "NodeList"


def F(v):
    return f"NodeField: {v}"


def T(v):
    return f"NodeText: {v}"


def A(a, b, c):
    f = lambda p: f"{{{p[0]} {'true' if p[1] else 'false'}}}"   # noqa: E731
    return f"NodeArray: [{f(a)} {f(b)} {f(c)}]"


FILT_EQ = "NodeFilter: NodeList == NodeList"
PARSER_CASES = [
    ("plain", "hello jsonpath", [T("hello jsonpath")]),
    ("variable", "hello {.jsonpath}", [T("hello "), L, F("jsonpath")]),
    ("arrayfiled", "hello {['jsonpath']}", [T("hello "), L, F("jsonpath")]),
    ("quote", '{"{"}', [L, T("{")]),
    ("array", "{[1:3]}", [L, A((1, True), (3, True), (0, False))]),
    ("allarray", "{.book[*].author}", [L, F("book"), A((0, False), (0, False), (0, False)), F("author")]),
    ("wildcard", "{.bicycle.*}", [L, F("bicycle"), "NodeWildcard"]),
    ("filter", "{[?(@.price<3)]}", [L, "NodeFilter: NodeList < NodeList", L, F("price"), L, "NodeInt: 3"]),
    ("recursive", "{..}", [L, "NodeRecursive"]),
    ("recurField", "{..price}", [L, "NodeRecursive", F("price")]),
    ("arraydict", "{['book.price']}", [L, F("book"), F("price")]),
    ("union", "{['bicycle.price', 3, 'book.price']}", [L, "NodeUnion", L, F("bicycle"), F("price"), L,
                                                       A((3, True), (4, True), (0, False)), L, F("book"), F("price")]),
    ("range", "{range .items}{.name},{end}", [L, "NodeIdentifier: range", F("items"), L, F("name"), T(","), L,
                                               "NodeIdentifier: end"]),
    ("paired parentheses in quotes", '{[?(@.status.nodeInfo.osImage == "()")]}',
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T("()")]),
    ("paired parentheses in double quotes and with double quotes escape", r'{[?(@.status.nodeInfo.osImage == "(\"\")")]}',
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T('("")')]),
    ("unregular parentheses in double quotes", '{[?(@.test == "())(")]}', [L, FILT_EQ, L, F("test"), L, T("())(")]),
    ("plain text in single quotes", "{[?(@.status.nodeInfo.osImage == 'Linux')]}",
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T("Linux")]),
    ("test filter suffix", '{[?(@.status.nodeInfo.osImage == "{[()]}")]}',
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T("{[()]}")]),
    ("double inside single", """{[?(@.status.nodeInfo.osImage == "''")]}""",
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T("''")]),
    ("single inside double", """{[?(@.status.nodeInfo.osImage == '""')]}""",
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T('""')]),
    ("single containing escaped single", r"{[?(@.status.nodeInfo.osImage == '\\\'')]}",
     [L, FILT_EQ, L, F("status"), F("nodeInfo"), F("osImage"), L, T("\\'")]),
]


@pytest.mark.parametrize("name,text,expected", PARSER_CASES, ids=[c[0] for c in PARSER_CASES])
def test_parser(name, text, expected):
    assert nodes_of(text) == expected


def test_parser_malformed_input():
    with pytest.raises(jp.JSONPathError):
        jp.parse(r"{\\\}")


@pytest.mark.parametrize("text,err", [
    ("{.hello", "unclosed action"),
    ("{*}", "unrecognized character in action: U+002A '*'"),
    ("{+12.3.0}", "cannot parse number +12.3.0"),
    ("{[1}", "unterminated array"),
    ("{[::-1]}", "invalid array index ::-1"),
    ("{[?(.price]}", "unterminated filter"),
])
def test_fail_parser(text, err):
    with pytest.raises(jp.JSONPathError) as ei:
        jp.parse(text)
    assert str(ei.value) == err


# ---------------------------------------------------------------------------- evaluation
@dataclasses.dataclass
class Book:
    Category: str
    Author: str
    Title: str
    Price: float

    def go_string(self):
        return f"{{Category: {self.Category}, Author: {self.Author}, Title: {self.Title}, Price: {jp.go_fmt(self.Price)}}}"


@dataclasses.dataclass
class Bicycle:
    Color: str
    Price: float
    IsNew: bool


class GoMap(dict):
    def __init__(self, go_type, *a):
        super().__init__(*a)
        self.go_type = go_type


@dataclasses.dataclass
class Store:
    Book: list
    Bicycle: list
    Name: str
    Labels: dict
    Employees: dict


STORE = Store(
    Book=[Book("reference", "Nigel Rees", "Sayings of the Centurey", 8.95), Book("fiction", "Evelyn Waugh", "Sword of Honour", 12.99),
          Book("fiction", "Herman Melville", "Moby Dick", 8.99)],
    Bicycle=[Bicycle("red", 19.95, True), Bicycle("green", 20.01, False)],
    Name="jsonpath",
    Labels=GoMap("map[string]int", {"engieer": 10, "web/html": 15, "k8s-app": 20}),
    Employees=GoMap("map[main.empName]main.job", {"jason": "manager", "dan": "clerk"}))


def run(template, data, allow_missing=False):
    return jp.JSONPath("t", allow_missing).parse(template).execute(data)


STORE_CASES = [
    ("plain", "hello jsonpath", None, "hello jsonpath"),
    ("recursive", "{..}", [1, 2, 3], "[1 2 3]"),
    ("filter", "{[?(@<5)]}", [2, 6, 3, 7], "2 3"),
    ("quote", '{"{"}', None, "{"),
    ("union", "{[1,3,4]}", [0, 1, 2, 3, 4], "1 3 4"),
    ("array", "{[0:2]}", ["Monday", "Tudesday"], "Monday Tudesday"),
    ("variable", "hello {.Name}", STORE, "hello jsonpath"),
    ("dict/", "{$.Labels.web/html}", STORE, "15"),
    ("dict/", "{$.Employees.jason}", STORE, "manager"),
    ("dict/", "{$.Employees.dan}", STORE, "clerk"),
    ("dict-", "{.Labels.k8s-app}", STORE, "20"),
    ("nest", "{.Bicycle[*].Color}", STORE, "red green"),
    ("allarray", "{.Book[*].Author}", STORE, "Nigel Rees Evelyn Waugh Herman Melville"),
    ("allfileds", "{.Bicycle.*}", STORE, "{red 19.95 true} {green 20.01 false}"),
    ("recurfileds", "{..Price}", STORE, "8.95 12.99 8.99 19.95 20.01"),
    ("lastarray", "{.Book[-1:]}", STORE, "{Category: fiction, Author: Herman Melville, Title: Moby Dick, Price: 8.99}"),
    ("recurarray", "{..Book[2]}", STORE, "{Category: fiction, Author: Herman Melville, Title: Moby Dick, Price: 8.99}"),
    ("bool", "{.Bicycle[?(@.IsNew==true)]}", STORE, "{red 19.95 true}"),
]


@pytest.mark.parametrize("name,template,data,expected", STORE_CASES, ids=[f"{i}-{c[0]}" for i, c in enumerate(STORE_CASES)])
def test_struct_input(name, template, data, expected):
    assert run(template, data) == expected


def test_struct_input_missing_key_allowed():
    assert run("{.hello}", STORE, allow_missing=True) == ""


@pytest.mark.parametrize("template,err", [
    ("{hello}", "unrecognized identifier hello"),
    ("{.hello}", "hello is not found"),
    ("{.Labels[0]}", "map[string]int is not array or slice"),
    ("{.Book[?(@.Price<>10)]}", "unrecognized filter operator <>"),
    ("{range .Labels.*}{@}{end}{end}", "not in range, nothing to end"),
])
def test_struct_input_failures(template, err):
    with pytest.raises(jp.JSONPathError) as ei:
        run(template, STORE)
    assert str(ei.value) == err


POINTS = json.loads("""[
    {"id": "i1", "x":4, "y":-5}, {"id": "i2", "x":-2, "y":-5, "z":1}, {"id": "i3", "x":  8, "y":  3 },
    {"id": "i4", "x": -6, "y": -1 }, {"id": "i5", "x":  0, "y":  2, "z": 1 }, {"id": "i6", "x":  1, "y":  4 }]""")


def test_json_input():
    assert run("{[?(@.z)].id}", POINTS) == "i2 i5"
    assert run("{[0]['id']}", POINTS) == "i1"


NODES = json.loads("""{
  "kind": "List",
  "items":[
    {"kind":"None", "metadata":{"name":"127.0.0.1", "labels":{"kubernetes.io/hostname":"127.0.0.1"}},
     "status":{"capacity":{"cpu":"4"}, "ready": true, "addresses":[{"type": "LegacyHostIP", "address":"127.0.0.1"}]}},
    {"kind":"None", "metadata":{"name":"127.0.0.2", "labels":{"kubernetes.io/hostname":"127.0.0.2"}},
     "status":{"capacity":{"cpu":"8"}, "ready": false,
               "addresses":[{"type": "LegacyHostIP", "address":"127.0.0.2"}, {"type": "another", "address":"127.0.0.3"}]}}
  ],
  "users":[{"name": "myself", "user": {}}, {"name": "e2e", "user": {"username": "admin", "password": "secret"}}]
}""")

K8S_CASES = [
    ("range item", "{range .items[*]}{.metadata.name}, {end}{.kind}", "127.0.0.1, 127.0.0.2, List"),
    ("range item with quote", '{range .items[*]}{.metadata.name}{"\\t"}{end}', "127.0.0.1\t127.0.0.2\t"),
    ("range addresss", "{.items[*].status.addresses[*].address}", "127.0.0.1 127.0.0.2 127.0.0.3"),
    ("double range", "{range .items[*]}{range .status.addresses[*]}{.address}, {end}{end}",
     "127.0.0.1, 127.0.0.2, 127.0.0.3, "),
    ("item name", "{.items[*].metadata.name}", "127.0.0.1 127.0.0.2"),
    ("union nodes capacity", "{.items[*]['metadata.name', 'status.capacity']}",
     "127.0.0.1 127.0.0.2 map[cpu:4] map[cpu:8]"),
    ("range nodes capacity", "{range .items[*]}[{.metadata.name}, {.status.capacity}] {end}",
     "[127.0.0.1, map[cpu:4]] [127.0.0.2, map[cpu:8]] "),
    ("user password", '{.users[?(@.name=="e2e")].user.password}', "secret"),
    ("hostname", r"{.items[0].metadata.labels.kubernetes\.io/hostname}", "127.0.0.1"),
    ("hostname filter", r'{.items[?(@.metadata.labels.kubernetes\.io/hostname=="127.0.0.1")].kind}', "None"),
    ("bool item", "{.items[?(@..ready==true)].metadata.name}", "127.0.0.1"),
]


@pytest.mark.parametrize("name,template,expected", K8S_CASES, ids=[c[0] for c in K8S_CASES])
def test_kubernetes(name, template, expected):
    assert run(template, NODES) == expected


def test_kubernetes_recursive_name_any_order():
    assert sorted(run("{..name}", NODES).split()) == sorted("127.0.0.1 127.0.0.2 myself e2e".split())


ANNOTATED = {"kind": "List", "items": [
    {"kind": "Pod", "metadata": {"name": "pod1", "annotations": {"color": "blue"}}},
    {"kind": "Pod", "metadata": {"name": "pod2"}},
    {"kind": "Pod", "metadata": {"name": "pod3", "annotations": {"color": "green"}}},
    {"kind": "Pod", "metadata": {"name": "pod4", "annotations": {"color": "blue"}}}]}


def test_filter_partial_matches_sometimes_missing_annotations():
    tpl = '{.items[?(@.metadata.annotations.color=="blue")].metadata.name}'
    assert run(tpl, ANNOTATED, allow_missing=True) == "pod1 pod4"
    with pytest.raises(jp.JSONPathError):
        run(tpl, ANNOTATED, allow_missing=False)


# ---------------------------------------------------------------------------- the verdict's probe
PODS = {"kind": "List", "items": [
    {"metadata": {"name": "a"}, "status": {"phase": "Running"},
     "spec": {"extendedResources": [{"name": "gpus", "assigned": ["GPU-0", "GPU-1"]}]},
     "node": {"labels": {"amd.com/gpu-type": "MI355X"}}},
    {"metadata": {"name": "b"}, "status": {"phase": "Pending"}, "spec": {}},
]}


def test_range_filters_and_escaped_keys():
    assert run('{range .items[*]}{.metadata.name}{"\\t"}{.spec.extendedResources[*].assigned}{"\\n"}{end}', PODS,
               allow_missing=True) == "a\t[GPU-0 GPU-1]\nb\t\n"
    assert run('{.items[?(@.status.phase=="Running")].metadata.name}', PODS) == "a"
    assert run(r"{.items[0].node.labels.amd\.com/gpu-type}", PODS) == "MI355X"


@pytest.mark.parametrize("value,text", [(1e6, "1e+06"), (123456.0, "123456"), (0.5, "0.5"), (1.25e-5, "1.25e-05"),
                                        (2.0, "2"), (-3.75, "-3.75"), (7, "7"), (True, "true")])
def test_values_print_like_go(value, text):
    assert jp.go_fmt(value) == text


@pytest.mark.parametrize("inp,out,err", [
    ("foo.bar", "{.foo.bar}", False), ("{foo.bar}", "{.foo.bar}", False), (".foo.bar", "{.foo.bar}", False),
    ("{.foo.bar}", "{.foo.bar}", False), ("", "", False), ("{foo.bar", None, True), ("foo.bar}", None, True),
    ("{foo.bar}}", None, True), ("{{foo.bar}", None, True)])
def test_massage_json_path(inp, out, err):
    """customcolumn_test.go TestMassageJSONPath (:33)."""
    if err:
        with pytest.raises(jp.JSONPathError):
            jp.relaxed_expression(inp)
    else:
        assert jp.relaxed_expression(inp) == out
