"""Derive amdkube's protobuf wire table from the reference's generated.proto files.

The Kubernetes protobuf encoding of API objects (`application/vnd.kubernetes.protobuf`, the
etcd3 storage format) is defined by the gogo-generated proto2 schemas under
staging/src/k8s.io/{api,apimachinery,apiextensions-apiserver,kube-aggregator}. amdkube keeps
only what the wire needs — per message: field name, number, label and type — in
amdkube/api/proto/k8s_wire.json, and builds descriptors from it at import time
(amdkube/api/protobuf.py). Comments and gogo options are not carried.

  python hack/gen_proto_tables.py /root/reference
"""
import glob
import json
import os
import re
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amdkube", "api", "proto", "k8s_wire.json")
TOK = re.compile(r"\s*(//[^\n]*|/\*.*?\*/|\"[^\"]*\"|'[^']*'|[A-Za-z_][A-Za-z0-9_.]*|\d+|[{}()<>;=,\[\]])", re.S)
SCALARS = {"double", "float", "int64", "uint64", "int32", "uint32", "bool", "string", "bytes", "sint32", "sint64",
           "fixed64", "fixed32", "sfixed32", "sfixed64"}


def tokens(text):
    out, pos = [], 0
    while pos < len(text):
        mt = TOK.match(text, pos)
        if not mt:
            if text[pos:].strip() == "":
                break
            raise SyntaxError(text[pos:pos + 60])
        pos = mt.end()
        t = mt.group(1)
        if not t.startswith(("//", "/*")):
            out.append(t)
    return out


def parse(path):
    toks = tokens(open(path).read())
    pkg, msgs, i = "", {}, 0
    while i < len(toks):
        t = toks[i]
        if t in ("syntax", "import", "option"):
            i = toks.index(";", i) + 1
        elif t == "package":
            pkg = toks[i + 1]
            i += 3
        elif t == "message":
            name, i = toks[i + 1], i + 3
            fields = []
            while toks[i] != "}":
                label = "optional"
                if toks[i] in ("optional", "repeated", "required"):
                    label, i = toks[i], i + 1
                if toks[i] == "map":
                    k, v = toks[i + 2], toks[i + 4]
                    fname, num = toks[i + 6], int(toks[i + 8])
                    ftype, i = f"map<{k},{v}>", i + 9
                    label = "repeated"
                else:
                    ftype, fname, num = toks[i], toks[i + 1], int(toks[i + 3])
                    i += 4
                if toks[i] == "[":
                    depth = 0
                    while True:
                        depth += toks[i] == "["
                        depth -= toks[i] == "]"
                        i += 1
                        if depth == 0:
                            break
                assert toks[i] == ";", (path, name, toks[i:i + 4])
                i += 1
                fields.append([fname, num, label, ftype])
            msgs[name] = fields
            i += 1
        else:
            raise SyntaxError(f"{path}: unexpected {t!r}")
    return pkg, msgs


def qualify(pkg, msgs, all_names, t):
    def one(x):
        if x in SCALARS:
            return x
        if x in msgs:
            return f".{pkg}.{x}"
        if x in all_names:
            return "." + x
        raise KeyError(f"{pkg}: unresolved type {x}")
    if t.startswith("map<"):
        k, v = t[4:-1].split(",")
        return f"map<{one(k)},{one(v)}>"
    return one(t)


def _swagger_pkg(defn):
    p, m = defn.rsplit(".", 1)
    p = (p.replace("io.k8s.apiextensions-apiserver", "k8s.io.apiextensions_apiserver")
          .replace("io.k8s.kube-aggregator", "k8s.io.kube_aggregator").replace("io.k8s.", "k8s.io."))
    return p, m


def json_overrides(ref, packages):
    """Where the JSON shape differs from the proto one: an embedded Go struct whose fields the
    JSON inlines into its parent (Volume.volumeSource, Probe.handler, ...) and fields whose JSON
    name differs ({message: {"inline": [field], "rename": {proto: json}}})."""
    sw = json.load(open(os.path.join(ref, "api", "openapi-spec", "swagger.json")))["definitions"]
    fields_of = {f"{p}.{m}": {f[0]: f for f in fs} for p, ms in packages.items() for m, fs in ms.items()}
    out = {}

    def json_props(fq):
        return fields_of.get(fq, {})
    for d, v in sw.items():
        pkg, m = _swagger_pkg(d)
        fq = f"{pkg}.{m}"
        if fq not in fields_of:
            continue
        props = set((v.get("properties") or {}))
        ov = {"inline": [], "rename": {}}
        for name, f in fields_of[fq].items():
            if name in props:
                continue
            t = f[3]
            sub = json_props(t[1:]) if t.startswith(".") else {}
            lower = {x.lower(): x for x in props}
            if sub and set(sub) <= props | {"apiVersion", "kind"}:
                ov["inline"].append(name)
            elif name.lower() in lower:
                ov["rename"][name] = lower[name.lower()]
            elif "$" + name in props:
                ov["rename"][name] = "$" + name
        if ov["inline"] or ov["rename"]:
            out[fq] = {k: x for k, x in ov.items() if x}
    return out


def main(ref):
    base = os.path.join(ref, "staging", "src", "k8s.io")
    files = sorted(glob.glob(os.path.join(base, "api", "*", "*", "generated.proto")) +
                   [f for f in glob.glob(os.path.join(base, "apimachinery", "pkg", "**", "generated.proto"), recursive=True)
                    if "testapigroup" not in f] +
                   glob.glob(os.path.join(base, "apiextensions-apiserver", "pkg", "apis", "apiextensions", "v1beta1", "generated.proto")) +
                   glob.glob(os.path.join(base, "kube-aggregator", "pkg", "apis", "apiregistration", "v1beta1", "generated.proto")))
    parsed = {}
    for f in files:
        if "/testing/" in f or "/test/" in f or "/example" in f:
            continue
        pkg, msgs = parse(f)
        parsed.setdefault(pkg, {}).update(msgs)
    all_names = {f"{p}.{m}" for p, ms in parsed.items() for m in ms}
    out = {}
    for pkg, msgs in sorted(parsed.items()):
        out[pkg] = {m: [[n, num, lab, qualify(pkg, msgs, all_names, t)] for n, num, lab, t in fields]
                    for m, fields in sorted(msgs.items())}
    json_map = json_overrides(ref, out)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump({"source": "reference staging/src/k8s.io/**/generated.proto (field names, numbers, labels, types); "
                             "JSON shape of inlined Go structs and renamed fields from api/openapi-spec/swagger.json",
                   "packages": out, "json": json_map}, f, separators=(",", ":"), sort_keys=True)
    print(f"{len(out)} packages, {sum(len(v) for v in out.values())} messages -> {OUT} ({os.path.getsize(OUT)} B)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
