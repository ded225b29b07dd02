"""Kubernetes protobuf serialization of API objects (`application/vnd.kubernetes.protobuf`).

Reference: staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go —
an encoded object is the 4-byte magic `k8s\\x00` followed by a runtime.Unknown message
{typeMeta{apiVersion, kind} = 1, raw = 2, contentEncoding = 3, contentType = 4} whose `raw` is
the object's own message (protobuf.go:42, :88 Decode, :171 Encode). The messages are the
gogo-generated proto2 schemas of staging/src/k8s.io/api/**/generated.proto (core/v1 includes the
fork's fields: Container.extendedResourceRequests = 22, PodSpec.extendedResources = 27,
NodeStatus.extendedResources = 11, ObjectReference.extendedResourceBinding = 8).

amdkube keeps the wire table (name, number, label, type per field; amdkube/api/proto/
k8s_wire.json, derived by hack/gen_proto_tables.py) and builds descriptors from it with
descriptor_pb2 at first use, then converts between the API's JSON dicts and messages:

  * meta/v1 Time / MicroTime  ↔ RFC 3339 strings     (seconds + nanos)
  * meta/v1 Duration          ↔ Go duration strings  ("1h2m3s")
  * resource.Quantity         ↔ strings              (the canonical string is the wire form)
  * intstr.IntOrString        ↔ int or string        (type 0 int, 1 string)
  * runtime.RawExtension      ↔ embedded JSON object (raw bytes)
  * bytes fields              ↔ base64 strings
  * Go structs the JSON inlines (Volume.volumeSource, Probe.handler, ...) are flattened, and
    the few fields whose JSON name differs are renamed, as the table records;
  * apiextensions JSONSchemaProps and friends carry free-form JSON Schema.

Fields the schema does not know are dropped by an encode, as the reference's typed decode
would; `lossless()` tells a caller (storage) whether an object survives the round trip.

The hot path is native: amdkube/_native/_kproto (native/kproto.cpp) walks the dicts and writes
/reads wire bytes directly from a flat table built here from the same descriptors, and reports
losslessness during the encode (`encode_checked`), so storage no longer decodes every write to
find out. The message-object path below stays for the rare types _kproto hands back by
callback (Duration, RawExtension, JSON Schema props) and as the fallback when the extension is
not built (AMDKUBE_REQUIRE_NATIVE=1 makes that an error).
Watch streams frame each WatchEvent with a 4-byte big-endian length
(apimachinery/pkg/util/framer LengthDelimitedFramer); the event's object is itself enveloped.
"""
from __future__ import annotations

import base64
import functools
import json
import os
import re
import struct
from datetime import datetime, timezone

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf.message import DecodeError

MAGIC = b"k8s\x00"
MEDIA_TYPE = "application/vnd.kubernetes.protobuf"
STREAM_MEDIA_TYPE = "application/vnd.kubernetes.protobuf;stream=watch"
WIRE = os.path.join(os.path.dirname(__file__), "proto", "k8s_wire.json")

META = "k8s.io.apimachinery.pkg.apis.meta.v1"
RUNTIME = "k8s.io.apimachinery.pkg.runtime"
TIME, MICROTIME, DURATION = f"{META}.Time", f"{META}.MicroTime", f"{META}.Duration"
QUANTITY = "k8s.io.apimachinery.pkg.api.resource.Quantity"
INTORSTR = "k8s.io.apimachinery.pkg.util.intstr.IntOrString"
RAWEXT = f"{RUNTIME}.RawExtension"
APIEXT = "k8s.io.apiextensions_apiserver.pkg.apis.apiextensions.v1beta1"
F = descriptor_pb2.FieldDescriptorProto
_SCALAR = {"double": F.TYPE_DOUBLE, "float": F.TYPE_FLOAT, "int64": F.TYPE_INT64, "uint64": F.TYPE_UINT64,
           "int32": F.TYPE_INT32, "uint32": F.TYPE_UINT32, "bool": F.TYPE_BOOL, "string": F.TYPE_STRING,
           "bytes": F.TYPE_BYTES, "sint32": F.TYPE_SINT32, "sint64": F.TYPE_SINT64, "fixed64": F.TYPE_FIXED64,
           "fixed32": F.TYPE_FIXED32, "sfixed32": F.TYPE_SFIXED32, "sfixed64": F.TYPE_SFIXED64}
_LABEL = {"optional": F.LABEL_OPTIONAL, "repeated": F.LABEL_REPEATED, "required": F.LABEL_OPTIONAL}


class ProtoError(ValueError):
    pass


def _camel(name: str) -> str:
    return name[:1].upper() + name[1:]


class Schema:
    """Descriptor pool + message classes for every package of the wire table."""

    def __init__(self, path: str = WIRE):
        with open(path) as f:
            table = json.load(f)
        self.packages = table["packages"]
        self.json = table.get("json", {})
        self.pool = descriptor_pool.DescriptorPool()
        files, deps = {}, {}
        for pkg, msgs in self.packages.items():
            fdp = descriptor_pb2.FileDescriptorProto(name=pkg.replace(".", "/") + "/generated.proto", package=pkg,
                                                     syntax="proto2")
            need = set()
            for mname, fields in msgs.items():
                md = fdp.message_type.add(name=mname)
                for fname, num, label, ftype in fields:
                    fd = md.field.add(name=fname, number=num, label=_LABEL[label], json_name=fname)
                    if ftype.startswith("map<"):
                        kt, vt = ftype[4:-1].split(",", 1)
                        entry = md.nested_type.add(name=_camel(fname) + "Entry")
                        entry.options.map_entry = True
                        for en, et, n in (("key", kt, 1), ("value", vt, 2)):
                            ef = entry.field.add(name=en, number=n, label=F.LABEL_OPTIONAL)
                            self._type(ef, et, need)
                        fd.type, fd.type_name = F.TYPE_MESSAGE, f".{pkg}.{mname}.{entry.name}"
                        fd.label = F.LABEL_REPEATED
                    else:
                        self._type(fd, ftype, need)
            need.discard(pkg)
            files[pkg], deps[pkg] = fdp, need
        done: set[str] = set()

        def add(pkg):
            if pkg in done:
                return
            done.add(pkg)
            for d in sorted(deps[pkg]):
                add(d)
                files[pkg].dependency.append(files[d].name)
            self.pool.Add(files[pkg])
        for pkg in sorted(files):
            add(pkg)
        self._classes: dict[str, type] = {}

    @staticmethod
    def _type(fd, ftype: str, need: set):
        if ftype in _SCALAR:
            fd.type = _SCALAR[ftype]
        else:
            fd.type, fd.type_name = F.TYPE_MESSAGE, ftype
            need.add(ftype[1:].rsplit(".", 1)[0])

    def cls(self, fq: str):
        c = self._classes.get(fq)
        if c is None:
            c = self._classes[fq] = message_factory.GetMessageClass(self.pool.FindMessageTypeByName(fq))
        return c

    def has(self, fq: str) -> bool:
        pkg, _, m = fq.rpartition(".")
        return m in self.packages.get(pkg, {})


@functools.lru_cache(maxsize=1)
def schema() -> Schema:
    return Schema()


# ------------------------------------------------------------------ kinds → messages
_GROUP_PKG = {"": "k8s.io.api.core", "apiextensions.k8s.io": "k8s.io.apiextensions_apiserver.pkg.apis.apiextensions",
              "apiregistration.k8s.io": "k8s.io.kube_aggregator.pkg.apis.apiregistration"}
_META_KINDS = {"Status", "WatchEvent", "APIGroup", "APIGroupList", "APIResourceList", "APIVersions", "DeleteOptions",
               "ListOptions", "GetOptions", "ExportOptions"}


def message_for(api_version: str, kind: str) -> str | None:
    """Fully-qualified message of a kind (None when the reference defines no protobuf for it:
    custom resources and amdkube-only kinds stay JSON, as CRDs do upstream)."""
    group, _, version = api_version.rpartition("/")
    if kind in _META_KINDS:
        fq = f"{META}.{kind}"
    else:
        base = _GROUP_PKG.get(group) or f"k8s.io.api.{group.split('.')[0]}"
        fq = f"{base}.{version}.{kind}"
    return fq if schema().has(fq) else None


# --------------------------------------------------------------------- special types
_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)")
_DUR_NS = {"ns": 1, "us": 1_000, "µs": 1_000, "ms": 1_000_000, "s": 1_000_000_000, "m": 60_000_000_000,
           "h": 3_600_000_000_000}


def parse_duration(s: str) -> int:
    s = s.strip()
    neg = s.startswith("-")
    s = s.lstrip("+-")
    if s in ("0", ""):
        return 0
    pos, total = 0, 0
    for mt in _DUR.finditer(s):
        if mt.start() != pos:
            raise ProtoError(f"invalid duration {s!r}")
        total += int(round(float(mt.group(1)) * _DUR_NS[mt.group(2)]))
        pos = mt.end()
    if pos != len(s):
        raise ProtoError(f"invalid duration {s!r}")
    return -total if neg else total


def format_duration(ns: int) -> str:
    """Go time.Duration.String()."""
    if ns == 0:
        return "0s"
    sign = "-" if ns < 0 else ""
    ns = abs(ns)
    if ns < 1_000_000_000:
        for unit, div in (("ms", 1_000_000), ("µs", 1_000), ("ns", 1)):
            if ns >= div:
                v = ns / div
                return sign + (f"{v:.9f}".rstrip("0").rstrip(".")) + unit
    h, rem = divmod(ns, 3_600_000_000_000)
    mnt, rem = divmod(rem, 60_000_000_000)
    sec = rem / 1e9
    s = f"{sec:.9f}".rstrip("0").rstrip(".") + "s"
    if h:
        return f"{sign}{h}h{mnt}m{s}"
    if mnt:
        return f"{sign}{mnt}m{s}"
    return sign + s


def _parse_time(s: str) -> tuple[int, int]:
    s = s.strip()
    frac = 0
    m = re.match(r"^(\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d)(\.\d+)?(Z|[+-]\d\d:\d\d)$", s)
    if not m:
        raise ProtoError(f"invalid RFC 3339 time {s!r}")
    dt = datetime.strptime(m.group(1), "%Y-%m-%dT%H:%M:%S")
    if m.group(2):
        frac = int((m.group(2)[1:] + "000000000")[:9])
    tz = m.group(3)
    off = 0 if tz == "Z" else (1 if tz[0] == "+" else -1) * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    secs = int(dt.replace(tzinfo=timezone.utc).timestamp()) - off
    return secs, frac


def _format_time(secs: int, nanos: int, micro: bool) -> str:
    dt = datetime.fromtimestamp(secs, tz=timezone.utc)
    base = dt.strftime("%Y-%m-%dT%H:%M:%S")
    return base + (f".{nanos // 1000:06d}" if micro else "") + "Z"


# -------------------------------------------------------------- conversion plans
# kinds of field in a plan entry
SCALAR, MSG, REP_SCALAR, REP_MSG, MAP_SCALAR, MAP_MSG = range(6)


def _conv(t):
    """JSON → wire value for a scalar field type."""
    if t == F.TYPE_BYTES:
        return lambda v: base64.b64decode(v) if isinstance(v, str) else bytes(v)
    if t == F.TYPE_STRING:
        return lambda v: v if isinstance(v, str) else str(v)
    if t == F.TYPE_BOOL:
        return bool
    if t in (F.TYPE_DOUBLE, F.TYPE_FLOAT):
        return float
    return int


def _unconv(t):
    if t == F.TYPE_BYTES:
        return lambda v: base64.b64encode(v).decode()
    return None


class _Plan:
    """Per-message conversion plan, built once: json key → (proto name, kind, sub message, conv),
    field number → (json key, kind, sub message, unconv), and the inlined sub-structs."""
    __slots__ = ("by_key", "by_num", "inline")

    def __init__(self, desc):
        ov = schema().json.get(desc.full_name) or {}
        rename = ov.get("rename") or {}
        inline = set(ov.get("inline") or ())
        self.by_key, self.by_num, self.inline = {}, {}, []
        for fd in desc.fields:
            mt = fd.message_type
            if fd.name in inline:
                self.inline.append((fd.name, mt.full_name, {f.name for f in mt.fields}))
                self.by_num[fd.number] = (None, "inline", mt.full_name, None)
                continue
            key = rename.get(fd.name, fd.name)
            if mt is not None and mt.GetOptions().map_entry:
                vfd = mt.fields_by_name["value"]
                if vfd.message_type is not None:
                    kind, sub, cv, ucv = MAP_MSG, vfd.message_type.full_name, None, None
                else:
                    kind, sub, cv, ucv = MAP_SCALAR, None, _conv(vfd.type), _unconv(vfd.type)
            elif fd.is_repeated:
                if mt is not None:
                    kind, sub, cv, ucv = REP_MSG, mt.full_name, None, None
                else:
                    kind, sub, cv, ucv = REP_SCALAR, None, _conv(fd.type), _unconv(fd.type)
            elif mt is not None:
                kind, sub, cv, ucv = MSG, mt.full_name, None, None
            else:
                kind, sub, cv, ucv = SCALAR, None, _conv(fd.type), _unconv(fd.type)
            self.by_key[key] = (fd.name, kind, sub, cv)
            self.by_num[fd.number] = (key, kind, sub, ucv)


_PLANS: dict[str, _Plan] = {}


def _plan(desc) -> _Plan:
    p = _PLANS.get(desc.full_name)
    if p is None:
        p = _PLANS[desc.full_name] = _Plan(desc)
    return p


# --------------------------------------------------------------------- JSON → message
def _fill_special(msg, d, fq) -> bool:
    if fq in (TIME, MICROTIME):
        msg.seconds, msg.nanos = _parse_time(d)
    elif fq == DURATION:
        msg.duration = parse_duration(d) if isinstance(d, str) else int(d)
    elif fq == QUANTITY:
        msg.string = str(d)
    elif fq == INTORSTR:
        if isinstance(d, bool) or not isinstance(d, (int, str)):
            raise ProtoError(f"int-or-string wants an int or a string, got {d!r}")
        if isinstance(d, int):
            msg.type, msg.intVal = 0, d
        else:
            msg.type, msg.strVal = 1, d
    elif fq == RAWEXT or fq == f"{APIEXT}.JSON":
        msg.raw = json.dumps(d, separators=(",", ":")).encode()
    elif fq == f"{APIEXT}.JSONSchemaPropsOrArray":
        if isinstance(d, list):
            for x in d:
                _fill(msg.jSONSchemas.add(), x, f"{APIEXT}.JSONSchemaProps")
        else:
            _fill(msg.schema, d, f"{APIEXT}.JSONSchemaProps")
    elif fq == f"{APIEXT}.JSONSchemaPropsOrBool":
        if isinstance(d, bool):
            msg.allows = d
        else:
            msg.allows = True
            _fill(msg.schema, d, f"{APIEXT}.JSONSchemaProps")
    elif fq == f"{APIEXT}.JSONSchemaPropsOrStringArray":
        if isinstance(d, list):
            msg.property.extend(d)
        else:
            _fill(msg.schema, d, f"{APIEXT}.JSONSchemaProps")
    elif fq.endswith(".ExtraValue"):          # a JSON list of strings (authentication ExtraValue)
        msg.items.extend(str(x) for x in d)
    else:
        return False
    return True


_SPECIAL = {TIME, MICROTIME, DURATION, QUANTITY, INTORSTR, RAWEXT, f"{APIEXT}.JSON", f"{APIEXT}.JSONSchemaPropsOrArray",
            f"{APIEXT}.JSONSchemaPropsOrBool", f"{APIEXT}.JSONSchemaPropsOrStringArray"}


def _is_special(fq: str) -> bool:
    return fq in _SPECIAL or fq.endswith(".ExtraValue")


def _fill(msg, d, fq: str):
    if _is_special(fq):
        _fill_special(msg, d, fq)
        return
    if not isinstance(d, dict):
        raise ProtoError(f"{fq}: expected an object, got {type(d).__name__}")
    plan = _plan(msg.DESCRIPTOR)
    by_key = plan.by_key
    for key, v in d.items():
        if v is None:
            continue
        ent = by_key.get(key)
        if ent is None:
            continue                     # a field the schema does not have (or an inlined one)
        name, kind, sub, cv = ent
        if kind == SCALAR:
            setattr(msg, name, cv(v))
        elif kind == MSG:
            m = getattr(msg, name)
            m.SetInParent()
            _fill(m, v, sub)
        elif kind == REP_MSG:
            target = getattr(msg, name)
            for x in v:
                _fill(target.add(), x, sub)
        elif kind == REP_SCALAR:
            getattr(msg, name).extend([cv(x) for x in v])
        elif kind == MAP_SCALAR:
            target = getattr(msg, name)
            for k, x in v.items():
                if x is not None:
                    target[k] = cv(x)
        else:   # MAP_MSG
            target = getattr(msg, name)
            for k, x in v.items():
                if x is not None:
                    _fill(target[k], x, sub)
    for name, sub, keys in plan.inline:      # embedded structs the JSON flattens
        part = {k: d[k] for k in keys if k in d}
        if part:
            _fill(getattr(msg, name), part, sub)


# --------------------------------------------------------------------- message → JSON
def _dump_special(msg, fq):
    if fq in (TIME, MICROTIME):
        return _format_time(msg.seconds, msg.nanos, fq == MICROTIME)
    if fq == DURATION:
        return format_duration(msg.duration)
    if fq == QUANTITY:
        return msg.string
    if fq == INTORSTR:
        return msg.strVal if msg.type == 1 else msg.intVal
    if fq == RAWEXT or fq == f"{APIEXT}.JSON":
        return json.loads(msg.raw) if msg.raw else None
    if fq == f"{APIEXT}.JSONSchemaPropsOrArray":
        return [_dump(x, f"{APIEXT}.JSONSchemaProps") for x in msg.jSONSchemas] if len(msg.jSONSchemas) else \
            _dump(msg.schema, f"{APIEXT}.JSONSchemaProps")
    if fq == f"{APIEXT}.JSONSchemaPropsOrBool":
        return _dump(msg.schema, f"{APIEXT}.JSONSchemaProps") if msg.HasField("schema") else msg.allows
    if fq == f"{APIEXT}.JSONSchemaPropsOrStringArray":
        return list(msg.property) if len(msg.property) else _dump(msg.schema, f"{APIEXT}.JSONSchemaProps")
    if fq.endswith(".ExtraValue"):
        return list(msg.items)
    raise KeyError(fq)


def _dump(msg, fq: str):
    if _is_special(fq):
        return _dump_special(msg, fq)
    by_num = _plan(msg.DESCRIPTOR).by_num
    out = {}
    for fd, v in msg.ListFields():
        key, kind, sub, ucv = by_num[fd.number]
        if kind == SCALAR:
            out[key] = ucv(v) if ucv else v
        elif kind == MSG:
            out[key] = _dump(v, sub)
        elif kind == REP_MSG:
            out[key] = [_dump(x, sub) for x in v]
        elif kind == REP_SCALAR:
            out[key] = [ucv(x) for x in v] if ucv else list(v)
        elif kind == MAP_SCALAR:
            out[key] = {k: ucv(x) for k, x in v.items()} if ucv else dict(v)
        elif kind == MAP_MSG:
            out[key] = {k: _dump(x, sub) for k, x in v.items()}
        else:   # inline
            out.update(_dump(v, sub))
    return out


# ------------------------------------------------------------------------- native layer
_SP_CODES = {TIME: 1, MICROTIME: 2, QUANTITY: 3, INTORSTR: 4}
_KINDS = {SCALAR: 0, MSG: 1, REP_SCALAR: 2, REP_MSG: 3, MAP_SCALAR: 4, MAP_MSG: 5}


class _Native:
    """The _kproto table: one entry per message of the wire table, in a fixed order."""

    def __init__(self, mod):
        self.mod = mod
        sc = schema()
        self.names = [f"{pkg}.{mn}" for pkg in sorted(sc.packages) for mn in sorted(sc.packages[pkg])]
        self.index = {n: i for i, n in enumerate(self.names)}
        descs = [sc.pool.FindMessageTypeByName(n) for n in self.names]
        entries = []
        for fq, desc in zip(self.names, descs):
            if fq in _SP_CODES:
                special = _SP_CODES[fq]
            elif fq.endswith(".ExtraValue"):
                special = 5
            elif fq in _SPECIAL:
                special = 9
            else:
                special = 0
            ov = sc.json.get(fq) or {}
            rename, inline = ov.get("rename") or {}, set(ov.get("inline") or ())
            fields = []
            for fd in sorted(desc.fields, key=lambda f: f.number):
                mt = fd.message_type
                if fd.name in inline:
                    fields.append((fd.number, None, 6, 0, 0, self.index[mt.full_name]))
                    continue
                key = rename.get(fd.name, fd.name)
                if mt is not None and mt.GetOptions().map_entry:
                    kfd, vfd = mt.fields_by_name["key"], mt.fields_by_name["value"]
                    if vfd.message_type is not None:
                        fields.append((fd.number, key, 5, 11, kfd.type, self.index[vfd.message_type.full_name]))
                    else:
                        fields.append((fd.number, key, 4, vfd.type, kfd.type, -1))
                elif mt is not None:
                    fields.append((fd.number, key, 3 if fd.is_repeated else 1, 11, 0, self.index[mt.full_name]))
                else:
                    fields.append((fd.number, key, 2 if fd.is_repeated else 0, fd.type, 0, -1))
            entries.append([special, fields, None])

        def keys(i, seen=()):
            out = set()
            for num, key, kind, _st, _kt, sub in entries[i][1]:
                if kind == 6:
                    if sub not in seen:
                        out |= keys(sub, seen + (i,))
                else:
                    out.add(key)
            return out
        for i, e in enumerate(entries):
            e[2] = frozenset(keys(i))
        mod.init([tuple(e) for e in entries], ProtoError, self._enc_cb, self._dec_cb)

    def _enc_cb(self, mi: int, value):
        fq = self.names[mi]
        msg = schema().cls(fq)()
        try:
            _fill(msg, value, fq)
        except (TypeError, AttributeError) as e:
            raise ProtoError(f"{fq}: {e}") from None
        if fq == DURATION:
            ok = isinstance(value, str) and format_duration(msg.duration) == value
        elif fq in (RAWEXT, f"{APIEXT}.JSON"):
            ok = True
        else:
            ok = _norm(_dump(msg, fq)) == _norm(value)
        return msg.SerializeToString(), ok

    def _dec_cb(self, mi: int, data: bytes):
        fq = self.names[mi]
        try:
            return _dump(schema().cls(fq).FromString(data), fq)
        except DecodeError as e:
            raise ProtoError(f"{fq}: {e}") from None


@functools.lru_cache(maxsize=1)
def native() -> _Native | None:
    try:
        from .._native import _kproto
    except ImportError as e:
        if os.environ.get("AMDKUBE_REQUIRE_NATIVE") == "1":
            raise ImportError(f"amdkube._native._kproto is not built ({e}); run native/build.py") from e
        return None
    return _Native(_kproto)


# ------------------------------------------------------------------------- public API
def to_message(obj: dict, fq: str):
    msg = schema().cls(fq)()
    _fill(msg, obj, fq)
    return msg


def from_message(msg) -> dict:
    return _dump(msg, msg.DESCRIPTOR.full_name)


def encode_raw(obj: dict, fq: str, strict: bool = False) -> tuple[bytes, bool | None]:
    """The object's own message bytes; with `strict` also whether a decode gives it back."""
    nat = native()
    if nat is not None:
        return nat.mod.encode(obj, nat.index[fq], strict)
    return to_message(obj, fq).SerializeToString(), None


def decode_raw(raw: bytes, fq: str) -> dict:
    nat = native()
    if nat is not None:
        return nat.mod.decode(raw, nat.index[fq])
    try:
        return from_message(schema().cls(fq).FromString(raw))
    except DecodeError as e:
        raise ProtoError(f"{fq}: {e}") from None


def _encode(obj: dict, strict: bool) -> tuple[bytes, bool | None]:
    av, kind = obj.get("apiVersion", ""), obj.get("kind", "")
    if not isinstance(av, str) or not isinstance(kind, str):
        raise ProtoError("apiVersion and kind must be strings")
    fq = message_for(av, kind)
    if fq is None:
        raise ProtoError(f"no protobuf schema for {av} {kind}")
    raw, ok = encode_raw(obj, fq, strict)
    return envelope(av, kind, raw), ok


def encode(obj: dict) -> bytes:
    """`k8s\\x00` + runtime.Unknown for an object of a kind with a protobuf schema."""
    return _encode(obj, False)[0]


def encode_checked(obj: dict) -> tuple[bytes, bool]:
    """(encode(obj), lossless(obj, that)) — natively in one pass."""
    data, ok = _encode(obj, True)
    return data, (lossless(obj, data) if ok is None else ok)


def envelope_parts(data: bytes) -> tuple[str, str, bytes, str]:
    """(apiVersion, kind, raw, contentType) of a `k8s\\x00` runtime.Unknown."""
    if not data.startswith(MAGIC):
        raise ProtoError("missing the k8s protobuf magic")
    nat = native()
    if nat is not None:
        parts = nat.mod.envelope_parts(data)
        if parts is None:
            raise ProtoError("malformed runtime.Unknown envelope")
        return parts
    try:
        unk = schema().cls(f"{RUNTIME}.Unknown").FromString(data[4:])
    except DecodeError as e:
        raise ProtoError(f"malformed runtime.Unknown envelope: {e}") from None
    return unk.typeMeta.apiVersion, unk.typeMeta.kind, unk.raw, unk.contentType


def decode(data: bytes) -> dict:
    av, kind, raw, ctype = envelope_parts(data)
    if ctype and "json" in ctype:      # a JSON payload in the envelope
        obj = json.loads(raw)
    else:
        fq = message_for(av, kind)
        if fq is None:
            raise ProtoError(f"no protobuf schema for {av} {kind}")
        obj = decode_raw(raw, fq)
    out = {"apiVersion": av, "kind": kind} if av or kind else {}
    out.update(obj)
    if kind.endswith("List") and isinstance(out.get("items"), list):
        # typed list items carry no TypeMeta on the wire; the JSON API shows it on each item
        ik = kind[:-4]
        out["items"] = [{"apiVersion": av, "kind": ik, **it} if isinstance(it, dict) else it for it in out["items"]]
    return out


def supports(obj: dict) -> bool:
    av, kind = obj.get("apiVersion", ""), obj.get("kind", "")
    return isinstance(av, str) and isinstance(kind, str) and message_for(av, kind) is not None


def _norm(v):
    """Drop what a typed round trip cannot keep apart from absence: None, [], {}."""
    if isinstance(v, dict):
        out = {k: _norm(x) for k, x in v.items()}
        return {k: x for k, x in out.items() if x not in (None, [], {})}
    if isinstance(v, list):
        return [_norm(x) for x in v]
    return v


def lossless(obj: dict, data: bytes | None = None) -> bool:
    """True when `obj` decodes back from its protobuf form unchanged (up to empty values)."""
    try:
        back = decode(data if data is not None else encode(obj))
    except (ProtoError, ValueError):
        return False
    return _norm(back) == _norm(obj)


def encode_watch_event(etype: str, obj: dict) -> bytes:
    """One frame of a protobuf watch: 4-byte big-endian length + meta/v1 WatchEvent{type = 1,
    object = 2 (RawExtension{raw = 1})} whose object is the enveloped object
    (staging/.../endpoints/handlers/watch.go, framer)."""
    return watch_frame(etype, encode(obj) if supports(obj) else MAGIC + _json_unknown(obj))


def watch_frame(etype: str, enveloped: bytes) -> bytes:
    b = _ld(1, etype.encode()) + _ld(2, _ld(1, enveloped))
    return struct.pack(">I", len(b)) + b


def _json_unknown(obj: dict) -> bytes:
    unk = schema().cls(f"{RUNTIME}.Unknown")(raw=json.dumps(obj, separators=(",", ":")).encode(),
                                              contentType="application/json")
    unk.typeMeta.apiVersion, unk.typeMeta.kind = obj.get("apiVersion", ""), obj.get("kind", "")
    return unk.SerializeToString()


def encode_any(obj: dict) -> bytes:
    """Protobuf when the kind has a schema, else the envelope around JSON (contentType set), as the
    reference's server does for types without protobuf support."""
    return encode(obj) if supports(obj) else MAGIC + _json_unknown(obj)


# ------------------------------------------------------------ byte-level fast paths
def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ld(num: int, payload: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(payload)) + payload


def unwrap_raw(data: bytes) -> bytes | None:
    """The object message inside a stored `k8s\x00` envelope (Unknown.raw), found by scanning the
    envelope's top-level fields — no decode; None if the payload is not a protobuf object."""
    if data[:4] != MAGIC:
        return None
    nat = native()
    if nat is not None:
        parts = nat.mod.envelope_parts(data)
        return None if parts is None or "json" in parts[3] else parts[2]
    i, n, raw, json_payload = 4, len(data), None, False
    while i < n:
        key, shift = 0, 0
        while True:
            b = data[i]
            i += 1
            key |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        if key & 7 != 2:
            return None
        ln, shift = 0, 0
        while True:
            b = data[i]
            i += 1
            ln |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        if key >> 3 == 2:
            raw = data[i:i + ln]
        elif key >> 3 == 4 and b"json" in data[i:i + ln]:
            json_payload = True
        i += ln
    return None if json_payload else raw


def envelope(api_version: str, kind: str, raw: bytes) -> bytes:
    tm = _ld(1, api_version.encode()) + _ld(2, kind.encode())
    return MAGIC + _ld(1, tm) + _ld(2, raw)


def list_from_stored(api_version: str, list_kind: str, resource_version: str, stored: list[bytes]) -> bytes | None:
    """A <Kind>List envelope spliced from stored protobuf objects (ListMeta = 1, items = 2) without
    decoding any item; None when an item is stored as JSON."""
    nat = native()
    if nat is not None:
        return nat.mod.splice_list(api_version, list_kind, resource_version, stored)
    parts = [_ld(1, _ld(2, resource_version.encode()))]       # ListMeta.resourceVersion = 2
    for v in stored:
        raw = unwrap_raw(v)
        if raw is None:
            return None
        parts.append(_ld(2, raw))
    return envelope(api_version, list_kind, b"".join(parts))


def decode_watch_frames(buf: bytes) -> tuple[list[tuple[str, dict]], bytes]:
    """Split complete frames off `buf`: ([(type, object)], rest)."""
    out = []
    while len(buf) >= 4:
        n = struct.unpack(">I", buf[:4])[0]
        if len(buf) < 4 + n:
            break
        try:
            ev = schema().cls(f"{META}.WatchEvent").FromString(buf[4:4 + n])
        except DecodeError as e:
            raise ProtoError(f"malformed watch frame: {e}") from None
        out.append((ev.type, decode(ev.object.raw)))
        buf = buf[4 + n:]
    return out, buf
