"""Runtime proto3 compiler: schema text → FileDescriptorProto → message classes + gRPC
service glue, with no protoc / grpc_tools in the loop (neither exists in this image).

The reference generates gogo-protobuf Go code from .proto files
(hack/update-generated-device-plugin.sh); amdkube instead keeps compact proto3 schema
text next to the Python that uses it and builds descriptors with `descriptor_pb2` at
import time. Supported grammar (what the Kubernetes node APIs and the etcd3 API need): package, message (no
nested messages), enum (top-level or nested in a message), `oneof`, scalar / message / enum
fields, `repeated`, `map<k,v>`, service with unary, server-, client- and bidi-streaming rpcs.
A dotted type reference (`mvccpb.KeyValue`) resolves by its last component inside the one
package. Wire compatibility is pinned by golden-bytes and reference-descriptor tests.
"""
from __future__ import annotations

import re

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
SCALARS = {
    "double": F.TYPE_DOUBLE, "float": F.TYPE_FLOAT, "int64": F.TYPE_INT64, "uint64": F.TYPE_UINT64,
    "int32": F.TYPE_INT32, "uint32": F.TYPE_UINT32, "bool": F.TYPE_BOOL, "string": F.TYPE_STRING,
    "bytes": F.TYPE_BYTES, "sint32": F.TYPE_SINT32, "sint64": F.TYPE_SINT64, "fixed64": F.TYPE_FIXED64,
    "fixed32": F.TYPE_FIXED32,
}

_TOK = re.compile(r"\s*(//[^\n]*|/\*.*?\*/|\"[^\"]*\"|[A-Za-z_][A-Za-z0-9_.]*|\d+|[{}()<>;=,\[\]])", re.S)


def _tokens(text: str):
    pos, out = 0, []
    text = text.strip()
    while pos < len(text):
        mt = _TOK.match(text, pos)
        if not mt:
            raise SyntaxError(f"proto parse error near {text[pos:pos + 40]!r}")
        t = mt.group(1)
        pos = mt.end()
        if not t.startswith("//") and not t.startswith("/*"):
            out.append(t)
    return out


def _camel(name: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


class Service:
    def __init__(self, full_name: str, methods: list[tuple]):
        self.full_name = full_name
        self.methods = methods  # (name, req_cls, resp_cls, server_streaming, client_streaming)

    def handler(self, impl) -> grpc.GenericRpcHandler:
        """Generic handler dispatching to `impl.<Method>` (sync or async callables)."""
        handlers = {}
        for name, req, resp, stream, cstream in self.methods:
            fn = getattr(impl, name, None)
            if fn is None:
                continue
            mk = {(False, False): grpc.unary_unary_rpc_method_handler, (True, False): grpc.unary_stream_rpc_method_handler,
                  (False, True): grpc.stream_unary_rpc_method_handler,
                  (True, True): grpc.stream_stream_rpc_method_handler}[(stream, cstream)]
            handlers[name] = mk(fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
        return grpc.method_handlers_generic_handler(self.full_name, handlers)

    def stub(self, channel):
        return _Stub(self, channel)


class _Stub:
    def __init__(self, svc: Service, channel):
        for name, req, resp, stream, cstream in svc.methods:
            mk = {(False, False): channel.unary_unary, (True, False): channel.unary_stream,
                  (False, True): channel.stream_unary, (True, True): channel.stream_stream}[(stream, cstream)]
            setattr(self, name, mk(f"/{svc.full_name}/{name}", request_serializer=req.SerializeToString,
                                   response_deserializer=resp.FromString))


class ProtoModule:
    """Namespace of message classes, enum values and services built from one schema."""

    def __init__(self, text: str, filename: str):
        self.pool = descriptor_pool.DescriptorPool()
        fdp = descriptor_pb2.FileDescriptorProto(name=filename, syntax="proto3")
        toks = _tokens(text)
        i = 0
        services = []
        # pre-scan enum names (simple name -> fully-qualified names) so field types resolve in one pass
        enums: dict[str, list[str]] = {}
        pkg = next((toks[j + 1] for j, t in enumerate(toks) if t == "package"), "")
        scope, depth = [], 0
        for j, t in enumerate(toks):
            if t in ("message", "enum") and j + 2 < len(toks) and toks[j + 2] == "{":
                if t == "enum":
                    enums.setdefault(toks[j + 1], []).append(".".join(["", pkg] + [n for n, _ in scope] + [toks[j + 1]]))
                scope.append((toks[j + 1], depth))
            elif t == "{":
                depth += 1
            elif t == "}":
                depth -= 1
                if scope and scope[-1][1] == depth:
                    scope.pop()
        while i < len(toks):
            t = toks[i]
            if t == "syntax":
                i = toks.index(";", i) + 1
            elif t == "package":
                fdp.package = toks[i + 1]
                i += 3
            elif t == "option" or t == "import":
                i = toks.index(";", i) + 1
            elif t == "message":
                i = self._message(fdp, toks, i, enums)
            elif t == "enum":
                i = self._enum(fdp.enum_type.add(), toks, i)
            elif t == "service":
                i = self._service(fdp, toks, i, services)
            else:
                raise SyntaxError(f"unexpected token {t!r}")
        self.package = fdp.package
        self.file = self.pool.Add(fdp)
        self.messages = {}
        for md in fdp.message_type:
            cls = message_factory.GetMessageClass(self.pool.FindMessageTypeByName(f"{fdp.package}.{md.name}"))
            self.messages[md.name] = cls
            setattr(self, md.name, cls)
        for ed in fdp.enum_type:
            for v in ed.value:
                setattr(self, v.name, v.number)
        self.services = {}
        for sname, methods in services:
            ms = [(n, self.messages[a.split(".")[-1]], self.messages[b.split(".")[-1]], st, cst) for n, a, b, st, cst in methods]
            svc = Service(f"{fdp.package}.{sname}", ms)
            self.services[sname] = svc
            setattr(self, sname, svc)
        self.descriptor_proto = fdp

    def _type(self, fdp, name, enums, field, msg: str = ""):
        name = name.split(".")[-1]
        if name in SCALARS:
            field.type = SCALARS[name]
        elif name in enums:
            field.type = F.TYPE_ENUM
            own = f".{fdp.package}.{msg}.{name}"
            field.type_name = own if own in enums[name] else enums[name][0]
        else:
            field.type = F.TYPE_MESSAGE
            field.type_name = f".{fdp.package}.{name}"

    def _message(self, fdp, toks, i, enums):
        md = fdp.message_type.add()
        md.name = toks[i + 1]
        assert toks[i + 2] == "{"
        i += 3
        while toks[i] != "}":
            if toks[i] == "enum":
                i = self._enum(md.enum_type.add(), toks, i)
                continue
            if toks[i] == "oneof":
                idx = len(md.oneof_decl)
                md.oneof_decl.add(name=toks[i + 1])
                i += 3
                while toks[i] != "}":
                    i = self._field(fdp, md, toks, i, enums, oneof=idx)
                i += 1
                continue
            i = self._field(fdp, md, toks, i, enums)
        return i + 1

    def _field(self, fdp, md, toks, i, enums, oneof: int | None = None):
        f = md.field.add()
        f.label = F.LABEL_OPTIONAL
        if oneof is not None:
            f.oneof_index = oneof
        if toks[i] == "repeated":
            f.label = F.LABEL_REPEATED
            i += 1
        if toks[i] == "map":
            kt, vt = toks[i + 2], toks[i + 4]
            assert toks[i + 1] == "<" and toks[i + 3] == "," and toks[i + 5] == ">"
            f.name, f.number = toks[i + 6], int(toks[i + 8])
            entry = md.nested_type.add()
            entry.name = _camel(f.name) + "Entry"
            entry.options.map_entry = True
            k = entry.field.add(name="key", number=1, label=F.LABEL_OPTIONAL)
            self._type(fdp, kt, enums, k, md.name)
            v = entry.field.add(name="value", number=2, label=F.LABEL_OPTIONAL)
            self._type(fdp, vt, enums, v, md.name)
            if v.type_name and v.type == F.TYPE_MESSAGE:
                pass
            f.label = F.LABEL_REPEATED
            f.type = F.TYPE_MESSAGE
            f.type_name = f".{fdp.package}.{md.name}.{entry.name}"
            i += 9
        else:
            self._type(fdp, toks[i], enums, f, md.name)
            f.name, f.number = toks[i + 1], int(toks[i + 3])
            assert toks[i + 2] == "="
            i += 4
        f.json_name = _json_name(f.name)
        if toks[i] == "[":  # field options (ignored)
            i = toks.index("]", i) + 1
        assert toks[i] == ";", toks[i:i + 3]
        return i + 1

    def _enum(self, ed, toks, i):
        ed.name = toks[i + 1]
        i += 3
        while toks[i] != "}":
            ed.value.add(name=toks[i], number=int(toks[i + 2]))
            i += 4
        return i + 1

    def _service(self, fdp, toks, i, services):
        sd = fdp.service.add()
        sd.name = toks[i + 1]
        i += 3
        methods = []
        while toks[i] != "}":
            assert toks[i] == "rpc", toks[i]
            name = toks[i + 1]
            cstream = toks[i + 3] == "stream"
            req = toks[i + 4] if cstream else toks[i + 3]
            j = i + (6 if cstream else 5)
            assert toks[j] == "returns"
            stream = toks[j + 2] == "stream"
            resp = toks[j + 3] if stream else toks[j + 2]
            j = j + (5 if stream else 4)
            if toks[j] == "{":
                j = toks.index("}", j) + 1
            elif toks[j] == ";":
                j += 1
            m = sd.method.add(name=name, input_type=f".{fdp.package}.{req}", output_type=f".{fdp.package}.{resp}")
            m.server_streaming = stream
            m.client_streaming = cstream
            methods.append((name, req, resp, stream, cstream))
            i = j
        services.append((sd.name, methods))
        return i + 1


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])
