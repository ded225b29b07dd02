"""Wire parity pinned to the reference's own descriptors (tests/fixtures/reference_descriptors,
extracted byte-for-byte from the generated api.pb.go files, see PROVENANCE.md there).

For every message, field, enum, map entry and RPC in the reference descriptor the runtime-built
amdkube descriptor must carry the same package, name, number, type, label and method path.
amdkube may add fields/messages (later CRI revisions it implements) only from the allow-list
below, and never on a number the reference uses. A deliberate field-number change in
amdkube/grpcdesc/deviceplugin.py turns this red (test_a_renumbered_field_is_detected)."""
import gzip
import os

import pytest
from google.protobuf import descriptor_pb2

from amdkube.grpcdesc import cri, deviceplugin as dp
from amdkube.grpcdesc.compiler import ProtoModule

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "reference_descriptors")

# amdkube-only additions (newer CRI revisions): name → why
ALLOWED_EXTRA_MESSAGES = {"ContainerEventResponse": "evented PLEG (CRI v1 GetContainerEvents)",
                          "GetEventsRequest": "evented PLEG request"}
ALLOWED_EXTRA_FIELDS = {("MemoryUsage", f) for f in ("available_bytes", "usage_bytes", "rss_bytes", "page_faults",
                                                     "major_page_faults")}
ALLOWED_EXTRA_METHODS = {("RuntimeService", "GetContainerEvents")}


def load(name):
    with open(os.path.join(FIX, name + ".pb.gz"), "rb") as f:
        return descriptor_pb2.FileDescriptorProto.FromString(gzip.decompress(f.read()))


def messages(fd):
    out = {}

    def walk(prefix, msgs):
        for m in msgs:
            out[prefix + m.name] = m
            walk(prefix + m.name + ".", m.nested_type)
    walk("", fd.message_type)
    return out


def field_sig(f):
    # type_name is compared by its last component (packages differ only by file layout)
    return f.number, f.type, f.label, f.type_name.rsplit(".", 1)[-1]


def compare(ref, ours):
    problems = []
    if ref.package != ours.package:
        problems.append(f"package {ref.package!r} != {ours.package!r}")
    rm, om = messages(ref), messages(ours)
    for name, m in rm.items():
        o = om.get(name)
        if o is None:
            problems.append(f"missing message {name}")
            continue
        if m.options.map_entry != o.options.map_entry:
            problems.append(f"{name}: map_entry differs")
        of = {f.name: f for f in o.field}
        for f in m.field:
            if f.name not in of:
                problems.append(f"{name}.{f.name}: missing field #{f.number}")
            elif field_sig(f) != field_sig(of[f.name]):
                problems.append(f"{name}.{f.name}: reference {field_sig(f)} amdkube {field_sig(of[f.name])}")
        used = {f.number for f in m.field}
        for f in o.field:
            if f.name not in {x.name for x in m.field}:
                if (name, f.name) not in ALLOWED_EXTRA_FIELDS:
                    problems.append(f"{name}.{f.name}: extra field not in the allow-list")
                elif f.number in used:
                    problems.append(f"{name}.{f.name}: extra field reuses reference number {f.number}")
    for name in set(om) - set(rm):
        base = name.split(".")[0]
        if base not in ALLOWED_EXTRA_MESSAGES:
            problems.append(f"extra message {name}")
    re_ = {e.name: {v.name: v.number for v in e.value} for e in ref.enum_type}
    oe = {e.name: {v.name: v.number for v in e.value} for e in ours.enum_type}
    for name, vals in re_.items():
        if oe.get(name) != vals:
            problems.append(f"enum {name}: reference {vals} amdkube {oe.get(name)}")
    rs = {(s.name, x.name): x for s in ref.service for x in s.method}
    os_ = {(s.name, x.name): x for s in ours.service for x in s.method}
    for k, x in rs.items():
        y = os_.get(k)
        if y is None:
            problems.append(f"missing rpc /{ref.package}.{k[0]}/{k[1]}")
            continue
        sig = lambda z: (z.input_type.rsplit(".", 1)[-1], z.output_type.rsplit(".", 1)[-1],  # noqa: E731
                         z.client_streaming, z.server_streaming)
        if sig(x) != sig(y):
            problems.append(f"rpc {k}: reference {sig(x)} amdkube {sig(y)}")
    for k in set(os_) - set(rs):
        if k not in ALLOWED_EXTRA_METHODS:
            problems.append(f"extra rpc {k}")
    return problems


@pytest.mark.parametrize("fixture,module", [("deviceplugin_v1alpha", dp.V1ALPHA2),
                                            ("pluginregistration_v1beta", dp.REGISTRATION),
                                            ("cri_v1alpha1_runtime", cri.CRI)])
def test_descriptor_matches_reference(fixture, module):
    ref = load(fixture)
    assert compare(ref, module.descriptor_proto) == []
    # every reference rpc is served under the same method path
    for s in ref.service:
        for x in s.method:
            assert f"/{ref.package}.{s.name}/{x.name}" in {f"/{module.package}.{sn}/{n}" for sn, svc in module.services.items()
                                                            for n, *_ in svc.methods}


def test_a_renumbered_field_is_detected():
    src = open(dp.__file__).read()
    start = src.index('V1ALPHA2 = ProtoModule("""') + len('V1ALPHA2 = ProtoModule("""')
    text = src[start:src.index('""",', start)]
    assert "string resource_name = 1;" in text or "ID = 1" in text or "= 1;" in text
    # renumber Device.health (reference #2) to #7
    mutated = text.replace("string health = 2;", "string health = 7;", 1)
    assert mutated != text, "fixture text changed: update the mutation"
    problems = compare(load("deviceplugin_v1alpha"), ProtoModule(mutated, "mut.proto").descriptor_proto)
    assert any("Device.health" in p for p in problems), problems


# ------------------------------------------------------------------ OpenAPI vs swagger.json
# amdkube serves these reference-absent fields (later Kubernetes features it implements);
# every other shared definition must equal the reference's property set, types and required.
OPENAPI_EXTENSIONS = {
    "io.k8s.apiextensions-apiserver.pkg.apis.apiextensions.v1beta1.CustomResourceDefinitionNames": {"categories"},
    "io.k8s.apiextensions-apiserver.pkg.apis.apiextensions.v1beta1.CustomResourceDefinitionSpec": {"subresources"},
}


def _sig(p: dict) -> str:      # same signature as hack/extract_openapi.py
    if "$ref" in p:
        return p["$ref"].rsplit(".", 1)[-1]
    t = p.get("type", "")
    if t == "array":
        return "[]" + _sig(p.get("items") or {})
    if t == "object" and "additionalProperties" in p:
        return "{}" + _sig(p["additionalProperties"])
    return t + (":" + p["format"] if p.get("format") else "")


def openapi_problems(ref: dict, ours: dict) -> list[str]:
    problems = []
    for name in sorted(set(ref) & set(ours)):
        rp = ref[name]["properties"]
        op = {n: _sig(p) for n, p in (ours[name].get("properties") or {}).items()}
        ext = OPENAPI_EXTENSIONS.get(name, set())
        for n in sorted(set(rp) - set(op)):
            problems.append(f"{name}: missing property {n}")
        for n in sorted(set(op) - set(rp) - ext):
            problems.append(f"{name}: extra property {n}")
        for n in sorted(set(rp) & set(op)):
            if rp[n] != op[n]:
                problems.append(f"{name}.{n}: reference {rp[n]} amdkube {op[n]}")
        if sorted(ours[name].get("required") or []) != ref[name]["required"]:
            problems.append(f"{name}: required reference {ref[name]['required']} amdkube {sorted(ours[name].get('required') or [])}")
    return problems


def test_openapi_matches_reference_swagger():
    import json
    from amdkube.api import openapi
    with open(os.path.join(os.path.dirname(__file__), "fixtures", "reference_openapi_properties.json")) as f:
        ref = json.load(f)
    ours = openapi.definitions()
    shared = set(ref) & set(ours)
    assert len(shared) >= 340, len(shared)
    assert openapi_problems(ref, ours) == []
    # the fork's device-granular surface is among the shared definitions
    for d in ("io.k8s.api.core.v1.PodExtendedResource", "io.k8s.api.core.v1.ExtendedResourceDomain",
              "io.k8s.api.core.v1.ExtendedResourceList", "io.k8s.api.core.v1.ExtendedResourceAffinity", "io.k8s.api.core.v1.Event"):
        assert d in shared, d


def test_openapi_parity_detects_a_dropped_field():
    import copy
    import json
    from amdkube.api import openapi
    with open(os.path.join(os.path.dirname(__file__), "fixtures", "reference_openapi_properties.json")) as f:
        ref = json.load(f)
    ours = copy.deepcopy(openapi.definitions())
    del ours["io.k8s.api.core.v1.Event"]["properties"]["reportingInstance"]
    assert openapi_problems(ref, ours) == ["io.k8s.api.core.v1.Event: missing property reportingInstance"]
