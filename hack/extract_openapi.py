"""Derive the property table of the reference's published OpenAPI document
(api/openapi-spec/swagger.json) into tests/fixtures/reference_openapi_properties.json:
{definition: {"required": [...], "properties": {name: type signature}}}. Descriptions are
dropped; the signature is the JSON type/format, or the last component of a $ref, with
arrays as "[]T" and string maps as "{}T".

  python hack/extract_openapi.py /root/reference
"""
import json
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "reference_openapi_properties.json")


def sig(p: dict) -> str:
    if "$ref" in p:
        return p["$ref"].rsplit(".", 1)[-1]
    t = p.get("type", "")
    if t == "array":
        return "[]" + sig(p.get("items") or {})
    if t == "object" and "additionalProperties" in p:
        return "{}" + sig(p["additionalProperties"])
    return t + (":" + p["format"] if p.get("format") else "")


def main(ref):
    defs = json.load(open(os.path.join(ref, "api", "openapi-spec", "swagger.json")))["definitions"]
    out = {k: {"required": sorted(d.get("required") or []), "properties": {n: sig(p) for n, p in (d.get("properties") or {}).items()}}
           for k, d in sorted(defs.items())}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"{len(out)} definitions -> {OUT}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
