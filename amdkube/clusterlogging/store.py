"""amdkube log-store: the `elasticsearch-logging` service of the fluentd-elasticsearch addon.

cluster/addons/fluentd-elasticsearch runs Elasticsearch 5.6 (es-statefulset.yaml, service
elasticsearch-logging:9200) for fluentd to write to and Kibana to read. No Elasticsearch ships
with this image, so the log store serves the subset of its REST API that pipeline uses:
* `GET /` (cluster info), `GET /_cluster/health`;
* `POST /_bulk` — NDJSON `index` / `create` actions with their documents (per-item results and
  the top-level `errors` flag, as Elasticsearch answers);
* `GET|POST /<index>/_search` — `match_all`, `term`, `match` (every word of the text in the
  field), `range` on `@timestamp`, `bool` with must / filter / must_not / should, and `?q=`
  (`field:value` terms and free words, ANDed), with `size`, `from` and a `sort` on one field;
  the index may be a comma list or wildcard (`logstash-*`);
* `GET /_cat/indices`, `DELETE /<index>`, `GET /<index>/_count`.
Documents live per index in an append-only NDJSON file under --data-dir (read back on start);
--retention-days drops logstash-YYYY.MM.DD indices older than that, as the addon's curator did.
Search is a scan over the matching indices: the store is sized for a cluster's recent logs,
not for Elasticsearch's scale.
"""
from __future__ import annotations

import datetime
import fnmatch
import json
import logging
import os
import re
import threading
import time
import uuid

from aiohttp import web

log = logging.getLogger("amdkube.log-store")

VERSION = "5.6.4"
_INDEX_NAME = re.compile(r"^[a-z0-9][a-z0-9._+-]*$")


class LogStore:
    def __init__(self, data_dir: str, retention_days: int = 0):
        self.dir = data_dir
        self.retention_days = retention_days
        self.indices: dict[str, list[dict]] = {}
        self._lock = threading.Lock()
        os.makedirs(data_dir, exist_ok=True)
        for f in sorted(os.listdir(data_dir)):
            if f.endswith(".ndjson"):
                docs = []
                with open(os.path.join(data_dir, f)) as fh:
                    for line in fh:
                        try:
                            docs.append(json.loads(line))
                        except ValueError:
                            continue          # a torn last line after a crash
                self.indices[f[:-len(".ndjson")]] = docs

    # ------------------------------------------------------------------ writes
    def bulk(self, body: str) -> dict:
        t0 = time.monotonic()
        lines = [ln for ln in body.split("\n") if ln.strip()]
        items, errors, appended = [], False, {}
        i = 0
        while i < len(lines):
            try:
                action = json.loads(lines[i])
                (op, meta), = action.items()
            except (ValueError, AttributeError):
                return {"error": {"type": "illegal_argument_exception", "reason": f"Malformed action/metadata line [{i + 1}]"},
                        "status": 400}
            if op == "delete":
                i += 1
                items.append({op: {"_index": meta.get("_index"), "_id": meta.get("_id"), "status": 404, "result": "not_found"}})
                continue
            if op not in ("index", "create") or i + 1 >= len(lines):
                return {"error": {"type": "illegal_argument_exception", "reason": f"unsupported bulk action {op!r}"},
                        "status": 400}
            index, doc_id = meta.get("_index", ""), meta.get("_id") or uuid.uuid4().hex[:20]
            try:
                doc = json.loads(lines[i + 1])
            except ValueError:
                doc = None
            i += 2
            if not _INDEX_NAME.match(index or "") or not isinstance(doc, dict):
                errors = True
                items.append({op: {"_index": index, "_id": doc_id, "status": 400,
                                   "error": {"type": "mapper_parsing_exception" if doc is None or not isinstance(doc, dict)
                                             else "invalid_index_name_exception", "reason": "failed to parse"}}})
                continue
            rec = {"_id": doc_id, "_type": meta.get("_type", "fluentd"), "_source": doc}
            appended.setdefault(index, []).append(rec)
            items.append({op: {"_index": index, "_type": rec["_type"], "_id": doc_id, "_version": 1, "result": "created",
                               "status": 201}})
        with self._lock:
            for index, recs in appended.items():
                self.indices.setdefault(index, []).extend(recs)
                with open(os.path.join(self.dir, index + ".ndjson"), "a") as f:
                    f.write("".join(json.dumps(r, separators=(",", ":")) + "\n" for r in recs))
        return {"took": int((time.monotonic() - t0) * 1000), "errors": errors, "items": items}

    def delete_index(self, pattern: str) -> bool:
        with self._lock:
            names = self._resolve(pattern)
            for n in names:
                self.indices.pop(n, None)
                try:
                    os.unlink(os.path.join(self.dir, n + ".ndjson"))
                except OSError:
                    pass
        return bool(names)

    def enforce_retention(self, now: datetime.date | None = None) -> list[str]:
        if self.retention_days <= 0:
            return []
        today = now or datetime.datetime.now(datetime.timezone.utc).date()
        old = []
        for n in list(self.indices):
            m = re.fullmatch(r"logstash-(\d{4})\.(\d{2})\.(\d{2})", n)
            if m and (today - datetime.date(*map(int, m.groups()))).days > self.retention_days:
                old.append(n)
        for n in old:
            self.delete_index(n)
        return old

    # ------------------------------------------------------------------ reads
    def _resolve(self, pattern: str) -> list[str]:
        out = []
        for p in (pattern or "_all").split(","):
            if p in ("_all", "*"):
                out += list(self.indices)
            else:
                out += [n for n in self.indices if fnmatch.fnmatchcase(n, p)]
        return sorted(set(out))

    def search(self, pattern: str, query: dict | None = None, q: str = "", size: int = 10, from_: int = 0,
               sort: list | None = None) -> dict:
        t0 = time.monotonic()
        pred = _compile(query or {"match_all": {}})
        if q:
            qp = _query_string(q)
            pred = (lambda a, b: (lambda d: a(d) and b(d)))(pred, qp)
        with self._lock:
            hits = [(n, r) for n in self._resolve(pattern) for r in self.indices.get(n, ()) if pred(r["_source"])]
        if sort:
            spec = sort[0]
            field, order = (spec, "asc") if isinstance(spec, str) else next(iter(spec.items()))
            order = order.get("order", "asc") if isinstance(order, dict) else order
            hits.sort(key=lambda h: _sort_key(_get(h[1]["_source"], field)), reverse=(order == "desc"))
        page = hits[from_:from_ + size]
        return {"took": int((time.monotonic() - t0) * 1000), "timed_out": False,
                "_shards": {"total": 1, "successful": 1, "failed": 0},
                "hits": {"total": len(hits), "max_score": 1.0 if hits else None,
                         "hits": [{"_index": n, "_type": r["_type"], "_id": r["_id"], "_score": 1.0, "_source": r["_source"]}
                                  for n, r in page]}}

    def cat_indices(self) -> str:
        with self._lock:
            return "".join(f"green open {n} 1 0 {len(d)} 0 {sum(len(json.dumps(r)) for r in d)}b\n"
                           for n, d in sorted(self.indices.items()))


def _get(doc, field: str):
    for part in field.split("."):
        if not isinstance(doc, dict) or part not in doc:
            return None
        doc = doc[part]
    return doc


def _sort_key(v):
    return (v is None, str(v) if not isinstance(v, (int, float)) else "", v if isinstance(v, (int, float)) else 0)


def _words(v) -> list[str]:
    return re.findall(r"\w+", str(v).lower())


def _compile(query: dict):
    """A query DSL clause -> predicate over a document's source."""
    (kind, arg), = query.items()
    if kind == "match_all":
        return lambda d: True
    if kind == "term":
        (field, v), = arg.items()
        v = v.get("value") if isinstance(v, dict) else v
        return lambda d: _get(d, field) == v or (isinstance(_get(d, field), list) and v in _get(d, field))
    if kind == "match":
        (field, v), = arg.items()
        v = v.get("query") if isinstance(v, dict) else v
        want = _words(v)
        return lambda d: all(w in _words(_get(d, field) or "") for w in want)
    if kind == "range":
        (field, bounds), = arg.items()

        def in_range(d):
            x = _get(d, field)
            if x is None:
                return False
            for op, b in bounds.items():
                if op == "gte" and not x >= b or op == "gt" and not x > b or op == "lte" and not x <= b or \
                        op == "lt" and not x < b:
                    return False
            return True
        return in_range
    if kind == "query_string":
        return _query_string(arg.get("query", ""))
    if kind == "bool":
        def clauses(key):
            c = arg.get(key) or []
            return [_compile(x) for x in (c if isinstance(c, list) else [c])]
        must, filt, must_not, should = clauses("must"), clauses("filter"), clauses("must_not"), clauses("should")
        return lambda d: (all(p(d) for p in must + filt) and not any(p(d) for p in must_not)
                          and (not should or any(p(d) for p in should)))
    raise ValueError(f"unsupported query {kind!r}")


def _query_string(q: str):
    terms = []
    for tok in re.findall(r'(\w[\w.@-]*):"([^"]*)"|(\w[\w.@-]*):(\S+)|"([^"]*)"|(\S+)', q):
        f1, v1, f2, v2, phrase, word = tok
        if word.upper() == "AND":
            continue
        if f1 or f2:
            field, v = (f1, v1) if f1 else (f2, v2)
            terms.append(_compile({"match": {field: v}}))
        else:
            want = _words(phrase or word)
            terms.append(lambda d, want=want: all(w in _words(json.dumps(d)) for w in want))
    return lambda d: all(t(d) for t in terms)


def app(store: LogStore) -> web.Application:
    def err(status, etype, reason):
        return web.json_response({"error": {"type": etype, "reason": reason}, "status": status}, status=status)

    async def root(_r):
        return web.json_response({"name": "amdkube-log-store", "cluster_name": "kubernetes-logging",
                                  "version": {"number": VERSION}, "tagline": "You Know, for Search"})

    async def health(_r):
        return web.json_response({"cluster_name": "kubernetes-logging", "status": "green", "number_of_nodes": 1,
                                  "active_primary_shards": len(store.indices), "active_shards": len(store.indices)})

    async def bulk(r):
        out = store.bulk(await r.text())
        return web.json_response(out, status=out.get("status", 200))

    async def search(r, index=None):
        try:
            body = json.loads(await r.text() or "{}")
            size = int(r.query.get("size", body.get("size", 10)))
            from_ = int(r.query.get("from", body.get("from", 0)))
            sort = body.get("sort")
            if "sort" in r.query:
                f, _, o = r.query["sort"].partition(":")
                sort = [{f: o or "asc"}]
            out = store.search(index or r.match_info["index"], body.get("query"), r.query.get("q", ""), size, from_, sort)
        except ValueError as e:
            return err(400, "parsing_exception", str(e))
        return web.json_response(out)

    async def search_all(r):
        return await search(r, "_all")

    async def count(r):
        body = json.loads(await r.text() or "{}")
        out = store.search(r.match_info["index"], body.get("query"), r.query.get("q", ""), 0, 0)
        return web.json_response({"count": out["hits"]["total"]})

    async def cat(_r):
        return web.Response(text=store.cat_indices())

    async def delete(r):
        if not store.delete_index(r.match_info["index"]):
            return err(404, "index_not_found_exception", f"no such index [{r.match_info['index']}]")
        return web.json_response({"acknowledged": True})

    a = web.Application(client_max_size=64 << 20)
    a.router.add_get("/", root)
    a.router.add_get("/_cluster/health", health)
    a.router.add_post("/_bulk", bulk)
    a.router.add_get("/_cat/indices", cat)
    for method in ("GET", "POST"):
        a.router.add_route(method, "/{index}/_search", search)
        a.router.add_route(method, "/_search", search_all)
        a.router.add_route(method, "/{index}/_count", count)
    a.router.add_delete("/{index}", delete)
    return a

