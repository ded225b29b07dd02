"""amdkube log-shipper: the fluentd DaemonSet of the fluentd-elasticsearch addon.

cluster/addons/fluentd-elasticsearch/fluentd-es-configmap.yaml configures fluentd per node; the
shipper does the same work:
* containers.input.conf — tail /var/log/containers/*.log (the kubelet's legacy symlinks,
  `<pod>_<namespace>_<container>-<id>.log`), each line Docker JSON (`log`/`stream`/`time`),
  CRI (`<time> <stream> <P|F> <log>`, partial lines joined) or plain text (rocshim writes the
  process's output as is; the time is when it was read); tag `kubernetes.<path with dots>`;
* system.input.conf — glog-format component logs (kubelet, kube-proxy, apiserver, ...),
  `format_firstline /^\\w\\d{4}/` multi-line records with severity/time/pid/source/message;
* the kubernetes_metadata filter — `kubernetes: {pod_name, namespace_name, container_name,
  pod_id, labels, host}` and `docker: {container_id}` from the file name and the pod object
  (cached per pod, refreshed after a minute);
* output.conf — the elasticsearch output: logstash_format (`logstash-YYYY.MM.DD` by record
  time), include_tag_key, buffer_chunk_limit 2M, buffer_queue_limit 8, flush_interval 5s,
  retries doubling to max_retry_wait 30s with no retry limit. A full queue pauses reading
  (the files are the buffer) instead of dropping;
* pos_file — per file inode and offset, written after each delivered chunk, so a restart
  resumes where delivery stopped; a rotated (new inode) or truncated file starts from 0.
"""
from __future__ import annotations

import asyncio
import datetime
import glob
import json
import logging
import os
import re
import time

log = logging.getLogger("amdkube.log-shipper")

CONTAINER_LOG = re.compile(r"^(?P<pod>[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*)_(?P<ns>[^_]+)_"
                           r"(?P<container>.+)-(?P<cid>[a-z0-9]+)\.log$")
CRI_LINE = re.compile(r"^(?P<time>\S+) (?P<stream>stdout|stderr) (?P<tag>[PF]) ?(?P<log>.*)$", re.S)
GLOG_FIRST = re.compile(r"^\w\d{4}")
GLOG = re.compile(r"^(?P<severity>\w)(?P<time>\d{4} [^\s]*)\s+(?P<pid>\d+)\s+(?P<source>[^ \]]+)\] (?P<message>.*)", re.S)


def _now_iso() -> str:
    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_container_line(line: str):
    """-> (record, partial) for one line of a container log."""
    if line.startswith("{"):
        try:
            d = json.loads(line)
            if isinstance(d, dict) and "log" in d:
                return {"log": d["log"], "stream": d.get("stream", "stdout"), "time": d.get("time") or _now_iso()}, False
        except ValueError:
            pass
    m = CRI_LINE.match(line)
    if m:
        return {"log": m["log"] + ("" if m["tag"] == "P" else "\n"), "stream": m["stream"], "time": m["time"]}, m["tag"] == "P"
    return {"log": line + "\n", "stream": "stdout", "time": _now_iso()}, False


def parse_glog(text: str, year: int | None = None) -> dict:
    m = GLOG.match(text)
    if not m:
        return {"message": text, "time": _now_iso()}
    year = year or datetime.datetime.now(datetime.timezone.utc).year
    try:
        t = datetime.datetime.strptime(f"{year}{m['time']}", "%Y%m%d %H:%M:%S.%f").replace(tzinfo=datetime.timezone.utc)
        ts = t.strftime("%Y-%m-%dT%H:%M:%S.%fZ")
    except ValueError:
        ts = _now_iso()
    return {"severity": m["severity"], "pid": m["pid"], "source": m["source"], "message": m["message"], "time": ts}


def index_for(ts: str, prefix: str = "logstash") -> str:
    return f"{prefix}-{ts[:4]}.{ts[5:7]}.{ts[8:10]}" if re.match(r"\d{4}-\d{2}-\d{2}", ts or "") else \
        f"{prefix}-{datetime.datetime.now(datetime.timezone.utc):%Y.%m.%d}"


class Tail:
    """One followed file: inode + offset, complete lines only."""

    def __init__(self, path: str, tag: str, kind: str, pos: dict | None = None):
        self.path, self.tag, self.kind = path, tag, kind
        self.inode, self.offset = (pos or {}).get("inode"), (pos or {}).get("offset", 0)
        self.pending = ""          # glog: the record being assembled; container: a partial CRI line
        self.pending_rec: dict | None = None

    def read_lines(self, limit: int) -> list[str]:
        try:
            st = os.stat(self.path)
        except OSError:
            return []
        if st.st_ino != self.inode or st.st_size < self.offset:
            self.inode, self.offset = st.st_ino, 0        # new or rotated or truncated: from the start
        if st.st_size == self.offset:
            return []
        with open(self.path, "rb") as f:
            f.seek(self.offset)
            data = f.read(limit)
        cut = data.rfind(b"\n")
        if cut < 0:
            return []
        self.offset += cut + 1
        return data[:cut].decode(errors="replace").split("\n")


class Shipper:
    def __init__(self, es_url: str, containers_glob: str = "/var/log/containers/*.log", component_logs=(),
                 pos_file: str = "/var/log/amdkube-log-shipper.pos", client=None, node_name: str = "",
                 flush_interval: float = 5.0, chunk_limit: int = 2 << 20, queue_limit: int = 8, max_retry_wait: float = 30.0,
                 index_prefix: str = "logstash"):
        self.es_url = es_url.rstrip("/")
        self.containers_glob, self.component_logs = containers_glob, list(component_logs)
        self.pos_file, self.client, self.node_name = pos_file, client, node_name
        self.flush_interval, self.chunk_limit, self.queue_limit = flush_interval, chunk_limit, queue_limit
        self.max_retry_wait, self.prefix = max_retry_wait, index_prefix
        self.tails: dict[str, Tail] = {}
        self._pods: dict[tuple[str, str], tuple[float, dict | None]] = {}
        self.queue: list[tuple[bytes, dict]] = []      # (bulk body, positions once delivered)
        self.stats = {"records": 0, "chunks": 0, "retries": 0, "errors": 0}
        self._load_pos()

    # ------------------------------------------------------------------ positions
    def _load_pos(self):
        try:
            with open(self.pos_file) as f:
                self._saved = json.load(f)
        except (OSError, ValueError):
            self._saved = {}

    def _save_pos(self, positions: dict):
        self._saved.update(positions)
        self._saved = {p: v for p, v in self._saved.items() if os.path.exists(p)}
        tmp = self.pos_file + ".tmp"
        os.makedirs(os.path.dirname(self.pos_file) or ".", exist_ok=True)
        with open(tmp, "w") as f:
            json.dump(self._saved, f)
        os.replace(tmp, self.pos_file)

    # ------------------------------------------------------------------ sources
    def discover(self):
        for p in glob.glob(self.containers_glob):
            if p not in self.tails and CONTAINER_LOG.match(os.path.basename(p)):
                tag = "kubernetes." + p.strip("/").replace("/", ".")
                self.tails[p] = Tail(p, tag, "container", self._saved.get(p))
        for spec in self.component_logs:
            path, _, tag = spec.partition(":")
            if path not in self.tails:
                self.tails[path] = Tail(path, tag or os.path.basename(path).rsplit(".", 1)[0], "glog", self._saved.get(path))
        for p in [p for p in self.tails if not os.path.exists(p)]:
            del self.tails[p]

    async def _pod(self, ns: str, name: str) -> dict | None:
        if self.client is None:
            return None
        hit = self._pods.get((ns, name))
        if hit and time.monotonic() - hit[0] < 60:
            return hit[1]
        try:
            pod = await self.client.get_or_none("pods", name, ns)
        except Exception as e:
            log.debug("pod %s/%s metadata: %r", ns, name, e)
            pod = hit[1] if hit else None
        self._pods[(ns, name)] = (time.monotonic(), pod)
        return pod

    async def _enrich(self, t: Tail, rec: dict) -> dict:
        m = CONTAINER_LOG.match(os.path.basename(t.path))
        pod = await self._pod(m["ns"], m["pod"])
        md = (pod or {}).get("metadata") or {}
        k = {"pod_name": m["pod"], "namespace_name": m["ns"], "container_name": m["container"],
             "host": ((pod or {}).get("spec") or {}).get("nodeName") or self.node_name}
        if md.get("uid"):
            k["pod_id"] = md["uid"]
        if md.get("labels"):
            k["labels"] = md["labels"]
        rec["kubernetes"] = k
        rec["docker"] = {"container_id": m["cid"]}
        return rec

    async def _records(self, t: Tail, budget: int) -> list[dict]:
        out = []
        for line in t.read_lines(budget):
            if t.kind == "container":
                rec, partial = parse_container_line(line)
                if t.pending_rec is not None:
                    t.pending_rec["log"] += rec["log"]
                    rec, t.pending_rec = t.pending_rec, None
                if partial:
                    t.pending_rec = rec
                    continue
                out.append(await self._enrich(t, rec))
            else:
                if GLOG_FIRST.match(line) and t.pending:
                    out.append(parse_glog(t.pending))
                    t.pending = ""
                t.pending = f"{t.pending}\n{line}" if t.pending else line
        if t.kind == "glog" and t.pending and t.offset == os.path.getsize(t.path):
            out.append(parse_glog(t.pending))      # the file's last record is complete once nothing follows
            t.pending = ""
        return out

    # ------------------------------------------------------------------ buffer / output
    def _chunk(self, batch: list[tuple[str, dict]]) -> bytes:
        parts = []
        for tag, rec in batch:
            ts = rec.pop("time", None) or _now_iso()
            doc = dict(rec, **{"@timestamp": ts, "tag": tag})
            parts.append(json.dumps({"index": {"_index": index_for(ts, self.prefix), "_type": "fluentd"}},
                                    separators=(",", ":")))
            parts.append(json.dumps(doc, separators=(",", ":")))
        return ("\n".join(parts) + "\n").encode()

    async def collect(self) -> int:
        """Read what the files have (up to the free queue room) into chunks; how many records."""
        self.discover()
        n = 0
        for t in list(self.tails.values()):
            while len(self.queue) < self.queue_limit:
                recs = await self._records(t, self.chunk_limit // 2)
                if not recs:
                    break
                self.queue.append((self._chunk([(t.tag, r) for r in recs]), {t.path: {"inode": t.inode, "offset": t.offset}}))
                n += len(recs)
        self.stats["records"] += n
        return n

    async def flush(self, session) -> bool:
        """Deliver queued chunks in order; False when the store refused (retry later)."""
        while self.queue:
            body, positions = self.queue[0]
            try:
                async with session.post(f"{self.es_url}/_bulk", data=body,
                                        headers={"Content-Type": "application/x-ndjson"}) as r:
                    res = await r.json(content_type=None)
                    if r.status >= 300:
                        raise RuntimeError(f"HTTP {r.status}: {res}")
            except Exception as e:
                self.stats["errors"] += 1
                log.warning("elasticsearch %s: %s", self.es_url, e)
                return False
            if (res or {}).get("errors"):
                # per-document rejections (mapping errors) are not retried, as fluent-plugin-elasticsearch
                log.warning("elasticsearch rejected %d record(s)",
                            sum(1 for it in res.get("items", []) for v in it.values() if v.get("status", 200) >= 300))
            self.queue.pop(0)
            self.stats["chunks"] += 1
            self._save_pos(positions)
        return True

    async def run(self, stop: asyncio.Event | None = None):
        import aiohttp
        stop = stop or asyncio.Event()
        wait = 1.0
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30)) as session:
            while not stop.is_set():
                await self.collect()
                if await self.flush(session):
                    wait, delay = 1.0, self.flush_interval
                else:
                    self.stats["retries"] += 1
                    delay, wait = wait, min(self.max_retry_wait, wait * 2)
                try:
                    await asyncio.wait_for(stop.wait(), delay)
                except asyncio.TimeoutError:
                    pass
            await self.collect()
            await self.flush(session)
