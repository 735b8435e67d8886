"""Job store with Elasticsearch-document semantics.

The reference keeps every analysis job as a document in the ES index
``documents`` (``foremast-service/pkg/search/elasticsearchstore.go``); the
service creates it with ``status: "initial"`` and the brain moves it through
the state diagram.  This module provides that table behind one interface:

* :class:`MemoryJobStore` — in-process (tests, single-process deployments);
* :class:`SqliteJobStore` — durable, shareable by several brain processes on
  one host (checkpoint/resume: a restarted brain re-claims open jobs);
* ``foremast_amd.store.es.ElasticJobStore`` — talks to a real ES 6.x so the
  engine can replace the reference brain next to the reference service.

Job ids are content addressed: HMAC-SHA256 with an empty key over the
concatenated request fields (``foremast-service/pkg/common/stringutils.go:11-17``),
so an identical request returns the same job (idempotent create).

Claims are lease based: a worker may take a job whose status
is open (``initial``/``reprogress``) or that has been in progress longer than
``MAX_STUCK_IN_SECONDS`` (stuck-job takeover, ``foremast-brain.yaml:80-81``).
"""

from __future__ import annotations

import abc
import copy
import hashlib
import hmac
import json
import os
import sqlite3
import threading
import time
from typing import Any, Dict, Iterable, List, Optional

from ..api import rest as r
from ..utils.timeutil import format_rfc3339_nano, parse_rfc3339


def job_id_for(req: r.DocumentRequest) -> str:
    """``UUIDGen(ConvertDocumentRequestToString(doc))``."""
    return hmac.new(b"", req.hash_input().encode("utf-8"), hashlib.sha256).hexdigest()


def new_document(req: r.DocumentRequest, job_id: str, now: Optional[float] = None) -> Dict[str, Any]:
    """Build the ES document (``elasticsearchstore.go:37-53``).

    Raises :class:`~foremast_amd.utils.timeutil.TimeFormatError` on a bad
    start/end time (the reference crashes the process — Q5).
    """
    now = time.time() if now is None else now
    start = parse_rfc3339(req.start_time) if req.start_time else None
    end = parse_rfc3339(req.end_time) if req.end_time else None
    ts = format_rfc3339_nano(now)
    return {
        "id": job_id,
        "appName": req.app_name,
        "created_at": ts,
        "startTime": format_rfc3339_nano(start.timestamp()) if start else "0001-01-01T00:00:00Z",
        "endTime": format_rfc3339_nano(end.timestamp()) if end else "0001-01-01T00:00:00Z",
        "modified_at": ts,
        "currentConfig": req.current_config,
        "baselineConfig": req.baseline_config,
        "historicalConfig": req.historical_config,
        "currentMetricStore": req.current_metric_store,
        "baselineMetricStore": req.baseline_metric_store,
        "historicalMetricStore": req.historical_metric_store,
        "status": r.ST_INITIAL,
        "statusCode": req.status_code,
        "strategy": req.strategy,
        "reason": "",
        "processingContent": "",
        "anomalyInfo": "",
        # engine-side lease bookkeeping (ignored by the reference service)
        "claimed_by": "",
        "claimed_at": 0.0,
        "modified_ts": now,
    }


def is_claimable(doc: Dict[str, Any], now: float, max_stuck_s: float, steal_from=None,
                 beats: Optional[Dict[str, float]] = None) -> bool:
    """Open (and due), stuck for longer than ``max_stuck_s``, or leased by a
    worker in ``steal_from`` (a brain rank the node has declared dead: its jobs
    move at once instead of after the stuck-job timeout).

    A lease is alive while the document was modified, or its holder sent a
    worker heartbeat (``beats``: worker -> last :meth:`JobStore.heartbeat`),
    within ``max_stuck_s``: a resident engine holding 100k series renews all of
    its leases with one heartbeat per tick instead of one write per job."""
    st = doc.get("status")
    if st in r.OPEN_STATUSES:
        return float(doc.get("not_before", 0.0) or 0.0) <= now
    if st in r.INPROGRESS_STATUSES:
        holder = doc.get("claimed_by")
        if steal_from and holder in steal_from:
            return True
        alive = float(doc.get("modified_ts", 0.0) or 0.0)
        if beats and holder:
            alive = max(alive, float(beats.get(holder, 0.0)))
        return now - alive > max_stuck_s
    return False


class JobStore(abc.ABC):
    """The shared job table."""

    @abc.abstractmethod
    def get(self, job_id: str) -> Optional[Dict[str, Any]]: ...

    @abc.abstractmethod
    def _insert_if_absent(self, doc: Dict[str, Any]) -> bool: ...

    @abc.abstractmethod
    def update(self, job_id: str, fields: Dict[str, Any],
               expect_claimed_by: Optional[str] = None) -> bool:
        """Patch a document; with ``expect_claimed_by`` the write only lands if
        the caller still holds the lease (lost-update protection)."""

    def update_many(self, items: List[tuple], expect_claimed_by: Optional[str] = None) -> List[bool]:
        """``update`` for many ``(job_id, fields)`` (one transaction / lock where
        the backend has one); returns which writes landed."""
        return [self.update(j, f, expect_claimed_by=expect_claimed_by) for j, f in items]

    @abc.abstractmethod
    def claim(self, worker: str, now: Optional[float] = None, max_stuck_s: float = 90.0,
              limit: int = 64, only=None, steal_from=None, only_batch=None) -> List[Dict[str, Any]]:
        """Lease up to ``limit`` claimable documents (``only(doc)`` filters,
        e.g. by strategy: the streaming monitor takes continuous jobs;
        ``only_batch(docs) -> [bool]`` is the same filter over every candidate at
        once (the rollout engine decodes a deploy burst in one native batch);
        ``steal_from``: worker ids whose leases are void, see is_claimable)."""

    @abc.abstractmethod
    def heartbeat(self, worker: str, now: Optional[float] = None) -> None:
        """Renew every lease ``worker`` holds (see :func:`is_claimable`)."""

    @abc.abstractmethod
    def all(self) -> List[Dict[str, Any]]: ...

    # small engine-side records next to the job table (e.g. the node health table
    # rank 0 publishes for GET /v1/healthcheck/cluster)
    @abc.abstractmethod
    def put_meta(self, key: str, value: Dict[str, Any]) -> None: ...

    @abc.abstractmethod
    def get_meta(self, key: str) -> Optional[Dict[str, Any]]: ...

    def create(self, req: r.DocumentRequest, now: Optional[float] = None) -> str:
        job_id = job_id_for(req)
        if self.get(job_id) is None:
            self._insert_if_absent(new_document(req, job_id, now))
        return job_id

    def by_status(self, statuses: Iterable[str]) -> List[Dict[str, Any]]:
        s = set(statuses)
        return [d for d in self.all() if d.get("status") in s]

    def close(self) -> None:
        pass


def _filter(cand: List[Dict[str, Any]], only, only_batch) -> List[Dict[str, Any]]:
    """Candidates passing ``only`` / ``only_batch`` (in order)."""
    if only_batch is not None and cand:
        cand = [d for d, ok in zip(cand, only_batch(cand)) if ok]
    if only is not None:
        cand = [d for d in cand if only(d)]
    return cand


_STAMP_CACHE: Dict[float, str] = {}


_FLAT = frozenset((str, int, float, bool, type(None)))


def _flat_copy(fields: Dict[str, Any]) -> Dict[str, Any]:
    """A copy that shares nothing mutable: job documents are flat (str / number
    values), so a dict copy suffices; nested values are deep-copied."""
    for v in fields.values():
        if type(v) not in _FLAT:
            return copy.deepcopy(fields)
    return dict(fields)


def _stamp(d: Dict[str, Any], fields: Dict[str, Any]) -> None:
    d.update(fields)
    ts = fields.get("modified_ts", time.time())
    d["modified_ts"] = ts
    at = _STAMP_CACHE.get(ts)
    if at is None:  # a tick's writes share one timestamp: format it once
        if len(_STAMP_CACHE) > 64:
            _STAMP_CACHE.clear()
        at = _STAMP_CACHE[ts] = format_rfc3339_nano(ts)
    d["modified_at"] = at


class MemoryJobStore(JobStore):
    """In-process table with claim indexes: open documents and in-progress
    documents per lease holder, so a claim touches only the open jobs and the
    leases of workers whose heartbeat is stale — not every document ever
    created (a node holds tens of thousands of running jobs)."""

    def __init__(self) -> None:
        self._docs: Dict[str, Dict[str, Any]] = {}
        self._meta: Dict[str, Dict[str, Any]] = {}
        self._open: Dict[str, Dict[str, Any]] = {}
        self._held: Dict[str, Dict[str, Dict[str, Any]]] = {}   # holder -> in-progress docs
        self._beats: Dict[str, float] = {}
        self._lock = threading.RLock()

    def _index(self, d: Dict[str, Any], before: Optional[tuple] = None) -> None:
        """Move ``d`` between the claim indexes after a status / holder change
        (``before``: its (status, claimed_by) prior to the change)."""
        jid = d["id"]
        if before is not None:
            st, holder = before
            if st in r.OPEN_STATUSES:
                self._open.pop(jid, None)
            elif st in r.INPROGRESS_STATUSES:
                h = self._held.get(holder or "")
                if h is not None:
                    h.pop(jid, None)
                    if not h:
                        del self._held[holder or ""]
        st = d.get("status")
        if st in r.OPEN_STATUSES:
            self._open[jid] = d
        elif st in r.INPROGRESS_STATUSES:
            self._held.setdefault(d.get("claimed_by") or "", {})[jid] = d

    def get(self, job_id):
        with self._lock:
            d = self._docs.get(job_id)
            return copy.deepcopy(d) if d is not None else None

    def _insert_if_absent(self, doc):
        with self._lock:
            if doc["id"] in self._docs:
                return False
            d = copy.deepcopy(doc)
            self._docs[doc["id"]] = d
            self._index(d)
            return True

    def _update_locked(self, job_id, fields, expect_claimed_by):
        d = self._docs.get(job_id)
        if d is None:
            return False
        if expect_claimed_by is not None and d.get("claimed_by") != expect_claimed_by:
            return False
        before = (d.get("status"), d.get("claimed_by"))
        _stamp(d, _flat_copy(fields))
        self._index(d, before)
        return True

    def update(self, job_id, fields, expect_claimed_by=None):
        with self._lock:
            return self._update_locked(job_id, fields, expect_claimed_by)

    def update_many(self, items, expect_claimed_by=None):
        with self._lock:
            return [self._update_locked(j, f, expect_claimed_by) for j, f in items]

    def heartbeat(self, worker, now=None):
        with self._lock:
            self._beats[worker] = time.time() if now is None else float(now)

    def claim(self, worker, now=None, max_stuck_s=90.0, limit=64, only=None, steal_from=None, only_batch=None):
        now = time.time() if now is None else now
        out = []
        stamp = format_rfc3339_nano(now)
        with self._lock:
            cand = list(self._open.values())
            for holder, docs in self._held.items():
                if steal_from and holder in steal_from:
                    cand.extend(docs.values())
                elif now - self._beats.get(holder, 0.0) > max_stuck_s:
                    cand.extend(d for d in docs.values() if now - float(d.get("modified_ts", 0.0) or 0.0) > max_stuck_s)
            cand.sort(key=lambda x: x.get("modified_ts", 0.0))
            cand = [d for d in cand if is_claimable(d, now, max_stuck_s, steal_from, self._beats)]
            for d in _filter(cand, only, only_batch)[:limit]:
                before = (d.get("status"), d.get("claimed_by"))
                d["status"] = r.ST_PREPROCESS_INPROGRESS
                d["claimed_by"] = worker
                d["claimed_at"] = now
                d["modified_ts"] = now
                d["modified_at"] = stamp
                self._index(d, before)
                out.append(dict(d))  # documents are flat (str / number values): a shallow copy is a copy
        return out

    def all(self):
        with self._lock:
            return [copy.deepcopy(d) for d in self._docs.values()]

    def put_meta(self, key, value):
        with self._lock:
            self._meta[key] = copy.deepcopy(value)

    def get_meta(self, key):
        with self._lock:
            v = self._meta.get(key)
            return copy.deepcopy(v) if v is not None else None


class SqliteJobStore(JobStore):
    """Durable store; safe across processes (``BEGIN IMMEDIATE`` claims).  The
    claim query selects only due open documents and in-progress documents whose
    lease (document write and holder heartbeat) is stale, through indexed columns."""

    def __init__(self, path: str) -> None:
        self.path = path
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._local = threading.local()
        with self._conn() as c:
            c.execute("PRAGMA journal_mode=WAL")
            c.execute("CREATE TABLE IF NOT EXISTS documents ("
                      "id TEXT PRIMARY KEY, status TEXT, modified_ts REAL, doc TEXT)")
            cols = {row[1] for row in c.execute("PRAGMA table_info(documents)")}
            added = False
            for col, decl in (("claimed_by", "TEXT DEFAULT ''"), ("not_before", "REAL DEFAULT 0")):
                if col not in cols:  # stores written by an older version
                    c.execute(f"ALTER TABLE documents ADD COLUMN {col} {decl}")
                    added = True
            if added:  # the new columns index what the JSON documents already say
                c.execute("UPDATE documents SET claimed_by=COALESCE(json_extract(doc,'$.claimed_by'),''), "
                          "not_before=COALESCE(json_extract(doc,'$.not_before'),0)")
            c.execute("CREATE INDEX IF NOT EXISTS documents_status ON documents(status, modified_ts)")
            c.execute("CREATE TABLE IF NOT EXISTS meta (key TEXT PRIMARY KEY, value TEXT)")
            c.execute("CREATE TABLE IF NOT EXISTS workers (worker TEXT PRIMARY KEY, beat REAL)")

    def _conn(self) -> sqlite3.Connection:
        c = getattr(self._local, "conn", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30.0, isolation_level=None)
            self._local.conn = c
        return c

    def get(self, job_id):
        row = self._conn().execute("SELECT doc FROM documents WHERE id=?", (job_id,)).fetchone()
        return json.loads(row[0]) if row else None

    def _insert_if_absent(self, doc):
        cur = self._conn().execute(
            "INSERT OR IGNORE INTO documents(id, status, modified_ts, doc, claimed_by, not_before) "
            "VALUES (?,?,?,?,?,?)",
            (doc["id"], doc["status"], doc["modified_ts"], json.dumps(doc), doc.get("claimed_by", ""),
             float(doc.get("not_before", 0.0) or 0.0)))
        return cur.rowcount == 1

    def _write(self, c, d):
        c.execute("UPDATE documents SET status=?, modified_ts=?, doc=?, claimed_by=?, not_before=? WHERE id=?",
                  (d["status"], d["modified_ts"], json.dumps(d), d.get("claimed_by", "") or "",
                   float(d.get("not_before", 0.0) or 0.0), d["id"]))

    def _update_in(self, c, job_id, fields, expect_claimed_by):
        row = c.execute("SELECT doc FROM documents WHERE id=?", (job_id,)).fetchone()
        if row is None:
            return False
        d = json.loads(row[0])
        if expect_claimed_by is not None and d.get("claimed_by") != expect_claimed_by:
            return False
        _stamp(d, fields)
        self._write(c, d)
        return True

    def update(self, job_id, fields, expect_claimed_by=None):
        return self.update_many([(job_id, fields)], expect_claimed_by)[0]

    def update_many(self, items, expect_claimed_by=None):
        c = self._conn()
        c.execute("BEGIN IMMEDIATE")
        try:
            res = [self._update_in(c, j, f, expect_claimed_by) for j, f in items]
            c.execute("COMMIT")
            return res
        except Exception:
            c.execute("ROLLBACK")
            raise

    def heartbeat(self, worker, now=None):
        self._conn().execute("INSERT OR REPLACE INTO workers(worker, beat) VALUES (?, ?)",
                             (worker, time.time() if now is None else float(now)))

    def claim(self, worker, now=None, max_stuck_s=90.0, limit=64, only=None, steal_from=None, only_batch=None):
        now = time.time() if now is None else now
        cutoff = now - max_stuck_s
        steal = sorted(steal_from or ())
        c = self._conn()
        c.execute("BEGIN IMMEDIATE")
        try:
            q_open = ",".join("?" * len(r.OPEN_STATUSES))
            q_prog = ",".join("?" * len(r.INPROGRESS_STATUSES))
            q_steal = ("OR claimed_by IN (" + ",".join("?" * len(steal)) + ")") if steal else ""
            rows = c.execute(
                f"SELECT doc FROM documents WHERE (status IN ({q_open}) AND not_before <= ?) OR "
                f"(status IN ({q_prog}) AND ((modified_ts < ? AND COALESCE((SELECT beat FROM workers w "
                f"WHERE w.worker = documents.claimed_by), 0) < ?) {q_steal})) ORDER BY modified_ts",
                r.OPEN_STATUSES + (now,) + r.INPROGRESS_STATUSES + (cutoff, cutoff) + tuple(steal)).fetchall()
            out = []
            cand = [d for d in (json.loads(raw) for (raw,) in rows) if is_claimable(d, now, max_stuck_s, steal_from)]
            stamp = format_rfc3339_nano(now)
            for d in _filter(cand, only, only_batch)[:limit]:
                d.update(status=r.ST_PREPROCESS_INPROGRESS, claimed_by=worker, claimed_at=now,
                         modified_ts=now, modified_at=stamp)
                self._write(c, d)
                out.append(d)
            c.execute("COMMIT")
            return out
        except Exception:
            c.execute("ROLLBACK")
            raise

    def all(self):
        return [json.loads(x[0]) for x in self._conn().execute("SELECT doc FROM documents")]

    def put_meta(self, key, value):
        self._conn().execute("INSERT OR REPLACE INTO meta(key, value) VALUES (?, ?)", (key, json.dumps(value)))

    def get_meta(self, key):
        row = self._conn().execute("SELECT value FROM meta WHERE key=?", (key,)).fetchone()
        return json.loads(row[0]) if row else None

    def close(self):
        c = getattr(self._local, "conn", None)
        if c is not None:
            c.close()
            self._local.conn = None


def open_store(url: Optional[str]) -> JobStore:
    """``memory://`` | ``sqlite:///path`` | ``http(s)://es-host:9200`` (ES)."""
    if not url or url.startswith("memory"):
        return MemoryJobStore()
    if url.startswith("sqlite://"):
        return SqliteJobStore(url[len("sqlite://"):] or "foremast_jobs.db")
    if url.startswith("http://") or url.startswith("https://"):
        from .es import ElasticJobStore
        return ElasticJobStore(url)
    return SqliteJobStore(url)
