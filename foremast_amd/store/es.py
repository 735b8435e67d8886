"""Elasticsearch 6.x job store (index ``documents``, type ``document``).

Drop-in for the reference deployment: the reference service writes job docs
into ES (``foremast-service/pkg/search/elasticsearchstore.go:17-18,37-53``)
and brains poll them.  This store speaks the same REST surface so the engine
can run next to the reference service, or the reference brain next to our
service:

* create  — ``PUT /documents/document/<id>/_create`` (409 ⇒ already exists,
  i.e. idempotent create of a content-addressed job);
* get     — ``GET /documents/document/<id>`` (``_source`` + ``_version``);
* update  — read-modify-write with ``?version=<v>`` (ES internal optimistic
  concurrency, available on 6.x) so two brains never both win a claim and a
  worker that lost its lease cannot overwrite the new owner's result;
* claim   — ``_search`` for open / in-progress docs, then one versioned
  write per candidate; only writes that land are returned.

The reference reconnects to ES every 3 s until it is up
(``foremast-service/cmd/manager/main.go:248-260``); :meth:`wait_ready` does
the same with a deadline instead of looping forever.
"""

from __future__ import annotations

import json
import time
from typing import Any, Dict, List, Optional, Tuple

import httpx

from ..api import rest as r
from ..utils.timeutil import format_rfc3339_nano
from .jobstore import JobStore, _filter, is_claimable

INDEX = "documents"
DOC_TYPE = "document"
META_INDEX = "foremast-engine"
# Worker heartbeats (lease renewal) get an index of their own: ES 6.x allows one mapping
# type per index, so they cannot share META_INDEX (type ``document``) under another type.
BEAT_INDEX = "foremast-workers"
PAGE = 1000  # hits per search page


def _kw_of(mapping: Dict[str, Any], field: str) -> Optional[str]:
    """Exact-match name of a string field under an index mapping (the ``properties``
    of its one type), or None when the mapping does not say yet.  Under ES dynamic
    mapping (how the reference service creates ``documents``:
    ``elasticsearchstore.go:54-59`` indexes without a mapping) a string is analysed
    ``text`` — ``node-m0-rollout`` is stored as the tokens ``node`` / ``m0`` /
    ``rollout`` — with an exact ``.keyword`` sub-field, which ``terms`` filters must
    use; an operator-created index that maps the field as ``keyword`` has no such
    sub-field and is matched on the bare field."""
    spec = mapping.get(field)
    if not isinstance(spec, dict):
        return None
    if spec.get("type") == "keyword":
        return field
    sub = spec.get("fields") or {}
    for name, f in sub.items():
        if isinstance(f, dict) and f.get("type") == "keyword":
            return f"{field}.{name}"
    return None


class ElasticJobStore(JobStore):
    def __init__(self, url: str, index: str = INDEX, doc_type: str = DOC_TYPE, timeout: float = 10.0,
                 transport: Optional[httpx.BaseTransport] = None, refresh: str = "true") -> None:
        self.base = url.rstrip("/")
        self.index, self.doc_type = index, doc_type
        self.refresh = refresh
        kw: Dict[str, Any] = {"timeout": timeout}
        if transport is not None:
            kw["transport"] = transport
        self.http = httpx.Client(**kw)
        self._kw_cache: Dict[str, str] = {}
        self._kw_miss: Dict[str, float] = {}   # field -> time of the last mapping read that did not name it
        self.kw_miss_ttl_s = 30.0

    def _kw(self, field: str) -> str:
        """Exact-match name of ``field`` in the job index, read from the index mapping
        once it names the field (dynamic mapping: ``<field>.keyword``; an explicit
        ``keyword`` mapping: the bare field).  Until then the dynamic-mapping name is
        used, and the mapping is asked again only after ``kw_miss_ttl_s`` (a negative
        answer is cached too: otherwise every search before the field's first write
        would cost one more round trip)."""
        got = self._kw_cache.get(field)
        if got is not None:
            return got
        miss = self._kw_miss.get(field)
        if miss is not None and time.monotonic() - miss < self.kw_miss_ttl_s:
            return field + ".keyword"
        name = None
        try:
            resp = self.http.get(f"{self.base}/{self.index}/_mapping")
            if resp.status_code == 200:
                for idx in resp.json().values():
                    mappings = idx.get("mappings") or {}
                    # ES 6.x: {type: {properties}}; a typeless (7.x) index: {properties}
                    types = [mappings] if "properties" in mappings else list(mappings.values())
                    for typ in types:
                        name = name or _kw_of((typ or {}).get("properties") or {}, field)
        except (httpx.HTTPError, ValueError, AttributeError):
            name = None
        if name is None:
            self._kw_miss[field] = time.monotonic()
            return field + ".keyword"
        self._kw_miss.pop(field, None)
        self._kw_cache[field] = name
        return name

    # ------------------------------------------------------------------ plumbing
    def _doc_url(self, job_id: str, suffix: str = "") -> str:
        return f"{self.base}/{self.index}/{self.doc_type}/{job_id}{suffix}"

    def wait_ready(self, deadline_s: float = 60.0, every_s: float = 3.0) -> None:
        t_end = time.time() + deadline_s
        while True:
            try:
                if self.http.get(self.base + "/").status_code < 500:
                    return
            except httpx.HTTPError:
                pass
            if time.time() >= t_end:
                raise ConnectionError(f"elasticsearch at {self.base} not reachable")
            time.sleep(every_s)

    def _get_versioned(self, job_id: str) -> Tuple[Optional[Dict[str, Any]], int]:
        resp = self.http.get(self._doc_url(job_id))
        if resp.status_code == 404:
            return None, 0
        resp.raise_for_status()
        body = resp.json()
        if not body.get("found", False):
            return None, 0
        return body["_source"], int(body.get("_version", 1))

    def _put_versioned(self, doc: Dict[str, Any], version: int) -> bool:
        resp = self.http.put(self._doc_url(doc["id"]), params={"version": version, "refresh": self.refresh},
                             content=json.dumps(doc), headers={"Content-Type": "application/json"})
        if resp.status_code == 409:
            return False
        resp.raise_for_status()
        return True

    # ------------------------------------------------------------------ JobStore
    def get(self, job_id):
        return self._get_versioned(job_id)[0]

    def _insert_if_absent(self, doc):
        resp = self.http.put(self._doc_url(doc["id"], "/_create"), params={"refresh": self.refresh},
                             content=json.dumps(doc), headers={"Content-Type": "application/json"})
        if resp.status_code == 409:
            return False
        resp.raise_for_status()
        return True

    def update(self, job_id, fields, expect_claimed_by=None, retries: int = 5):
        for _ in range(retries):
            d, ver = self._get_versioned(job_id)
            if d is None:
                return False
            if expect_claimed_by is not None and d.get("claimed_by") != expect_claimed_by:
                return False
            d.update(fields)
            d["modified_ts"] = fields.get("modified_ts", time.time())
            d["modified_at"] = format_rfc3339_nano(d["modified_ts"])
            if self._put_versioned(d, ver):
                return True
        return False

    def _search(self, statuses, size: int = PAGE, extra=(), must_not=(), index: Optional[str] = None,
                doc_type: Optional[str] = None, offset: int = 0) -> List[Tuple[Dict[str, Any], int]]:
        filt = ([{"terms": {self._kw("status"): list(statuses)}}] if statuses else []) + list(extra)
        body = {"query": {"bool": {"filter": filt, "must_not": list(must_not)}}, "from": offset,
                "size": size, "version": True, "sort": [{"modified_ts": {"order": "asc"}}]}
        resp = self.http.post(f"{self.base}/{index or self.index}/{doc_type or self.doc_type}/_search",
                              content=json.dumps(body), headers={"Content-Type": "application/json"})
        if resp.status_code == 404:  # index not created yet
            return []
        resp.raise_for_status()
        hits = resp.json().get("hits", {}).get("hits", [])
        return [(h["_source"], int(h.get("_version", 1))) for h in hits]

    def _search_pages(self, statuses, want: int, max_pages: int = 10, **kw) -> List[Tuple[Dict[str, Any], int]]:
        """Oldest-first pages until ``want`` hits or the result is exhausted."""
        out: List[Tuple[Dict[str, Any], int]] = []
        for p in range(max_pages):
            page = self._search(statuses, offset=p * PAGE, **kw)
            out += page
            if len(page) < PAGE or len(out) >= want:
                break
        return out

    def heartbeat(self, worker, now=None):
        now = time.time() if now is None else float(now)
        resp = self.http.put(f"{self.base}/{BEAT_INDEX}/{self.doc_type}/{worker}", params={"refresh": self.refresh},
                             content=json.dumps({"worker": worker, "beat": now, "modified_ts": now}),
                             headers={"Content-Type": "application/json"})
        resp.raise_for_status()

    def _beats(self, since: float) -> Dict[str, float]:
        hits = self._search((), size=10000, extra=[{"range": {"beat": {"gte": since}}}], index=BEAT_INDEX)
        return {d["worker"]: float(d["beat"]) for d, _ in hits if "worker" in d}

    def claim(self, worker, now=None, max_stuck_s=90.0, limit=64, only=None, steal_from=None, only_batch=None):
        """Two searches, so open jobs are never hidden behind thousands of live
        leases: due open documents, then in-progress ones whose lease is stale
        (not modified within ``max_stuck_s`` and the holder has no fresh
        heartbeat) or held by a worker in ``steal_from``."""
        now = time.time() if now is None else now
        cutoff = now - max_stuck_s
        beats = self._beats(cutoff)
        # not_before is checked below (docs of other writers lack it)
        cand = self._search_pages(r.OPEN_STATUSES, 4 * PAGE)
        # stale leases: live workers' leases are filtered out in the query (they are renewed by
        # heartbeat, so their modified_ts is old) and the rest is paged, so stuck jobs are never
        # crowded out of the oldest-first window
        cand += self._search_pages(r.INPROGRESS_STATUSES, 4 * PAGE,
                                   extra=[{"range": {"modified_ts": {"lt": cutoff}}}],
                                   must_not=[{"terms": {self._kw("claimed_by"): sorted(beats)}}] if beats else [])
        if steal_from:
            cand += self._search_pages(r.INPROGRESS_STATUSES, 4 * PAGE,
                                       extra=[{"terms": {self._kw("claimed_by"): sorted(steal_from)}}])
        seen, keep = set(), []
        for d, ver in sorted(cand, key=lambda dv: dv[0].get("modified_ts", 0.0)):
            if d["id"] in seen:
                continue
            seen.add(d["id"])
            if is_claimable(d, now, max_stuck_s, steal_from, beats):
                keep.append((d, ver))
        vers = {id(d): ver for d, ver in keep}
        out = []
        stamp = format_rfc3339_nano(now)
        for d in _filter([d for d, _ in keep], only, only_batch):
            if len(out) >= limit:
                break
            d.update(status=r.ST_PREPROCESS_INPROGRESS, claimed_by=worker, claimed_at=now,
                     modified_ts=now, modified_at=stamp)
            if self._put_versioned(d, vers[id(d)]):  # lost races simply drop out
                out.append(d)
        if out:  # this process just wrote claimed_by: the mapping names it now
            self._kw_miss.pop("claimed_by", None)
        return out

    def all(self):
        body = {"query": {"match_all": {}}, "size": 10000}
        resp = self.http.post(f"{self.base}/{self.index}/{self.doc_type}/_search", content=json.dumps(body),
                              headers={"Content-Type": "application/json"})
        if resp.status_code == 404:
            return []
        resp.raise_for_status()
        return [h["_source"] for h in resp.json().get("hits", {}).get("hits", [])]

    # engine records live in their own index so the reference service's
    # ``documents`` searches never see them
    def _meta_url(self, key: str) -> str:
        return f"{self.base}/{META_INDEX}/{self.doc_type}/{key}"

    def put_meta(self, key, value):
        resp = self.http.put(self._meta_url(key), params={"refresh": self.refresh},
                             content=json.dumps({"value": value}), headers={"Content-Type": "application/json"})
        resp.raise_for_status()

    def get_meta(self, key):
        resp = self.http.get(self._meta_url(key))
        if resp.status_code == 404:
            return None
        resp.raise_for_status()
        body = resp.json()
        return body["_source"].get("value") if body.get("found", False) else None

    def close(self):
        self.http.close()
