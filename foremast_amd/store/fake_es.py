"""In-process fake of the Elasticsearch 6.x REST subset the job store uses
(WSGI app; mount with ``httpx.WSGITransport`` in tests, or serve it with any
WSGI server for local runs).

Supported: ``GET /``, ``GET|PUT /<index>/<type>/<id>`` (``?version=`` for
optimistic concurrency → 409 on mismatch), ``PUT .../<id>/_create`` (409 if
present), ``POST /<index>/<type>/_search`` with ``match_all`` or a
``bool.filter`` / ``bool.must_not`` of ``terms`` / ``term`` / ``range`` queries, ``size``, ``version`` and a single-key
``sort``.  Documents are versioned per id exactly like ES internal versions.

Two ES 6.x rules the real cluster enforces are modelled, so tests catch code that
only works against a lenient fake:

* one mapping type per index: a write under a second type is rejected with 400
  (``illegal_argument_exception``, "Rejecting mapping update ... more than 1 type");
* dynamic mapping of strings: a string field is analysed ``text`` (lower-cased,
  split on anything but letters, digits and ``_``) with an exact ``<field>.keyword``
  sub-field, so ``term`` / ``terms`` on the bare field match single tokens only.

An index created with explicit mappings (``PUT /<index>`` with ``{"mappings": {type:
{"properties": ...}}}``, as an operator might) keeps them: a field mapped ``keyword``
is matched exactly on its bare name and has no ``.keyword`` sub-field.
``GET /<index>/_mapping`` reports both kinds.
"""

from __future__ import annotations

import json
import re
import threading
from typing import Any, Dict, List, Tuple
from urllib.parse import parse_qs


class FakeElasticsearch:
    def __init__(self) -> None:
        self.docs: Dict[Tuple[str, str], Tuple[Dict[str, Any], int]] = {}
        self.types: Dict[str, str] = {}  # index -> its one mapping type
        self.explicit: Dict[str, Dict[str, Dict[str, Any]]] = {}  # index -> explicit field mappings
        self.lock = threading.Lock()
        self.requests: List[str] = []
        self.fail_next = 0  # fault injection: return 503 for the next N requests

    # ------------------------------------------------------------------ WSGI
    def __call__(self, environ, start_response):
        method = environ["REQUEST_METHOD"]
        path = environ.get("PATH_INFO", "/")
        qs = {k: v[-1] for k, v in parse_qs(environ.get("QUERY_STRING", "")).items()}
        n = int(environ.get("CONTENT_LENGTH") or 0)
        raw = environ["wsgi.input"].read(n) if n else b""
        self.requests.append(f"{method} {path}")
        if self.fail_next > 0:
            self.fail_next -= 1
            return self._reply(start_response, 503, {"error": "injected"})
        try:
            status, body = self.handle(method, path, qs, json.loads(raw) if raw else None)
        except (ValueError, KeyError) as e:
            status, body = 400, {"error": str(e)}
        return self._reply(start_response, status, body)

    @staticmethod
    def _reply(start_response, status, body):
        data = json.dumps(body).encode()
        reason = {200: "OK", 201: "Created", 400: "Bad Request", 404: "Not Found", 409: "Conflict",
                  503: "Service Unavailable"}.get(status, "")
        start_response(f"{status} {reason}", [("Content-Type", "application/json"),
                                              ("Content-Length", str(len(data)))])
        return [data]

    # ------------------------------------------------------------------ API
    def handle(self, method: str, path: str, qs: Dict[str, str], body: Any):
        parts = [p for p in path.split("/") if p]
        if not parts:
            return 200, {"version": {"number": "6.4.2"}, "tagline": "You Know, for Search"}
        if len(parts) == 1 and method == "PUT":
            return self._create_index(parts[0], body or {})
        if len(parts) == 2 and parts[1] == "_mapping" and method == "GET":
            return self._mapping(parts[0])
        if len(parts) == 3 and parts[2] == "_search" and method in ("GET", "POST"):
            return self._search(parts[0], body or {})
        if len(parts) == 4 and parts[3] == "_create" and method in ("PUT", "POST"):
            return self._put(parts[0], parts[2], body, create=True, version=None, typ=parts[1])
        if len(parts) == 3:
            idx, _typ, did = parts
            if method == "GET":
                with self.lock:
                    cur = self.docs.get((idx, did))
                if cur is None:
                    return 404, {"_index": idx, "_id": did, "found": False}
                return 200, {"_index": idx, "_type": _typ, "_id": did, "_version": cur[1], "found": True,
                             "_source": cur[0]}
            if method in ("PUT", "POST"):
                ver = int(qs["version"]) if "version" in qs else None
                return self._put(idx, did, body, create=False, version=ver, typ=_typ)
        return 400, {"error": f"unsupported {method} {path}"}

    def _create_index(self, idx: str, body: Dict[str, Any]):
        with self.lock:
            if idx in self.types:
                return 400, {"error": {"type": "resource_already_exists_exception"}}
            maps = body.get("mappings") or {}
            for typ, m in maps.items():
                self.types[idx] = typ
                self.explicit[idx] = dict((m or {}).get("properties") or {})
        return 200, {"acknowledged": True, "index": idx}

    def _mapping(self, idx: str):
        with self.lock:
            if idx not in self.types:
                return 404, {"error": {"type": "index_not_found_exception"}}
            props: Dict[str, Any] = {}
            for (i, _did), (d, _v) in self.docs.items():
                if i != idx:
                    continue
                for k, v in d.items():
                    if k in props:
                        continue
                    if isinstance(v, str):
                        props[k] = {"type": "text", "fields": {"keyword": {"type": "keyword", "ignore_above": 256}}}
                    elif isinstance(v, bool):
                        props[k] = {"type": "boolean"}
                    elif isinstance(v, (int, float)):
                        props[k] = {"type": "float" if isinstance(v, float) else "long"}
            props.update(self.explicit.get(idx, {}))
            return 200, {idx: {"mappings": {self.types[idx]: {"properties": props}}}}

    def _put(self, idx: str, did: str, doc: Any, create: bool, version, typ: str):
        with self.lock:
            if self.types.setdefault(idx, typ) != typ:
                return 400, {"error": {"type": "illegal_argument_exception",
                                       "reason": f"Rejecting mapping update to [{idx}] as the final mapping "
                                                 f"would have more than 1 type: [{self.types[idx]}, {typ}]"}}
            cur = self.docs.get((idx, did))
            if create and cur is not None:
                return 409, {"error": {"type": "version_conflict_engine_exception"}}
            if version is not None and (cur is None or cur[1] != version):
                return 409, {"error": {"type": "version_conflict_engine_exception"}}
            ver = 1 if cur is None else cur[1] + 1
            self.docs[(idx, did)] = (json.loads(json.dumps(doc)), ver)
        return (201 if ver == 1 else 200), {"_index": idx, "_id": did, "_version": ver,
                                            "result": "created" if ver == 1 else "updated"}

    def _search(self, idx: str, body: Dict[str, Any]):
        with self.lock:
            items = [(did, d, v) for (i, did), (d, v) in self.docs.items() if i == idx]
        if idx not in self.types:
            return 404, {"error": {"type": "index_not_found_exception"}}
        explicit = self.explicit.get(idx, {})
        q = body.get("query", {"match_all": {}})
        b = q.get("bool", {})

        def hit(doc, f) -> bool:
            if "terms" in f:
                (key, vals), = f["terms"].items()
                return any(_matches(doc, key, v, explicit) for v in vals)
            if "term" in f:
                (key, val), = f["term"].items()
                return _matches(doc, key, val, explicit)
            if "range" in f:
                (key, ops), = f["range"].items()
                v = doc.get(key, 0)
                return all({"lt": v < x, "lte": v <= x, "gt": v > x, "gte": v >= x}[op] for op, x in ops.items())
            return True
        items = [x for x in items if all(hit(x[1], f) for f in b.get("filter", []))
                 and not any(hit(x[1], f) for f in b.get("must_not", []))]
        for s in body.get("sort", []):
            (key, spec), = s.items()
            items.sort(key=lambda x: x[1].get(key, 0), reverse=spec.get("order") == "desc")
        start = int(body.get("from", 0))
        items = items[start:start + int(body.get("size", 10))]
        hits = []
        for did, d, v in items:
            h = {"_index": idx, "_id": did, "_source": json.loads(json.dumps(d))}
            if body.get("version"):
                h["_version"] = v
            hits.append(h)
        return 200, {"hits": {"total": len(hits), "hits": hits}}


_TOKEN = re.compile(r"[0-9A-Za-z_]+")


def _matches(doc: Dict[str, Any], key: str, want: Any, explicit: Dict[str, Dict[str, Any]] = None) -> bool:
    """ES term-level match under dynamic mapping: ``x.keyword`` is exact; a bare string
    field holds analysed tokens (a term query is not analysed, so it must equal one).
    A field mapped ``keyword`` explicitly is exact on its bare name and has no
    ``.keyword`` sub-field."""
    explicit = explicit or {}
    if key.endswith(".keyword") and key[: -len(".keyword")] in explicit:
        return False  # no such sub-field: matches nothing, silently (as ES does)
    if explicit.get(key, {}).get("type") == "keyword":
        return doc.get(key) == want
    if key.endswith(".keyword"):
        v = doc.get(key[: -len(".keyword")])
        return isinstance(v, str) and v == want
    v = doc.get(key)
    if isinstance(v, str):
        return isinstance(want, str) and want in {t.lower() for t in _TOKEN.findall(v)}
    return v == want
