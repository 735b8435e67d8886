"""foremast-service: the ``/v1/healthcheck`` job API and the query proxy.

Routes and behaviour follow ``foremast-service/cmd/manager/main.go:130-276``:

* ``POST /v1/healthcheck/create`` — validate, flatten the metric queries to
  ``alias== url`` config strings, create (or find) the content-addressed job
  document, answer ``{"jobId","statusCode":200,"status":"new"}``;
* ``GET /v1/healthcheck/id/{id}`` — status lookup with the internal→external
  status map; returns the ``anomaly`` map (fix of Q2);
* ``GET /api/v1/{queryproxy}`` — CORS proxy to
  ``QUERY_SERVICE_ENDPOINT + "api/v1/query_range?" + rawQuery``; the body is
  returned **as a JSON string** (double encoded) because the reference UI
  ``JSON.parse``s it (``foremast-browser/src/App.js:282``; Q1).  ``?raw=1``
  returns the Prometheus JSON unwrapped.

Extensions (not in the reference): ``GET /healthz`` and
``GET /v1/healthcheck/cluster`` (the node-level health table aggregated over
the GPU ranks: rank 0 of the node brain publishes it into the job store,
``brain/node.py``).
"""

from __future__ import annotations

import html
import json
import logging
import os
from typing import Any, Callable, Dict, Optional

import httpx
from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse, JSONResponse, PlainTextResponse

from ..api import rest as r
from ..api import status as st
from ..store import JobStore, open_store
from ..utils.timeutil import TimeFormatError
from . import urls

log = logging.getLogger("foremast.service")

DEFAULT_QUERY_ENDPOINT = "http://prometheus-k8s.monitoring.svc.cluster.local:9090/"


def _err(code: int, msg: str):
    return JSONResponse(status_code=code, content={"error": msg})


def anomaly_from_doc(doc: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    raw = doc.get("anomalyInfo")
    if not raw:
        return None
    if isinstance(raw, dict):
        return raw
    try:
        val = json.loads(raw)
    except (TypeError, ValueError):
        return None
    return val if isinstance(val, dict) and val else None


def status_response(doc: Dict[str, Any]) -> Dict[str, Any]:
    """``ConvertESToResp`` + anomaly (``converter.go:48-61``)."""
    try:
        code = int(doc.get("statusCode") or "")
    except ValueError:
        code = 200
    anomaly = anomaly_from_doc(doc)
    resp = r.ApplicationHealthAnalyzeResponse(
        job_id=doc.get("id", ""), status_code=code,
        status=st.internal_to_external(doc.get("status", "")),
        reason=doc.get("reason", "") or "",
        anomaly=None)
    d = resp.to_dict()
    if anomaly:
        d["anomaly"] = {k: {"tags": v.get("tags", ""), "values": [r._num(x) for x in v.get("values", [])]}
                        for k, v in sorted(anomaly.items())}
    return d


def register(store: JobStore, body: Any) -> tuple[int, Dict[str, Any]]:
    """The create handler as a pure function → (http status, json body)."""
    if not isinstance(body, dict):
        return 400, {"error": "Bad request"}
    try:
        req = r.ApplicationHealthAnalyzeRequest.from_dict(body)
    except Exception:  # shape errors → gin's BindJSON failure
        return 400, {"error": "Bad request"}
    if not isinstance(req.app_name, str) or not req.app_name.strip():
        return 400, {"error": "appName is empty"}
    code, reason, configs, sources = urls.flatten_metrics_info(req.metrics)
    if code != 0:
        return 400, {"error": reason}
    doc = r.DocumentRequest(
        app_name=req.app_name, start_time=req.start_time or "", end_time=req.end_time or "",
        current_config=configs[0], baseline_config=configs[1], historical_config=configs[2],
        current_metric_store=sources[0], baseline_metric_store=sources[1],
        historical_metric_store=sources[2], status_code="200", strategy=req.strategy or "")
    try:
        job_id = store.create(doc)
    except TimeFormatError as e:
        return 400, {"error": f"bad time: {e}"}
    return 200, r.ApplicationHealthAnalyzeResponseNew(
        job_id=job_id, status_code=200, status=st.EXT_NEW).to_dict()


def lookup(store: JobStore, job_id: str) -> Dict[str, Any]:
    doc = store.get(job_id)
    if doc is None:
        return r.ApplicationHealthAnalyzeResponseNew(
            job_id=job_id, status_code=200, status=st.EXT_UNKNOWN,
            reason=job_id + " not found.").to_dict()
    return status_response(doc)


def create_app(store: Optional[JobStore] = None, query_endpoint: Optional[str] = None,
               cluster_health: Optional[Callable[[], Dict[str, Any]]] = None,
               proxy_transport: Any = None):
    """Build the FastAPI application.

    ``proxy_transport`` lets tests route the proxy to an in-process ASGI app.
    """
    if store is None:
        store = open_store(os.environ.get("FOREMAST_JOB_STORE") or os.environ.get("ELASTIC_URL"))
    qe = query_endpoint or os.environ.get("QUERY_SERVICE_ENDPOINT") or DEFAULT_QUERY_ENDPOINT
    app = FastAPI(title="foremast-service", version="v1")
    app.state.store = store
    app.state.query_endpoint = qe

    @app.post("/v1/healthcheck/create")
    async def create(request: Request):
        try:
            body = await request.json()
        except Exception:
            return _err(400, "Bad request")
        code, resp = register(store, body)
        return JSONResponse(status_code=code, content=resp)

    @app.get("/v1/healthcheck/id/{job_id}")
    async def by_id(job_id: str):
        return JSONResponse(content=lookup(store, job_id))

    @app.get("/v1/healthcheck/cluster")
    async def cluster():
        if cluster_health is not None:
            return JSONResponse(content=cluster_health())
        table = None
        try:
            table = store.get_meta("cluster_health")  # published by the node brain's rank 0
        except Exception as e:  # noqa: BLE001 - store down: report "no table"
            log.warning("cluster health lookup failed: %s", e)
        return JSONResponse(content=table or {"ranks": 0, "apps": {}})

    @app.get("/healthz")
    async def healthz():
        return PlainTextResponse("ok")

    @app.get("/ui/{namespace}/{app_name}")
    async def dashboard(namespace: str, app_name: str):
        from . import ui
        return HTMLResponse(ui.page(namespace, app_name))

    @app.get("/ui")
    async def dashboard_index():
        apps = sorted({d.get("appName", "") for d in store.all() if d.get("appName")})
        items = "".join(f"<li>{html.escape(a)}</li>" for a in apps)
        return HTMLResponse("<!doctype html><title>Foremast</title><h1>Foremast jobs</h1>"
                            "<p>open <code>/ui/&lt;namespace&gt;/&lt;app&gt;</code></p><ul>" + items + "</ul>")

    @app.get("/api/v1/{queryproxy}")
    async def query_proxy(queryproxy: str, request: Request):
        raw_q = request.url.query
        want_raw = False
        if raw_q.endswith("&raw=1") or raw_q == "raw=1":
            want_raw = True
            raw_q = raw_q[: -len("raw=1")].rstrip("&")
        target = app.state.query_endpoint + "api/v1/query_range?" + raw_q
        headers = {"Access-Control-Allow-Origin": "*"}
        try:
            kw = {"timeout": 90.0}
            if proxy_transport is not None:
                kw["transport"] = proxy_transport
            async with httpx.AsyncClient(**kw) as client:
                resp = await client.get(target)
            body = resp.text
        except Exception:
            return JSONResponse(status_code=400, headers=headers,
                                content={"error": "invoke query " + target + " failed "})
        if want_raw:
            try:
                return JSONResponse(content=json.loads(body), headers=headers)
            except ValueError:
                return PlainTextResponse(body, headers=headers)
        return JSONResponse(content=body, headers=headers)

    return app
