"""A Kubernetes API server facade over :class:`FakeCluster` (ASGI).

Serves the REST paths :class:`~foremast_amd.k8s.http.HttpKube` uses —
core ``/api/v1`` kinds, ``/apis/apps/v1`` and the Foremast CRD group — with
``Status`` error bodies, label selectors, JSON merge-patch and streaming
``?watch=true`` (newline-delimited events; ``resourceVersion`` older than the
cluster's compaction horizon answers 410 Gone).  Used to test the HTTP client
and the controller end to end with a real socket (run it under uvicorn).
"""

from __future__ import annotations

import asyncio
import json
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, StreamingResponse

from .api import ApiError, KIND_OF
from .fake import FakeCluster


def _status(e: ApiError) -> JSONResponse:
    return JSONResponse({"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": str(e),
                         "reason": e.reason, "code": e.code}, status_code=e.code)


def create_apiserver(cluster: FakeCluster, min_watch_rv: int = 0) -> FastAPI:
    app = FastAPI()
    state = {"min_rv": min_watch_rv}
    app.state.cluster = cluster
    app.state.watch_state = state

    def current_rv() -> str:
        rvs = [int(o["metadata"].get("resourceVersion", 0)) for o in cluster._objs.values()]
        return str(max(rvs + [0]))

    async def handle(request: Request, kind: str, namespace: Optional[str], name: Optional[str]):
        if kind not in KIND_OF:
            return JSONResponse({"kind": "Status", "code": 404, "reason": "NotFound",
                                 "message": f"unknown resource {kind}"}, status_code=404)
        try:
            m = request.method
            if name is None:
                if m == "GET" and request.query_params.get("watch") in ("true", "1"):
                    rv = int(request.query_params.get("resourceVersion") or 0)
                    if rv and rv < state["min_rv"]:
                        return JSONResponse({"kind": "Status", "code": 410, "reason": "Expired",
                                             "message": "too old resource version"}, status_code=410)
                    return StreamingResponse(_watch(kind, namespace, rv), media_type="application/json")
                if m == "GET":
                    items = cluster.list_sync(kind, namespace, request.query_params.get("labelSelector"),
                                              request.query_params.get("fieldSelector"))
                    return JSONResponse({"kind": KIND_OF[kind] + "List", "items": items,
                                         "metadata": {"resourceVersion": current_rv()}})
                if m == "POST":
                    body = await request.json()
                    if namespace:
                        body.setdefault("metadata", {}).setdefault("namespace", namespace)
                    return JSONResponse(cluster.create_sync(kind, body), status_code=201)
            else:
                if m == "GET":
                    return JSONResponse(cluster.get_sync(kind, namespace or "", name))
                if m == "PUT":
                    return JSONResponse(cluster.update_sync(kind, await request.json()))
                if m == "PATCH":
                    return JSONResponse(cluster.patch_sync(kind, namespace or "", name, await request.json()))
                if m == "DELETE":
                    cluster.delete_sync(kind, namespace or "", name)
                    return JSONResponse({"kind": "Status", "status": "Success"})
            return JSONResponse({"kind": "Status", "code": 405, "reason": "MethodNotAllowed"}, status_code=405)
        except ApiError as e:
            return _status(e)

    async def _watch(kind: str, namespace: Optional[str], rv: int):
        agen = cluster.watch(kind, namespace)
        try:
            async for ev in agen:
                o = ev["object"]
                if ev.get("initial"):
                    # replay: objects changed after the requested resourceVersion
                    if int(o["metadata"].get("resourceVersion", 0)) > rv:
                        yield (json.dumps({"type": "MODIFIED", "object": o}) + "\n").encode()
                    continue
                if int(o["metadata"].get("resourceVersion", 0)) <= rv and ev["type"] != "DELETED":
                    continue
                yield (json.dumps({"type": ev["type"], "object": o}) + "\n").encode()
                await asyncio.sleep(0)
        finally:
            await agen.aclose()

    for prefix in ("/api/v1", "/apis/apps/v1", "/apis/deployment.foremast.ai/v1alpha1"):
        methods = ["GET", "POST", "PUT", "PATCH", "DELETE"]

        async def ns_coll(request: Request, namespace: str, kind: str):
            return await handle(request, kind, namespace, None)

        async def ns_item(request: Request, namespace: str, kind: str, name: str):
            return await handle(request, kind, namespace, name)

        async def coll(request: Request, kind: str):
            return await handle(request, kind, None, None)

        async def item(request: Request, kind: str, name: str):
            return await handle(request, kind, None, name)

        app.add_api_route(prefix + "/namespaces/{namespace}/{kind}", ns_coll, methods=methods)
        app.add_api_route(prefix + "/namespaces/{namespace}/{kind}/{name}", ns_item, methods=methods)
        app.add_api_route(prefix + "/{kind}", coll, methods=methods)
        app.add_api_route(prefix + "/{kind}/{name}", item, methods=methods)
    return app
