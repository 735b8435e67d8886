"""Analyst HTTP client (barrelman → foremast-service).

``foremast-barrelman/pkg/client/analyst/analystclient.go:63-238``:
``start_analyzing`` POSTs ``<endpoint>create`` and returns the job id;
``get_status`` GETs ``<endpoint>id/<jobId>`` and maps the external status to
a DeploymentMonitor phase.  The reference ``Interface`` omits the strategy
parameter (Q7); here the strategy is part of the signature.

A pluggable ``transport`` (``httpx`` transport, e.g. ``httpx.ASGITransport``)
lets the controller talk to an in-process service in tests.
"""

from __future__ import annotations

import json
import time
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import urljoin

import httpx

from ..api import crd
from ..api import rest as r
from ..api import status as st
from ..utils.timeutil import format_rfc3339
from . import queries


class AnalystError(RuntimeError):
    pass


class AnalystClient:
    def __init__(self, endpoint: str, transport: Any = None, timeout: float = 30.0,
                 user_agent: str = "foremast-barrelman") -> None:
        if endpoint and not endpoint.endswith("/"):
            endpoint = endpoint + "/"
        self.base = endpoint
        self.transport = transport
        self.timeout = timeout
        self.user_agent = user_agent

    def _client(self) -> httpx.AsyncClient:
        kw: Dict[str, Any] = {"timeout": self.timeout}
        if self.transport is not None:
            kw["transport"] = self.transport
        return httpx.AsyncClient(**kw)

    def build_request(self, namespace: str, app_name: str, pod_names: List[List[str]],
                      metrics: crd.Metrics, time_window_min: int, strategy: str,
                      now: Optional[float] = None) -> r.ApplicationHealthAnalyzeRequest:
        now = time.time() if now is None else now
        info = queries.create_metrics_info(namespace, app_name, pod_names, metrics,
                                           time_window_min, strategy, now)
        return r.ApplicationHealthAnalyzeRequest(
            app_name=app_name, start_time=format_rfc3339(now),
            end_time=format_rfc3339(now + time_window_min * 60), metrics=info, strategy=strategy)

    async def start_analyzing(self, namespace: str, app_name: str, pod_names: List[List[str]],
                              metrics: crd.Metrics, time_window_min: int, strategy: str,
                              now: Optional[float] = None) -> str:
        req = self.build_request(namespace, app_name, pod_names, metrics, time_window_min,
                                 strategy, now)
        url = urljoin(self.base, "create")
        async with self._client() as c:
            resp = await c.post(url, content=json.dumps(req.to_dict()),
                                headers={"Accept": "application/json",
                                         "Content-Type": "application/json",
                                         "User-Agent": self.user_agent})
        if resp.status_code != 200:
            raise AnalystError(f"{url} responded invalid server response:{resp.status_code}")
        body = resp.json()
        job_id = body.get("jobId", "")
        if not job_id:
            raise AnalystError(f"{url} responded invalid server response:{body.get('reason', '')}")
        return job_id

    async def get_status(self, job_id: str) -> Tuple[r.ApplicationHealthAnalyzeResponse, str]:
        """Returns (response, phase)."""
        url = urljoin(self.base, "id/" + job_id)
        try:
            async with self._client() as c:
                resp = await c.get(url, headers={"Accept": "application/json",
                                                 "User-Agent": self.user_agent})
        except httpx.HTTPError as e:
            raise AnalystError(f"GET {url}: {e}") from e
        try:
            body = resp.json()
        except ValueError as e:
            raise AnalystError(f"GET {url}: bad body") from e
        out = r.ApplicationHealthAnalyzeResponse.from_dict(body)
        return out, st.external_to_phase(out.status)
