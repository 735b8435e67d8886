"""App-side metrics instrumentation (the Python counterpart of the reference's
Spring Boot starter, ``foremast-spring-boot-k8s-metrics-starter``).

Foremast's recording rules read ``http_server_requests_seconds_{count,sum}``
with ``status`` and a per-app ``app`` tag.  :class:`ForemastMetrics` is an
ASGI middleware that records exactly that (Micrometer's naming), with the
starter's behaviour:

* common tags from ``"app:ENV.APP_NAME|info.app.name"``-style pairs —
  value from the environment variable, else the fallback
  (``K8sMetricsProperties.commonTagNameValuePairs``);
* zero-valued series pre-registered for statuses ``403,404,501,502`` so
  error-rate queries see 0 instead of no data before the first error
  (``initializeForStatuses``);
* a ``caller`` tag from the ``X-CALLER`` header (``CallerWebMvcTagsProvider``);
* exposition at ``/actuator/prometheus`` (Spring path) and ``/metrics``;
* optional ``whitelist``/``blacklist`` of metric name prefixes
  (``CommonMetricsFilter``).
"""

from __future__ import annotations

import os
import time
from typing import Dict, Iterable, Optional

import threading

from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, generate_latest
from prometheus_client.core import GaugeMetricFamily, SummaryMetricFamily

LABELS = ("app", "method", "uri", "status", "exception", "caller")


def parse_common_tags(spec: str, env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """``"app:ENV.APP_NAME|fallback,team:ENV.TEAM"`` → ``{"app": ..., "team": ...}``."""
    env = os.environ if env is None else env
    out: Dict[str, str] = {}
    for pair in filter(None, (p.strip() for p in spec.split(","))):
        name, _, src = pair.partition(":")
        value = ""
        for alt in src.split("|"):
            alt = alt.strip()
            if alt.startswith("ENV."):
                value = env.get(alt[4:], "")
            else:
                value = alt
            if value:
                break
        out[name.strip()] = value
    return out


class ForemastMetrics:
    def __init__(self, app, app_name: Optional[str] = None, registry: Optional[CollectorRegistry] = None,
                 common_tags: str = "app:ENV.APP_NAME|info.app.name",
                 initialize_for_statuses: Iterable[int] = (403, 404, 501, 502),
                 caller_header: str = "X-CALLER", paths=("/actuator/prometheus", "/metrics")) -> None:
        self.app = app
        self.registry = registry or CollectorRegistry()
        tags = parse_common_tags(common_tags)
        if app_name:
            tags["app"] = app_name
        self.app_name = tags.get("app") or "unknown"
        self.caller_header = caller_header.lower().encode()
        self.paths = set(paths)
        # Micrometer timer exposition: http_server_requests_seconds_{count,sum} + _max
        self._stats: Dict[tuple, list] = {}
        self._lock = threading.Lock()
        for st in initialize_for_statuses:
            self._stats[(self.app_name, "GET", "/**", str(st), "None", "UNKNOWN")] = [0, 0.0, 0.0]
        self.registry.register(self)

    def collect(self):
        summ = SummaryMetricFamily("http_server_requests_seconds", "HTTP server request timer", labels=LABELS)
        mx = GaugeMetricFamily("http_server_requests_seconds_max", "Max HTTP server request seconds", labels=LABELS)
        with self._lock:
            items = [(k, list(v)) for k, v in self._stats.items()]
        for k, (n, tot, m) in items:
            summ.add_metric(list(k), count_value=n, sum_value=tot)
            mx.add_metric(list(k), m)
        yield summ
        yield mx

    def observe(self, method: str, uri: str, status: int, seconds: float, exception: str = "None",
                caller: str = "UNKNOWN") -> None:
        k = (self.app_name, method, uri, str(status), exception, caller)
        with self._lock:
            st = self._stats.setdefault(k, [0, 0.0, 0.0])
            st[0] += 1
            st[1] += seconds
            st[2] = max(st[2], seconds)

    def count_of(self, status: int) -> int:
        with self._lock:
            return sum(v[0] for k, v in self._stats.items() if k[3] == str(status))

    def exposition(self) -> bytes:
        return generate_latest(self.registry)

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        path = scope.get("path", "")
        if path in self.paths:
            body = self.exposition()
            await send({"type": "http.response.start", "status": 200,
                        "headers": [(b"content-type", CONTENT_TYPE_LATEST.encode())]})
            await send({"type": "http.response.body", "body": body})
            return
        caller = "UNKNOWN"
        for k, v in scope.get("headers", []):
            if k == self.caller_header:
                caller = v.decode().strip() or "UNKNOWN"
        status = {"code": 500}

        async def send_wrapper(msg):
            if msg["type"] == "http.response.start":
                status["code"] = msg["status"]
            await send(msg)

        t0 = time.perf_counter()
        exc = "None"
        try:
            await self.app(scope, receive, send_wrapper)
        except Exception as e:
            exc = type(e).__name__
            raise
        finally:
            route = scope.get("route")
            uri = getattr(route, "path", None) or ("/**" if status["code"] == 404 else path)
            self.observe(scope.get("method", "GET"), uri, status["code"], time.perf_counter() - t0, exc, caller)
