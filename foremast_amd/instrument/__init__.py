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
* :class:`CommonMetricsFilter` — when enabled, every meter is hidden unless
  an explicit enable override, the whitelist or a name prefix admits it, and
  the blacklist hides; meters are toggled at run time through
  ``/actuator/k8s-metrics/{enable,disable}/<metric>`` (``CommonMetricsFilter``,
  ``K8sMetricsEndpoint``).
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


_UNIT_SUFFIXES = ("_seconds_max", "_seconds_count", "_seconds_sum", "_seconds", "_bytes", "_total", "_max",
                  "_count", "_sum")


def meter_name(name: str) -> str:
    """Micrometer meter name of a Prometheus family / meter name:
    ``http_server_requests_seconds`` → ``http.server.requests``."""
    for suf in _UNIT_SUFFIXES:
        if name.endswith(suf) and len(name) > len(suf):
            name = name[: -len(suf)]
            break
    return name.replace("_", ".")


def _split(spec) -> list:
    if not spec:
        return []
    if isinstance(spec, str):
        spec = spec.split(",")
    return [x.strip() for x in spec if x and x.strip()]


class CommonMetricsFilter:
    """The starter's meter filter (``CommonMetricsFilter.java:84-110``), applied to
    exposition.  Disabled → everything is shown.  Enabled → per meter, in order:
    an explicit enable override (``management.metrics.enable.<name>``: the
    longest dotted prefix in ``enable_overrides``, falling back to ``all``),
    the whitelist (shown), the blacklist (hidden), a name prefix (shown);
    anything else is hidden.  Names are compared in Micrometer's dotted form
    (``_`` → ``.``), prefixes against the dotted name as configured."""

    def __init__(self, enabled: bool = False, whitelist=None, blacklist=None, prefixes=None,
                 enable_overrides: Optional[Dict[str, bool]] = None) -> None:
        self.enabled = enabled
        self.whitelist = {meter_name(x) for x in _split(whitelist)}
        self.blacklist = {meter_name(x) for x in _split(blacklist)}
        self.prefixes = tuple(_split(prefixes))
        self.enable_overrides = dict(enable_overrides or {})
        self._lock = threading.Lock()

    @classmethod
    def from_env(cls, env: Optional[Dict[str, str]] = None) -> "CommonMetricsFilter":
        """``K8S_METRICS_ENABLE_COMMON_METRICS_FILTER`` / ``..._WHITELIST`` /
        ``..._BLACKLIST`` / ``..._PREFIX`` (the ``k8s.metrics.*`` properties)."""
        e = os.environ if env is None else env
        on = e.get("K8S_METRICS_ENABLE_COMMON_METRICS_FILTER", "false").strip().lower() in ("1", "true", "yes")
        return cls(on, e.get("K8S_METRICS_COMMON_METRICS_WHITELIST"), e.get("K8S_METRICS_COMMON_METRICS_BLACKLIST"),
                   e.get("K8S_METRICS_COMMON_METRICS_PREFIX"))

    def _override(self, name: str) -> Optional[bool]:
        if not self.enable_overrides:
            return None
        n = name
        while n:
            if n in self.enable_overrides:
                return self.enable_overrides[n]
            n = n.rpartition(".")[0]
        return self.enable_overrides.get("all")

    def accept(self, name: str) -> bool:
        if not self.enabled:
            return True
        m = meter_name(name)
        with self._lock:
            o = self._override(m)
            if o is not None:
                return o
            if m in self.whitelist:
                return True
            if m in self.blacklist:
                return False
            return any(m.startswith(p) for p in self.prefixes)

    def enable_metric(self, name: str) -> None:
        m = meter_name(name)
        with self._lock:
            self.blacklist.discard(m)
            self.whitelist.add(m)

    def disable_metric(self, name: str) -> None:
        m = meter_name(name)
        with self._lock:
            self.whitelist.discard(m)
            self.blacklist.add(m)


class _Filtered:
    def __init__(self, registry, flt: CommonMetricsFilter) -> None:
        self.registry, self.flt = registry, flt

    def collect(self):
        for fam in self.registry.collect():
            if self.flt.accept(fam.name):
                yield fam


class ForemastMetrics:
    def __init__(self, app, app_name: Optional[str] = None, registry: Optional[CollectorRegistry] = None,
                 common_tags: str = "app:ENV.APP_NAME|info.app.name",
                 initialize_for_statuses: Iterable[int] = (403, 404, 501, 502),
                 caller_header: str = "X-CALLER", paths=("/actuator/prometheus", "/metrics"),
                 metrics_filter: Optional[CommonMetricsFilter] = None,
                 actuator_prefix: str = "/actuator/k8s-metrics/") -> None:
        self.app = app
        self.registry = registry or CollectorRegistry()
        self.filter = metrics_filter if metrics_filter is not None else CommonMetricsFilter.from_env()
        self.actuator_prefix = actuator_prefix
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
        return generate_latest(_Filtered(self.registry, self.filter))

    def actuator(self, path: str) -> Optional[bytes]:
        """``/actuator/k8s-metrics/{enable,disable}/<metric>`` → ``OK``
        (``K8sMetricsEndpoint.java:21-34``); None if the path is not one."""
        if not path.startswith(self.actuator_prefix):
            return None
        action, _, metric = path[len(self.actuator_prefix):].partition("/")
        if metric:
            if action.lower() == "enable":
                self.filter.enable_metric(metric)
            elif action.lower() == "disable":
                self.filter.disable_metric(metric)
        return b"OK"

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        path = scope.get("path", "")
        act = self.actuator(path)
        if act is not None:
            await send({"type": "http.response.start", "status": 200,
                        "headers": [(b"content-type", b"text/plain; version=0.1.4; charset=utf-8")]})
            await send({"type": "http.response.body", "body": act})
            return
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
