"""Prometheus exposition for the brain (``:8000/metrics``).

UI-compatible model-band series (``foremast-browser/src/config/metrics.js``):
for every monitored recorded metric ``M`` (e.g.
``namespace_app_per_pod:http_server_requests_error_5xx``) the gauges
``foremastbrain:M_upper``, ``foremastbrain:M_lower`` and
``foremastbrain:M_anomaly`` with labels ``{namespace, app}``; the
``_anomaly`` value is the (unix-seconds) timestamp of the latest anomalous
point (the UI multiplies it by 1000, ``App.js:235``).

Engine metrics: ``foremast_series_scored_total``, ``foremast_jobs_total``,
``foremast_detect_latency_seconds`` (histogram → p50), ``foremast_tick_seconds``
and ``foremast_collective_seconds``.
"""

from __future__ import annotations

import re
import threading
from typing import Dict, Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

_BAD = re.compile(r"[^a-zA-Z0-9_:]")

LAT_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0)


class BrainMetrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None) -> None:
        self.registry = registry or CollectorRegistry()
        self._lock = threading.Lock()
        self._bands: Dict[str, Gauge] = {}
        r = self.registry
        self.series_scored = Counter("foremast_series_scored", "Metric series scored", registry=r)
        self.jobs = Counter("foremast_jobs", "Jobs finished by status", ["status"], registry=r)
        self.detect_latency = Histogram("foremast_detect_latency_seconds",
                                        "Claim-to-verdict latency per scoring cycle", buckets=LAT_BUCKETS,
                                        registry=r)
        self.tick = Histogram("foremast_tick_seconds", "GPU scoring tick duration", buckets=LAT_BUCKETS, registry=r)
        self.collective = Histogram("foremast_collective_seconds", "Health collective duration",
                                    buckets=LAT_BUCKETS, registry=r)

    def _gauge(self, name: str) -> Gauge:
        with self._lock:
            g = self._bands.get(name)
            if g is None:
                g = Gauge(name, "foremast brain model band", ["namespace", "app"], registry=self.registry)
                self._bands[name] = g
            return g

    @staticmethod
    def band_name(metric: str, suffix: str) -> str:
        return "foremastbrain:" + _BAD.sub("_", metric) + "_" + suffix

    def export_band(self, metric: str, namespace: str, app: str, upper: float, lower: float,
                    anomaly_ts: Optional[float] = None) -> None:
        self._gauge(self.band_name(metric, "upper")).labels(namespace=namespace, app=app).set(upper)
        self._gauge(self.band_name(metric, "lower")).labels(namespace=namespace, app=app).set(lower)
        if anomaly_ts is not None:
            self._gauge(self.band_name(metric, "anomaly")).labels(namespace=namespace, app=app).set(anomaly_ts)

    def render(self) -> bytes:
        return generate_latest(self.registry)

    def serve(self, port: int = 8000, addr: str = "0.0.0.0"):
        from prometheus_client import start_http_server
        return start_http_server(port, addr=addr, registry=self.registry)
