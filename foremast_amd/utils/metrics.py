"""Prometheus exposition for the brain (``:8000/metrics``).

UI-compatible model-band series (``foremast-browser/src/config/metrics.js``):
for every monitored recorded metric ``M`` (e.g.
``namespace_app_per_pod:http_server_requests_error_5xx``) the gauges
``foremastbrain:M_upper``, ``foremastbrain:M_lower`` and
``foremastbrain:M_anomaly`` with labels ``{namespace, app}``; the
``_anomaly`` value is the (unix-seconds) timestamp of the latest anomalous
point (the UI multiplies it by 1000, ``App.js:235``).

Band values are not pushed into per-label gauge children on every tick (at
100k series that is 300k Python calls per tick): ``export_band`` only records
the latest values and the resident engines register *band sources* —
callables yielding ``(metric, namespace, app, upper, lower, anomaly_ts)``
from their last tick's host arrays — that a custom collector turns into
gauge families when Prometheus scrapes.

Engine metrics: ``foremast_series_scored_total``, ``foremast_jobs_total``,
``foremast_detect_latency_seconds`` (histogram → p50), ``foremast_tick_seconds``
and ``foremast_collective_seconds``.
"""

from __future__ import annotations

import re
import threading
from typing import Callable, Dict, Iterable, List, Optional, Tuple

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest
from prometheus_client.core import GaugeMetricFamily

_BAD = re.compile(r"[^a-zA-Z0-9_:]")

LAT_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0)


BandRow = Tuple[str, str, str, float, float, Optional[float]]  # metric, namespace, app, upper, lower, anomaly ts


class _BandCollector:
    """Scrape-time exposition of the model bands (``foremastbrain:<m>_{upper,lower,anomaly}``)."""

    def __init__(self, owner: "BrainMetrics") -> None:
        self.owner = owner

    def collect(self):
        fams: Dict[str, GaugeMetricFamily] = {}

        def fam(metric: str, suffix: str) -> GaugeMetricFamily:
            name = BrainMetrics.band_name(metric, suffix)
            g = fams.get(name)
            if g is None:
                g = fams[name] = GaugeMetricFamily(name, "foremast brain model band", labels=["namespace", "app"])
            return g
        for metric, ns, app, up, lo, an in self.owner.band_rows():
            fam(metric, "upper").add_metric([ns, app], up)
            fam(metric, "lower").add_metric([ns, app], lo)
            if an is not None:
                fam(metric, "anomaly").add_metric([ns, app], an)
        return list(fams.values())


class BrainMetrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None) -> None:
        self.registry = registry or CollectorRegistry()
        self._lock = threading.Lock()
        self._bands: Dict[Tuple[str, str, str], List] = {}
        self._sources: Dict[str, Callable[[], Iterable[BandRow]]] = {}
        r = self.registry
        self.series_scored = Counter("foremast_series_scored", "Metric series scored", registry=r)
        self.jobs = Counter("foremast_jobs", "Jobs finished by status", ["status"], registry=r)
        self.detect_latency = Histogram("foremast_detect_latency_seconds",
                                        "Claim-to-verdict latency per scoring cycle", buckets=LAT_BUCKETS,
                                        registry=r)
        self.tick = Histogram("foremast_tick_seconds", "GPU scoring tick duration", buckets=LAT_BUCKETS, registry=r)
        self.collective = Histogram("foremast_collective_seconds", "Health collective duration",
                                    buckets=LAT_BUCKETS, registry=r)
        r.register(_BandCollector(self))

    @staticmethod
    def band_name(metric: str, suffix: str) -> str:
        return "foremastbrain:" + _BAD.sub("_", metric) + "_" + suffix

    def export_band(self, metric: str, namespace: str, app: str, upper: float, lower: float,
                    anomaly_ts: Optional[float] = None) -> None:
        with self._lock:
            row = self._bands.get((metric, namespace, app))
            if row is None:
                self._bands[(metric, namespace, app)] = [upper, lower, anomaly_ts]
            else:
                row[0], row[1] = upper, lower
                if anomaly_ts is not None:
                    row[2] = anomaly_ts

    def add_band_source(self, name: str, source: Callable[[], Iterable[BandRow]]) -> None:
        """Register (or replace) a resident engine's band rows, read at scrape time."""
        with self._lock:
            self._sources[name] = source

    def band_rows(self) -> List[BandRow]:
        with self._lock:
            rows = {k: (v[0], v[1], v[2]) for k, v in self._bands.items()}
            sources = list(self._sources.values())
        for src in sources:
            for metric, ns, app, up, lo, an in src():
                prev = rows.get((metric, ns, app))
                rows[(metric, ns, app)] = (up, lo, an if an is not None else (prev[2] if prev else None))
        return [(k[0], k[1], k[2], v[0], v[1], v[2]) for k, v in rows.items()]

    def render(self) -> bytes:
        return generate_latest(self.registry)

    def serve(self, port: int = 8000, addr: str = "0.0.0.0"):
        from prometheus_client import start_http_server
        return start_http_server(port, addr=addr, registry=self.registry)
