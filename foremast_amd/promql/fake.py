"""Fake Prometheus: ``/api/v1/query_range`` over synthetic series.

Series are registered with labels and a generator ``f(ts: np.ndarray) ->
np.ndarray`` (NaN = no sample).  ``query_range`` answers in the exact
Prometheus matrix JSON shape (``[[ts, "value"], ...]``), so the brain's
fetch/parse path and the service's query proxy run unchanged against it.

Fault-injection hooks: gaps (``drop``), NaN/``"NaN"`` values,
late data (samples newer than ``now - lag`` are withheld) and HTTP errors.
"""

from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np
from fastapi import FastAPI, Query
from fastapi.responses import JSONResponse

from .selector import parse_selector

Gen = Callable[[np.ndarray], np.ndarray]


@dataclass
class FakeSeries:
    labels: Dict[str, str]
    gen: Gen


@dataclass
class Faults:
    lag_seconds: float = 0.0
    error_rate: float = 0.0
    drop_prob: float = 0.0
    seed: int = 0


class FakePrometheus:
    def __init__(self, clock: Callable[[], float] = time.time) -> None:
        self.series: List[FakeSeries] = []
        self.clock = clock
        self.faults = Faults()
        self.queries: List[str] = []
        self._rng = np.random.default_rng(0)

    def add(self, name: str, labels: Dict[str, str], gen: Gen) -> FakeSeries:
        lab = dict(labels)
        lab["__name__"] = name
        s = FakeSeries(labels=lab, gen=gen)
        self.series.append(s)
        return s

    def remove(self, name: str, **labels) -> None:
        self.series = [s for s in self.series if not (s.labels.get("__name__") == name and
                                                      all(s.labels.get(k) == v for k, v in labels.items()))]

    def query_range(self, query: str, start: float, end: float, step: float) -> Dict:
        self.queries.append(query)
        if self.faults.error_rate and self._rng.random() < self.faults.error_rate:
            return {"status": "error", "errorType": "internal", "error": "injected failure"}
        sel = parse_selector(query)
        if step <= 0:
            return {"status": "error", "errorType": "bad_data", "error": "zero or negative step"}
        n = int(math.floor((end - start) / step)) + 1 if end >= start else 0
        ts = start + step * np.arange(max(n, 0))
        horizon = self.clock() - self.faults.lag_seconds
        ts = ts[ts <= horizon]
        result = []
        for s in self.series:
            if not sel.matches(s.labels):
                continue
            vals = np.asarray(s.gen(ts), dtype=np.float64) if len(ts) else np.zeros(0)
            keep = ~np.isnan(vals)
            if self.faults.drop_prob:
                keep &= self._rng.random(len(vals)) >= self.faults.drop_prob
            pts = [[float(t) if not float(t).is_integer() else int(t), _fmt(v)]
                   for t, v in zip(ts[keep], vals[keep])]
            if pts:
                result.append({"metric": dict(s.labels), "values": pts})
        return {"status": "success", "data": {"resultType": "matrix", "result": result}}

    def asgi_app(self):
        app = FastAPI(title="fake-prometheus")

        @app.get("/api/v1/query_range")
        async def qr(query: str = Query(...), start: float = Query(...), end: float = Query(...),
                     step: float = Query(...)):
            body = self.query_range(query, start, end, step)
            return JSONResponse(status_code=200 if body["status"] == "success" else 400, content=body)

        return app


def _fmt(v: float) -> str:
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    return repr(float(v)) if not float(v).is_integer() else str(int(v))
