"""Continuous jobs on the streaming engine: leased by strategy, one range
query per metric family, resident history, per-tick verdicts."""

import asyncio
import json

import httpx
import torch

from foremast_amd.brain.streaming import StreamingMonitor, is_continuous
from foremast_amd.promql import synth
from foremast_amd.promql.client import PromClient
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.service import app as svc
from foremast_amd.store import MemoryJobStore
from foremast_amd.utils.config import BrainConfig, reference_default_env
from foremast_amd.utils.metrics import BrainMetrics

T0 = 1_700_000_000.0
M = "namespace_app_per_pod:http_server_requests_error_5xx"


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def _job(app, strategy="continuous", end=T0 + 1800):
    from foremast_amd.utils.timeutil import format_rfc3339
    q = f'{M}{{namespace="ns",app="{app}"}}'
    params = {"endpoint": "http://prometheus:9090/api/v1/", "query": q, "step": 60}
    return {"appName": app, "startTime": format_rfc3339(T0), "endTime": format_rfc3339(end), "strategy": strategy,
            "metrics": {"current": {"error5xx": {"dataSourceType": "prometheus",
                                                 "parameters": dict(params, start=int(T0), end=int(end))}},
                        "historical": {"error5xx": {"dataSourceType": "prometheus",
                                                    "parameters": dict(params, start=int(T0 - 2 * 86400),
                                                                       end=int(T0))}}}}


import pytest


@pytest.mark.parametrize("where,algorithm", [
    ("cpu", "moving_average_all"),
    pytest.param("cuda", "moving_average_all", marks=pytest.mark.gpu),
    pytest.param("cuda", "holt_winters", marks=pytest.mark.gpu),
])
def test_streaming_monitor_continuous_jobs(where, algorithm):
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    for i, app in enumerate(("a", "b", "c")):
        gen = synth.error_rate(base=0.3 + 0.1 * i, spread=0.05, seed=i)
        if app == "b":
            gen = synth.step_change(gen, at=T0 + 120, factor=0.0, add=40.0)
        prom.add(M, {"namespace": "ns", "app": app}, gen)
    store = MemoryJobStore()
    ids = {app: svc.register(store, _job(app))[1]["jobId"] for app in ("a", "b", "c")}
    oneshot = svc.register(store, _job("a", strategy="rollingupdate"))[1]["jobId"]
    env = reference_default_env()
    env.update(MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", threshold0="4",  # bounded noise reaches 2 sigma
               ML_ALGORITHM=algorithm)
    cfg = BrainConfig.from_env(env)
    metrics = BrainMetrics()
    mon = StreamingMonitor(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                           device=torch.device(where), metrics=metrics, ring_len=2880, window=5, clock=clock)

    async def go():
        assert mon.sync() == 3                       # only the continuous jobs
        assert store.get(oneshot)["status"] == "initial"
        w = await mon.tick()
        assert set(w.values()) == {"preprocess_inprogress"} and len(mon.keys) == 3
        n_queries = len(prom.queries)
        clock.t = T0 + 300
        w = await mon.tick()
        assert len(prom.queries) == n_queries + 1    # one query for the whole metric family
        assert w[ids["b"]] == "completed_unhealth" and w[ids["a"]] == "preprocess_inprogress"
        doc = store.get(ids["b"])
        info = json.loads(doc["anomalyInfo"])
        assert info["error5xx"]["values"][1] > 30
        clock.t = T0 + 1900                          # past endTime
        w = await mon.tick()                         # rebuild without b's series, then finish
        assert len(mon.keys) == 2
        assert w[ids["a"]] == "completed_health" and w[ids["c"]] == "completed_health"

    asyncio.run(go())
    text = metrics.registry and __import__("prometheus_client").generate_latest(metrics.registry).decode()
    assert "foremastbrain:namespace_app_per_pod:http_server_requests_error_5xx_upper" in text
    assert is_continuous({"strategy": "Continuous"})
