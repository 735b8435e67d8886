"""Multi-metric canary jobs on the resident engine (brain/rollout.py ``_fit_joint`` /
``_score_joint``): under ``ML_ALGORITHM`` bivariate_normal / auto a 2-metric job keeps
its per-metric rows (moving_average_all) and gets the joint bivariate normal of
``docs/guides/design.md:78``, fitted at admission on the resident history and scored
every tick on the pod-mean current values; the verdicts and anomaly payloads equal
the per-job BrainWorker's on the same data."""

import asyncio
import json

import httpx
import numpy as np
import pytest
import torch

from foremast_amd.api import crd
from foremast_amd.api import rest as r
from foremast_amd.brain import plans as pl
from foremast_amd.brain.batch import BatchScorer
from foremast_amd.brain.rollout import RolloutMonitor, is_rollout_keyable
from foremast_amd.brain.worker import BrainWorker
from foremast_amd.controller import queries
from foremast_amd.promql.client import PromClient
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.promql.synth import _hash_noise
from foremast_amd.service import app as svc
from foremast_amd.store import MemoryJobStore
from foremast_amd.utils.config import BrainConfig, reference_default_env
from foremast_amd.utils.metrics import BrainMetrics
from foremast_amd.utils.timeutil import format_rfc3339

T0 = 1_700_000_040.0
NS = "ns"
EP = "http://prometheus:9090/api/v1/"
M2 = (("http_server_requests_error_5xx", "error5xx"), ("http_server_requests_latency", "latency"))
M3 = M2 + (("http_server_requests_error_4xx", "error4xx"),)
BREAK_AT = T0 + 180


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def request(app, new, old, metrics, strategy="canary"):
    mets = crd.Metrics(data_source_type="prometheus", endpoint=EP,
                       monitoring=[crd.Monitoring(metric_name=m, metric_alias=a) for m, a in metrics])
    info = queries.create_metrics_info(NS, app, [list(new), list(old)], mets, 10, strategy, now=T0)
    return r.ApplicationHealthAnalyzeRequest(app_name=app, start_time=format_rfc3339(T0),
                                             end_time=format_rfc3339(T0 + 600), metrics=info,
                                             strategy=strategy).to_dict()


def correlated(seed, j, flip_after=None, pod_seed=0):
    """Metric j of an app: a shared latent load u(t) drives every metric (error rate
    10 + 3u, latency 20 + 6u, ...), with a little independent noise.  After
    ``flip_after`` the latency moves against the load (20 - 6u): each metric alone
    stays inside its usual range, the pair does not."""
    lvl, amp = (10.0, 3.0) if j == 0 else (20.0 + 5 * j, 6.0)

    def f(ts):
        ts = np.asarray(ts, dtype=np.float64)
        u = _hash_noise(ts, seed)
        v = lvl + amp * u + 0.05 * _hash_noise(ts, seed + 1000 * (j + 1) + pod_seed)
        if flip_after is not None and j == 1:
            v = np.where(ts >= flip_after, lvl - amp * u + 0.05 * _hash_noise(ts, seed + 77 + pod_seed), v)
        return v
    return f


def world():
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    apps = {"a": M2, "b": M2, "c": M2[:1], "d": M3}   # a: correlation breaks; b: healthy; c: 1 metric; d: 3
    store = MemoryJobStore()
    ids = {}
    for i, (app, mets) in enumerate(apps.items()):
        new, old = [f"{app}-v2-{k}" for k in range(2)], [f"{app}-v1-{k}" for k in range(3)]
        for j, (m, _a) in enumerate(mets):
            prom.add("namespace_app_per_pod:" + m, {"namespace": NS, "app": app}, correlated(10 * i, j))
            for k, pod in enumerate(new + old):
                brk = BREAK_AT if (app == "a" and pod in new) else None
                prom.add("namespace_pod:" + m, {"namespace": NS, "pod": pod}, correlated(10 * i, j, brk, pod_seed=k))
        ids[app] = svc.register(store, request(app, new, old, mets))[1]["jobId"]
    return clock, prom, store, ids


def config(algorithm):
    env = reference_default_env()
    env.update(MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", ML_ALGORITHM=algorithm, ML_PAIRWISE_ALGORITHM="none",
               threshold="4", threshold0="4", threshold1="4", threshold2="4")
    return BrainConfig.from_env(env)


def run_resident(device, algorithm):
    clock, prom, store, ids = world()
    cfg = config(algorithm)
    mon = RolloutMonitor(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                         device=torch.device(device), metrics=BrainMetrics(), window=10, pods=5, clock=clock,
                         ring_len=2880, min_capacity=4)

    async def go():
        mon.sync()
        await mon.tick()
        for t in (T0 + 120, T0 + 240, T0 + 360, T0 + 660):
            clock.t = t
            mon.sync()
            await mon.tick()
    asyncio.run(go())
    return {app: store.get(j) for app, j in ids.items()}, ids


def run_worker(algorithm, claim_all=True):
    clock, prom, store, ids = world()
    cfg = config(algorithm)
    w = BrainWorker(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                    scorer=BatchScorer(cfg, device=torch.device("cpu")), worker_id="w", clock=clock)

    async def go():
        for t in (T0 + 120, T0 + 240, T0 + 360, T0 + 660):
            clock.t = t
            await w.cycle()
    asyncio.run(go())
    return {app: store.get(j) for app, j in ids.items()}


def test_joint_dispatch_and_keyability():
    clock, prom, store, ids = world()
    assert pl.joint_kind("auto", 1) is None and pl.joint_kind("auto", 2) == "biv" and pl.joint_kind("auto", 3) == "lstm"
    assert pl.joint_kind("bivariate_normal", 3) == "biv" and pl.joint_kind("lstm", 2) == "lstm"
    for algo in ("auto", "bivariate_normal"):
        assert is_rollout_keyable(store.get(ids["a"]), config(algo))
        assert is_rollout_keyable(store.get(ids["c"]), config(algo))
    assert is_rollout_keyable(store.get(ids["d"]), config("bivariate_normal"))


@pytest.mark.parametrize("device,algorithm", [
    ("cpu", "auto"), ("cpu", "bivariate_normal"),
    pytest.param("cuda", "auto", marks=pytest.mark.gpu),
    pytest.param("cuda", "bivariate_normal", marks=pytest.mark.gpu),
])
def test_bivariate_rollout_matches_worker(device, algorithm):
    docs, ids = run_resident(device, algorithm)
    ref = run_worker(algorithm)
    # the broken correlation fails app a's canary; each metric alone stays in its band
    assert docs["a"]["status"] == r.ST_COMPLETED_UNHEALTH, docs["a"].get("reason")
    info = json.loads(docs["a"]["anomalyInfo"])
    assert set(info) == {"error5xx"} and info["error5xx"]["tags"] == ""
    assert min(info["error5xx"]["values"][0::2]) >= BREAK_AT
    for app in ("b", "c"):
        assert docs[app]["status"] == r.ST_COMPLETED_HEALTH, (app, docs[app].get("reason"))
    keyed = ("a", "b", "c", "d") if algorithm == "bivariate_normal" else ("a", "b", "c")
    for app in keyed:
        assert "resident engine" in docs[app]["processingContent"], app
        assert docs[app]["status"] == ref[app]["status"], app
        if docs[app].get("anomalyInfo"):
            got, want = json.loads(docs[app]["anomalyInfo"]), json.loads(ref[app]["anomalyInfo"])
            assert set(got) == set(want), app
            for alias in got:
                gv, wv = np.array(got[alias]["values"]), np.array(want[alias]["values"])
                # the worker scores at its own cycle times: the resident points are the ones it saw
                gp = dict(zip(gv[0::2].tolist(), gv[1::2].tolist()))
                wp = dict(zip(wv[0::2].tolist(), wv[1::2].tolist()))
                common = sorted(set(gp) & set(wp))
                assert common, (app, alias)
                np.testing.assert_allclose([gp[t] for t in common], [wp[t] for t in common], rtol=1e-5)
    # 3 metrics under auto: the joint LSTM's job (test_lstm_rollout_jobs_on_the_resident_lstm), still resident
    assert "resident engine" in docs["d"]["processingContent"]


def lstm_world(bad_app="d3"):
    """3-metric canary jobs on apps whose metrics move together; the new pods of
    ``bad_app`` triple every metric from the third minute on."""
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    store = MemoryJobStore()
    ids = {}
    from foremast_amd.promql import synth
    for i in range(4):
        app = f"d{i}"
        new, old = [f"{app}-v2-{k}" for k in range(2)], [f"{app}-v1-{k}" for k in range(3)]
        for j, (m, _a) in enumerate(M3):
            base = synth.seasonal(level=10.0 + i + 5 * j, amp=2.0, noise=0.2, seed=10 * i + j)
            prom.add("namespace_app_per_pod:" + m, {"namespace": NS, "app": app}, base)
            for k, pod in enumerate(new + old):
                g = synth.seasonal(level=10.0 + i + 5 * j, amp=2.0, noise=0.2, seed=10 * i + j + 100 * (k + 1))
                if app == bad_app and pod in new:
                    g = synth.step_change(g, at=T0 + 120, factor=3.0)
                prom.add("namespace_pod:" + m, {"namespace": NS, "pod": pod}, g)
        ids[app] = svc.register(store, request(app, new, old, M3))[1]["jobId"]
    return clock, prom, store, ids


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_lstm_rollout_jobs_on_the_resident_lstm(device, monkeypatch):
    """ML_ALGORITHM=auto, 3-metric canary jobs: keyed by the resident engine (none reach
    BrainWorker); per-metric rows cannot fire (threshold 1000), the joint LSTM over the
    three metrics — the node's resident LSTM engine fed with the canary pods' mean —
    fails the degraded rollout and names every metric."""
    monkeypatch.setenv("FOREMAST_LSTM_PRETRAIN", "40")
    monkeypatch.setenv("FOREMAST_LSTM_PRETRAIN_PER_TICK", "40")
    clock, prom, store, ids = lstm_world()
    env = reference_default_env()
    env.update(MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", ML_ALGORITHM="auto", ML_PAIRWISE_ALGORITHM="none",
               threshold="1000", threshold0="1000", threshold1="1000", threshold2="1000", ML_LSTM_THRESHOLD="4",
               FOREMAST_LSTM_WINDOW="8", FOREMAST_LSTM_HIDDEN="16")
    cfg = BrainConfig.from_env(env)
    assert all(is_rollout_keyable(store.get(j), cfg) for j in ids.values())
    mon = RolloutMonitor(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                         device=torch.device(device), metrics=BrainMetrics(), window=10, pods=5, clock=clock,
                         ring_len=2880, min_capacity=4)
    assert mon.joint_lstm is not None
    written = {}

    async def go():
        for k in range(12):
            clock.t = T0 + 60 * k
            mon.sync()
            written.update(await mon.tick())
    asyncio.run(go())
    assert written.get(ids["d3"]) == r.ST_COMPLETED_UNHEALTH, written
    info = json.loads(store.get(ids["d3"])["anomalyInfo"])
    assert set(info) == {a for _m, a in M3}
    assert all(written.get(ids[a]) == r.ST_COMPLETED_HEALTH for a in ("d0", "d1", "d2")), written
    assert not mon.jobs and not mon.joint_lstm.jobs
