"""One-shot canary / rollingUpdate jobs on the resident engine (brain/rollout.py):
the exact barrelman queries (controller/queries.py = metricsquery.go), resident
history, baseline fetched once, per-tick pod windows, fail-fast verdicts, and
the same verdicts as the per-job BrainWorker on the same data."""

import asyncio
import json

import httpx
import numpy as np
import pytest
import torch

from foremast_amd.api import crd
from foremast_amd.api import rest as r
from foremast_amd.brain.batch import BatchScorer
from foremast_amd.brain.rollout import RolloutMonitor, is_rollout_keyable, plan_rollout
from foremast_amd.brain.worker import BrainWorker
from foremast_amd.controller import queries
from foremast_amd.promql import synth
from foremast_amd.promql.client import PromClient
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.service import app as svc
from foremast_amd.store import MemoryJobStore
from foremast_amd.utils.config import BrainConfig, reference_default_env
from foremast_amd.utils.metrics import BrainMetrics
from foremast_amd.utils.timeutil import format_rfc3339

T0 = 1_700_000_040.0  # aligned to the minute
NS = "ns"
METRICS = (("http_server_requests_error_5xx", "error5xx"), ("http_server_requests_latency", "latency"))


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def request(app, new_pods, old_pods, strategy, now=T0, metrics=METRICS):
    mets = crd.Metrics(data_source_type="prometheus", endpoint="http://prometheus:9090/api/v1/",
                       monitoring=[crd.Monitoring(metric_name=m, metric_alias=a) for m, a in metrics])
    info = queries.create_metrics_info(NS, app, [list(new_pods), list(old_pods)], mets, 10, strategy, now=now)
    return r.ApplicationHealthAnalyzeRequest(app_name=app, start_time=format_rfc3339(now),
                                             end_time=format_rfc3339(now + 600), metrics=info,
                                             strategy=strategy).to_dict()


def world(spike_app="a", spike_at=T0 + 120, metrics=METRICS):
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    apps = {"a": "canary", "b": "rollingUpdate", "c": "canary"}
    pods = {}
    for i, app in enumerate(apps):
        new, old = [f"{app}-v2-{k}" for k in range(2)], [f"{app}-v1-{k}" for k in range(3)]
        pods[app] = (new, old)
        for j, (m, _a) in enumerate(metrics):
            base = 0.3 + 0.1 * i + j
            prom.add("namespace_app_per_pod:" + m, {"namespace": NS, "app": app},
                     synth.error_rate(base=base, spread=0.05, seed=10 * i + j))
            for k, pod in enumerate(new + old):
                gen = synth.error_rate(base=base, spread=0.05, seed=100 + 10 * i + k + 50 * j)
                if app == spike_app and pod in new and j == 0:
                    gen = synth.step_change(gen, at=spike_at, factor=0.0, add=40.0)
                prom.add("namespace_pod:" + m, {"namespace": NS, "pod": pod}, gen)
    store = MemoryJobStore()
    ids = {app: svc.register(store, request(app, *pods[app], strategy))[1]["jobId"] for app, strategy in apps.items()}
    return clock, prom, store, ids


def config(algorithm="moving_average_all"):
    env = reference_default_env()
    env.update(MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", threshold0="4", threshold1="4", ML_ALGORITHM=algorithm)
    return BrainConfig.from_env(env)


def monitor(store, prom, clock, device, cfg, **kw):
    return RolloutMonitor(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                          device=torch.device(device), metrics=kw.pop("metrics", BrainMetrics()), window=10, pods=5,
                          clock=clock, ring_len=2880, min_capacity=4, **kw)


def test_plan_matches_barrelman_queries():
    clock, prom, store, ids = world()
    doc = store.get(ids["a"])
    p = plan_rollout(doc, config())
    assert p is not None and p.app == (NS, "a") and [s.alias for s in p.series] == ["error5xx", "latency"]
    s = p.series[0]
    assert s.hkey == ("http://prometheus:9090/api/v1/", "namespace_app_per_pod:http_server_requests_error_5xx",
                      NS, "a")
    assert s.fam == ("http://prometheus:9090/api/v1/", "namespace_pod:http_server_requests_error_5xx")
    assert s.cur_pods == ("a-v2-0", "a-v2-1") and s.base_pods == ("a-v1-0", "a-v1-1", "a-v1-2")
    assert s.cur_start == T0 + 60 and s.cur_n == 11 and s.hist_end == T0
    assert s.base_start == T0 - 600 and s.base_n == 11
    b = plan_rollout(store.get(ids["b"]), config())
    assert b is not None and b.series[0].base_pods == ()           # rollingUpdate: no baseline
    # not keyable: continuous, a wavefront source; multi-metric algorithms are (joint models,
    # tests/test_rollout_joint.py)
    assert not is_rollout_keyable(dict(doc, strategy="continuous", id="x1"), config())
    assert not is_rollout_keyable(dict(doc, id="x2", currentMetricStore="error5xx== wavefront"), config())
    assert is_rollout_keyable(doc, config("lstm")) and is_rollout_keyable(doc, config("auto"))


def _run(device, algorithm):
    clock, prom, store, ids = world()
    cfg = config(algorithm)
    metrics = BrainMetrics()
    mon = monitor(store, prom, clock, device, cfg, metrics=metrics)
    out = {}

    async def go():
        assert mon.sync() == 3
        w = await mon.tick()
        assert w == {} and len(mon.jobs) == 3 and mon.n_live == 6
        hq = mon.history.history_queries
        assert hq > 0
        for k, t in enumerate((T0 + 120, T0 + 300)):
            clock.t = t
            w = await mon.tick()
            out[t] = dict(w)
        assert mon.history.history_queries == hq          # resident: never refetched
        clock.t = T0 + 660
        out["end"] = dict(await mon.tick())
        assert not mon.jobs and mon.n_live == 0
    asyncio.run(go())
    docs = {app: store.get(j) for app, j in ids.items()}
    return out, docs, ids, metrics


@pytest.mark.parametrize("device,algorithm", [
    ("cpu", "moving_average_all"), ("cpu", "holt_winters"), ("cpu", "exponential_smoothing"),
    pytest.param("cuda", "moving_average_all", marks=pytest.mark.gpu),
    pytest.param("cuda", "holt_winters", marks=pytest.mark.gpu),
    pytest.param("cuda", "exponential_smoothing", marks=pytest.mark.gpu),
])
def test_rollout_monitor_canary_and_rolling_update(device, algorithm):
    out, docs, ids, metrics = _run(device, algorithm)
    # the spike starts at T0+120: the tick that ingests that minute fails the canary job of app a
    assert out[T0 + 120] == {ids["a"]: r.ST_COMPLETED_UNHEALTH}, out
    info = json.loads(docs["a"]["anomalyInfo"])
    assert set(info) == {"error5xx"}
    vals = info["error5xx"]["values"]
    assert vals[1] > 30 and vals[0] >= T0 + 120
    assert set(info["error5xx"]["tags"].split(",")) <= {"a-v2-0", "a-v2-1"}
    assert out["end"] == {ids["b"]: r.ST_COMPLETED_HEALTH, ids["c"]: r.ST_COMPLETED_HEALTH}
    assert docs["b"]["claimed_by"] == "" and "resident engine" in docs["b"]["processingContent"]
    text = metrics.render().decode()
    assert 'foremastbrain:namespace_app_per_pod:http_server_requests_error_5xx_upper{app="a",namespace="ns"}' in text


def test_rollout_monitor_matches_brain_worker_verdicts():
    """Same jobs, same data: the resident engine and the per-job worker agree."""
    out, docs, ids, _ = _run("cpu", "moving_average_all")
    clock, prom, store, ids2 = world()
    cfg = config("moving_average_all")
    worker = BrainWorker(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                         scorer=BatchScorer(cfg, device=torch.device("cpu")), worker_id="w", clock=clock)

    async def go():
        for t in (T0 + 120, T0 + 300, T0 + 660):
            clock.t = t
            await worker.cycle()
    asyncio.run(go())
    for app in ids:
        assert store.get(ids2[app])["status"] == docs[app]["status"], app
    wa = json.loads(store.get(ids2["a"])["anomalyInfo"])["error5xx"]["values"]
    ra = json.loads(docs["a"]["anomalyInfo"])["error5xx"]["values"]
    assert set(zip(wa[0::2], wa[1::2])) >= set(zip(ra[0::2], ra[1::2]))


def test_rollout_monitor_unknown_without_current_data():
    clock, prom, store, ids = world()
    prom.series = [s for s in prom.series if "v2" not in s.labels.get("pod", "")]  # new pods never report
    mon = monitor(store, prom, clock, "cpu", config())

    async def go():
        mon.sync()
        await mon.tick()
        clock.t = T0 + 660
        return await mon.tick()
    w = asyncio.run(go())
    assert set(w.values()) == {r.ST_COMPLETED_UNKNOWN}
    assert store.get(ids["a"])["reason"] == "no current metric data"


def test_rollout_release_and_failed_fetch_retry():
    """Re-sharding hands leases back; a failed window fetch is retried (no NaN hole)."""
    clock, prom, store, ids = world(spike_at=T0 + 60)
    mon = monitor(store, prom, clock, "cpu", config())

    async def go():
        mon.sync()
        await mon.tick()
        prom.faults.error_rate = 1.0          # Prometheus down for this tick
        clock.t = T0 + 120
        assert await mon.tick() == {}
        prom.faults.error_rate = 0.0
        clock.t = T0 + 180                     # both missed minutes arrive now
        w = await mon.tick()
        assert w.get(ids["a"]) == r.ST_COMPLETED_UNHEALTH
        vals = json.loads(store.get(ids["a"])["anomalyInfo"])["error5xx"]["values"]
        assert T0 + 120 in vals[0::2]         # the minute fetched late is scored
        n = mon.release(lambda d: d["appName"] == "b")
        assert n == 1 and store.get(ids["b"])["status"] == r.ST_REPROGRESS and ids["b"] not in mon.jobs
    asyncio.run(go())


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_node_brain_serves_rollout_jobs(device):
    """Canary jobs through the production node brain (streaming + rollout
    monitors on one rank): the GPU run writes the same verdicts and anomalous
    points as the CPU reference run, and the node health table names the app."""
    from foremast_amd.brain.node import NodeBrain
    from foremast_amd.brain.streaming import StreamingMonitor

    def run(dev):
        clock, prom, store, ids = world()
        cfg = config("holt_winters")
        client = PromClient(transport=httpx.ASGITransport(app=prom.asgi_app()))
        stream = StreamingMonitor(store, cfg, prom=client, device=torch.device(dev), ring_len=2880, window=10,
                                  clock=clock)
        roll = monitor(store, prom, clock, dev, cfg)
        node = NodeBrain(stream, None, store, torch.device(dev), extra=(roll,))
        tables = []

        async def go():
            for t in (T0, T0 + 60, T0 + 120, T0 + 180, T0 + 660):
                clock.t = t
                tables.append(await node.tick())
        asyncio.run(go())
        return {app: store.get(j) for app, j in ids.items()}, tables, node

    docs, tables, node = run(device)
    assert tables[2]["anomalous_apps"] == ["ns/a"] and tables[1]["anomalous_apps"] == []
    assert store_status(docs) == {"a": r.ST_COMPLETED_UNHEALTH, "b": r.ST_COMPLETED_HEALTH,
                                  "c": r.ST_COMPLETED_HEALTH}
    if device != "cpu":
        ref, _, _ = run("cpu")
        assert store_status(ref) == store_status(docs)
        got = json.loads(docs["a"]["anomalyInfo"])["error5xx"]["values"]
        want = json.loads(ref["a"]["anomalyInfo"])["error5xx"]["values"]
        assert got[0::2] == want[0::2]
        np.testing.assert_allclose(got[1::2], want[1::2], rtol=1e-6)


def store_status(docs):
    return {app: d["status"] for app, d in docs.items()}


def test_pod_slots_next_fit_and_refcounts():
    """Pod slots: shared pods are reference counted, a released pod's key is retired,
    and new pods take the free slots after the cursor in order (a tick's pods sit in
    slot order, so the decode's block writes walk forwards), wrapping and growing."""
    from foremast_amd.brain.rollout import PodSlots
    ps = PodSlots(cap=8)
    h = np.arange(1, 100, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    a = ps.acquire(h[:6])
    assert a.tolist() == list(range(6))
    assert ps.acquire(h[[2, 3]]).tolist() == [2, 3]          # shared: same slots, two references
    ps.release(h[:4])                                          # 0, 1 free; 2, 3 still referenced
    assert ps.slot_of(h[:4]).tolist() == [-1, -1, 2, 3] and len(ps) == 4
    assert ps.acquire(h[6:9]).tolist() == [6, 7, 0]            # after the cursor, then wrap
    assert ps.acquire(h[9:13]).tolist() == [8, 9, 10, 11]      # grown: the fresh half, in order
    assert ps.cap == 16 and len(ps) == 11
    ps.release(h[[2, 3, 4, 5, 6]])
    ps.release(h[[2, 3]])
    assert ps.slot_of(h[[2, 3, 4]]).tolist() == [-1, -1, -1]
    assert ps.acquire(h[20:25]).tolist() == [12, 13, 14, 15, 1]  # after the cursor, then wrap


class _FlakyStore:
    """Wraps a job store; ``fail`` names methods that raise until cleared."""

    def __init__(self, inner):
        self.inner, self.fail = inner, set()

    def __getattr__(self, name):
        f = getattr(self.inner, name)
        if name in self.fail:
            def boom(*a, **k):
                raise ConnectionError(f"store down ({name})")
            return boom
        return f


def test_node_keeps_ticking_when_the_store_fails_during_intake():
    """a store error inside the intake half (the endTime writes) is
    logged, the node keeps ticking, and the settled endTime verdicts are written by a
    later intake once the store is back (nothing is lost)."""
    from foremast_amd.brain.node import NodeBrain
    from foremast_amd.brain.streaming import StreamingMonitor
    clock, prom, raw, ids = world(spike_app=None)
    store = _FlakyStore(raw)
    cfg = config()
    stream = StreamingMonitor(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                              device=torch.device("cpu"), ring_len=2880, window=10, clock=clock)
    roll = monitor(store, prom, clock, "cpu", cfg)
    node = NodeBrain(stream, None, store, torch.device("cpu"), publish=False, extra=(roll,))

    async def go():
        for t in (T0, T0 + 60, T0 + 120):
            clock.t = t
            await node.tick()
        assert len(roll.jobs) == 3
        store.fail = {"update_many", "update"}
        for t in (T0 + 660, T0 + 720):          # every job past endTime; its writes fail
            clock.t = t
            await node.tick()
        assert {raw.get(j)["status"] for j in ids.values()} == {r.ST_PREPROCESS_INPROGRESS}
        assert len(roll.jobs) == 3 and roll._ending   # kept: written when the store is back
        store.fail = set()
        clock.t = T0 + 780
        await node.tick()
    asyncio.run(go())
    assert {app: raw.get(j)["status"] for app, j in ids.items()} == {
        "a": r.ST_COMPLETED_HEALTH, "b": r.ST_COMPLETED_HEALTH, "c": r.ST_COMPLETED_HEALTH}
    assert not roll.jobs and roll.n_live == 0


def test_retired_plan_holds_no_rows():
    """a finished job's memoised plan keeps no rows or pod
    references, so a later claim of the same job id cannot free another job's."""
    out, docs, ids, _ = _run("cpu", "moving_average_all")
    from foremast_amd.brain import plans as pl
    got = [p for p in pl._PLANS.values() if p is not None and p.doc_id in set(ids.values())]
    assert len(got) == 3
    for p in got:
        assert len(p.rows) == 0 and len(p.pod_keys) == 0 and p.jslot == -1
