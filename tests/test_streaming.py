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
        assert set(w.values()) == {"preprocess_inprogress"} and mon.n_live == 3
        # 2 days of history + window in <= 1-day chunks: 3 queries, one app group
        assert mon.history_queries == 3
        n_queries = len(prom.queries)
        clock.t = T0 + 300
        w = await mon.tick()
        assert len(prom.queries) == n_queries + 1    # one query for the whole metric family
        assert w[ids["b"]] == "completed_unhealth" and w[ids["a"]] == "preprocess_inprogress"
        doc = store.get(ids["b"])
        info = json.loads(doc["anomalyInfo"])
        assert info["error5xx"]["values"][1] > 30
        clock.t = T0 + 1900                          # past endTime
        w = await mon.tick()                         # b's row freed in place (no rebuild), then finish
        assert mon.n_live == 2 and mon.history_queries == 3
        assert w[ids["a"]] == "completed_health" and w[ids["c"]] == "completed_health"

    asyncio.run(go())
    text = metrics.registry and __import__("prometheus_client").generate_latest(metrics.registry).decode()
    assert "foremastbrain:namespace_app_per_pod:http_server_requests_error_5xx_upper" in text
    assert is_continuous({"strategy": "Continuous"})


def test_streaming_monitor_resumes_from_snapshot(tmp_path):
    """A restarted monitor adopts its snapshot (no week-long history refetch)
    and scores exactly like the monitor that kept running."""
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    for i, app in enumerate(("a", "b")):
        prom.add(M, {"namespace": "ns", "app": app}, synth.error_rate(base=0.3 + 0.1 * i, spread=0.05, seed=i))
    store = MemoryJobStore()
    for app in ("a", "b"):
        svc.register(store, _job(app))
    cfg = BrainConfig.from_env(dict(reference_default_env(), MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", threshold0="8"))
    transport = httpx.ASGITransport(app=prom.asgi_app())
    snap = str(tmp_path / "stream.safetensors")

    def monitor(worker):
        return StreamingMonitor(store, cfg, prom=PromClient(transport=transport), device=torch.device("cpu"),
                                worker_id=worker, ring_len=2880, window=5, clock=clock)

    async def go():
        m1 = monitor("w1")
        m1.sync()
        await m1.tick()
        clock.t = T0 + 120
        await m1.tick()
        assert m1.save_snapshot(snap)
        m2 = monitor("w1")          # restart of the same worker: re-leases its jobs
        m2.jobs = dict(m1.jobs)
        n_q = len(prom.queries)
        assert m2.restore_snapshot(snap)
        clock.t = T0 + 240
        await m1.tick()
        await m2.tick()
        assert len(prom.queries) == n_q + 2      # one incremental query each, no history rebuild
        for k in ("verdict", "std", "upper", "lower", "score"):
            torch.testing.assert_close(m1.shard.out[k], m2.shard.out[k], rtol=0, atol=0, equal_nan=True,
                                       msg=k)  # free rows are NaN in both
        m3 = monitor("w1")
        m3.jobs = dict(list(m1.jobs.items())[:1])
        assert not m3.restore_snapshot(snap)      # different series set: load rows from Prometheus instead
        clock.t = T0 + 2 * 86400
        m4 = monitor("w1")
        m4.jobs = dict(m1.jobs)
        assert not m4.restore_snapshot(snap)      # too old

    asyncio.run(go())


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [True, False])
def test_graph_tick_matches_eager(overlap):
    """tick_graph (ingest + rank tests + HW fit as one HIP-graph replay, ring state
    read from device memory) gives the same outputs as the eager calls, tick for
    tick, through the ring wrap, the window slot cycle and eager ticks in between
    (the device tick record resyncs); with the rank tests on a side stream beside the
    fit (the default from OVERLAP_MIN_SERIES series) and before it on the main stream."""
    from foremast_amd.brain.engine import ShardSpec, StreamingShard, synthetic_history
    from foremast_amd.ingest.ringbuffer import RingState
    from foremast_amd.ops import _native
    from foremast_amd.utils.config import BrainConfig
    _native.require()
    dev = torch.device("cuda:0")
    n, R, m, P, W = 64, 2880, 1440, 3, 6
    cfg = BrainConfig()
    cfg.min_historical_points = 0
    shards = []
    hist = synthetic_history(n, R + 40, m, dev, seed=3)
    for _ in range(2):
        sh = StreamingShard(ShardSpec(n_series=n, ring_len=R, season=m, pods=P, window=W, n_apps=8), cfg, dev,
                            app_id=(torch.arange(n, device=dev) % 8).int())
        sh.overlap_pairwise = overlap
        sh.load_history(hist[:, :R])
        # start near the end of the ring so the head wraps during the run (same data in both)
        sh.hist.state = RingState(head=R - 12, length=R)
        sh.set_baseline(hist[:, R - W:R].repeat(1, P).float())
        shards.append(sh)
    eager, graph = shards
    newv = torch.empty((n, P), device=dev)
    replays = 0
    for k in range(30):
        newv.copy_(hist[:, R + k:R + k + 1].repeat(1, P).float() * (1.0 + 0.3 * (k % 7 == 3)))
        eager.ingest_tick(newv)
        oe = {key: v.clone() for key, v in eager.score().items()}
        se = eager.app_stats.clone()
        replays += graph._graph is not None
        if k in (17, 18):  # eager ticks in between: the device tick record must resync
            graph.ingest_tick(newv)
            og = graph.score()
        else:
            og = graph.tick_graph(newv)
        torch.cuda.synchronize()
        for key in ("verdict", "sigma", "level", "trend", "best", "forecast", "count"):
            assert torch.equal(oe[key], og[key]), (k, key)
        assert torch.equal(se, graph.app_stats), k
        assert eager.hist.head == graph.hist.head and eager.cur.ticks == graph.cur.ticks
    assert graph._graph is not None and replays >= 20
    assert torch.equal(eager.hist.data, graph.hist.data) and torch.equal(eager.cur.data, graph.cur.data)


@pytest.mark.gpu
def test_overlapped_rank_tests_match_inline_detection():
    """Rank tests on a side stream concurrently with the Holt-Winters fit, band and
    verdict from the deferred-detection kernel: identical to the fused epilogue
    (pairwise-scaled thresholds, verdicts, app counters, K9 anomaly list)."""
    from foremast_amd.brain.engine import ShardSpec, StreamingShard, synthetic_history
    from foremast_amd.ops import _native
    from foremast_amd.utils.config import BrainConfig
    _native.require()
    dev = torch.device("cuda:0")
    n, R, m, P, W = 96, 4320, 1440, 5, 10
    cfg = BrainConfig()
    cfg.min_historical_points = 0
    hist = synthetic_history(n, R + 30, m, dev, seed=9)
    shards = []
    for overlap in (False, True):
        sh = StreamingShard(ShardSpec(n_series=n, ring_len=R, season=m, pods=P, window=W, n_apps=12), cfg, dev,
                            app_id=(torch.arange(n, device=dev) % 12).int(),
                            threshold=torch.full((n,), 3.0, device=dev))
        sh.overlap_pairwise = overlap
        sh.load_history(hist[:, :R])
        sh.set_baseline(hist[:, R - W:R].repeat(1, P))
        sh.enable_anomaly_list(4096)
        shards.append(sh)
    g = torch.Generator(device=dev).manual_seed(1)
    for k in range(W + 4):
        newv = hist[:, R + k:R + k + 1].repeat(1, P) + torch.randn(n, P, device=dev, generator=g)
        newv[::7] *= 2.5  # a shifted canary on some series: pairwise tests fire, thresholds drop
        outs = []
        for sh in shards:
            sh.ingest_tick(newv.contiguous())
            outs.append({key: v.clone() for key, v in sh.score().items() if torch.is_tensor(v)})
        torch.cuda.synchronize()
        for key in ("verdict", "count", "score", "forecast", "upper", "lower", "sigma", "level", "best"):
            assert torch.equal(outs[0][key], outs[1][key]), (k, key)
        assert torch.equal(shards[0].app_stats, shards[1].app_stats)
        assert torch.equal(shards[0].pw_out["differs"], shards[1].pw_out["differs"])
        a0 = sorted(zip(*[x.tolist() for x in shards[0].anomalies.fetch()[:2]]))
        a1 = sorted(zip(*[x.tolist() for x in shards[1].anomalies.fetch()[:2]]))
        assert a0 == a1
    from foremast_amd.ops import kernels as K
    assert K.last_detect_deferred and int(shards[1].pw_out["differs"].sum()) > 0


def test_streaming_rows_grow_incrementally_with_chunked_history():
    """New jobs join a running shard without a rebuild: only their series'
    history is fetched (1-day x 2-app chunks, regex app selectors), the shard
    grows by doubling, rows of live series keep their state, and the result
    equals a monitor that loaded everything at once."""
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    apps = ["a", "b.v2", "c", "d", "e"]
    for i, app in enumerate(apps):
        prom.add(M, {"namespace": "ns", "app": app}, synth.error_rate(base=0.3 + 0.05 * i, spread=0.05, seed=i))
    prom.add(M, {"namespace": "ns", "app": "bXv2"}, synth.error_rate(base=9.0, spread=0.05, seed=99))  # regex decoy
    store = MemoryJobStore()
    ids = {app: svc.register(store, _job(app))[1]["jobId"] for app in apps}
    cfg = BrainConfig.from_env(dict(reference_default_env(), MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10"))
    transport = httpx.ASGITransport(app=prom.asgi_app())

    def monitor(worker, owns=None):
        return StreamingMonitor(store, cfg, prom=PromClient(transport=transport), device=torch.device("cpu"),
                                worker_id=worker, ring_len=2880, window=5, clock=clock, min_capacity=2,
                                apps_per_query=2, owns=owns)

    first = {ids["a"], ids["b.v2"]}

    async def go():
        inc = monitor("inc", owns=lambda d: d["id"] in first)
        assert inc.sync() == 2
        await inc.tick()
        assert inc.shard.spec.n_series == 2 and inc.history_queries == 3   # 1 app group x 3 day chunks
        inc.owns = None
        assert inc.sync() == 3
        clock.t = T0 + 60
        await inc.tick()
        assert inc.shard.spec.n_series == 8 and inc.n_live == 5
        assert inc.history_queries == 3 + 2 * 3                            # only the 3 new series: 2 groups
        assert inc.roster_version == 2 and len(inc.apps) == 5
        # a fresh monitor over the same jobs, everything loaded at once
        for jid in ids.values():
            store.update(jid, {"claimed_by": "", "status": "reprogress"})
        ref = monitor("ref")
        assert ref.sync() == 5
        await ref.tick()
        for key, row in inc.rows.items():
            r2 = ref.rows[key]
            assert torch.equal(inc.shard.hist.logical()[row], ref.shard.hist.logical()[r2]), key
            assert torch.equal(inc.shard.out["verdict"][row], ref.shard.out["verdict"][r2])
            torch.testing.assert_close(inc.shard.out["upper"][row], ref.shard.out["upper"][r2], rtol=0, atol=0)
        # the decoy app never leaks into b.v2's row
        row = inc.rows[[k for k in inc.rows if k[3] == "b.v2"][0]]
        assert float(inc.shard.hist.logical()[row].nanmean()) < 5.0

    asyncio.run(go())


def test_streaming_failed_fetches_are_retried_not_nan_filled():
    """a failed history load keeps its series pending (reloaded next
    tick); a failed tick query leaves the ring where it was (the next tick
    refetches those minutes) instead of ingesting NaN."""
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    prom.add(M, {"namespace": "ns", "app": "a"}, synth.error_rate(base=0.3, spread=0.05, seed=1))
    store = MemoryJobStore()
    svc.register(store, _job("a"))
    env = reference_default_env()
    env.update(MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", ML_ALGORITHM="moving_average_all")
    mon = StreamingMonitor(store, BrainConfig.from_env(env),
                           prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                           device=torch.device("cpu"), ring_len=480, window=5, clock=clock)

    async def go():
        mon.sync()
        prom.faults.error_rate = 1.0
        await mon.tick()
        assert mon.pending, "a failed history load must stay pending"
        prom.faults.error_rate = 0.0
        clock.t = T0 + 60
        await mon.tick()
        assert not mon.pending
        hist = mon.shard.hist.logical()[0]
        assert torch.isnan(hist).float().mean() < 0.05          # the week arrived on the retry
        t_before = mon.t_last
        prom.faults.error_rate = 1.0
        clock.t = T0 + 180
        await mon.tick()
        assert mon.t_last == t_before                            # ring not advanced over the outage
        prom.faults.error_rate = 0.0
        clock.t = T0 + 240
        await mon.tick()
        assert mon.t_last == (T0 + 240) // 60 * 60
        newest = mon.shard.hist.logical()[0][-8:]                # graduated window points, no NaN hole
        assert not torch.isnan(newest).any(), newest
    asyncio.run(go())
