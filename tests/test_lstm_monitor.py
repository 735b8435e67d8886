"""Continuous multi-metric jobs on the resident DP LSTM-AE engine
(brain/lstm_monitor.py): resident history, per-tick append, one data-parallel
step per tick, calibration of joining entities, fail-fast verdicts."""

import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import httpx
import pytest
import torch

from foremast_amd.brain.lstm_monitor import LstmMonitor, lstm_features
from foremast_amd.brain.streaming import StreamingMonitor
from foremast_amd.promql import synth
from foremast_amd.promql.client import PromClient
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.service import app as svc
from foremast_amd.store import MemoryJobStore
from foremast_amd.utils.config import BrainConfig, reference_default_env
from foremast_amd.utils.timeutil import format_rfc3339

T0 = 1_700_000_040.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METRICS = (("namespace_app_per_pod:http_server_requests_latency", "latency"),
           ("namespace_app_per_pod:http_server_requests_error_5xx", "error5xx"))


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def job(app, endpoint="http://prometheus:9090/api/v1/", now=T0, end=T0 + 3600):
    cur, hist = {}, {}
    for m, alias in METRICS:
        q = f'{m}{{namespace="ns",app="{app}"}}'
        p = {"endpoint": endpoint, "query": q, "step": 60}
        cur[alias] = {"dataSourceType": "prometheus", "parameters": dict(p, start=int(now), end=int(end))}
        hist[alias] = {"dataSourceType": "prometheus", "parameters": dict(p, start=int(now - 86400), end=int(now))}
    return {"appName": app, "startTime": format_rfc3339(now), "endTime": format_rfc3339(end),
            "strategy": "continuous", "metrics": {"current": cur, "historical": hist}}


def add_series(prom, apps, bad=None, at=None):
    for i, app in enumerate(apps):
        for j, (m, _a) in enumerate(METRICS):
            gen = synth.seasonal(level=10.0 + i + 5 * j, amp=2.0, noise=0.2, seed=10 * i + j)
            if app == bad:
                gen = synth.step_change(gen, at=at, factor=3.0)
            prom.add(m, {"namespace": "ns", "app": app}, gen)


def config():
    env = reference_default_env()
    env.update(ML_ALGORITHM="lstm", ML_LSTM_THRESHOLD="4")
    return BrainConfig.from_env(env)


def test_lstm_features_selection():
    cfg = config()
    store = MemoryJobStore()
    d = store.get(svc.register(store, job("a"))[1]["jobId"])
    feats = lstm_features(d, cfg)
    assert [a for a, _ in feats] == ["error5xx", "latency"] and feats[0][1][3] == "a"
    env = reference_default_env()
    env.update(ML_ALGORITHM="auto")
    assert lstm_features(d, BrainConfig.from_env(env)) is None          # auto: 3+ metrics
    assert lstm_features(dict(d, strategy="canary"), cfg) is None


def test_lstm_monitor_flags_degraded_app_cpu():
    clock = Clock(T0)
    prom = FakePrometheus(clock=clock)
    apps = [f"app{i}" for i in range(6)]
    add_series(prom, apps, bad="app2", at=T0 + 5 * 60)
    store = MemoryJobStore()
    ids = {a: svc.register(store, job(a))[1]["jobId"] for a in apps}
    cfg = config()
    client = PromClient(transport=httpx.ASGITransport(app=prom.asgi_app()))
    mon = LstmMonitor(store, cfg, prom=client, device=torch.device("cpu"), ring_len=2880, window=16, hidden=16,
                      min_capacity=4, clock=clock)
    stream = StreamingMonitor(store, cfg, prom=client, device=torch.device("cpu"), ring_len=480, window=5,
                              clock=clock)
    stream.exclude = mon.is_mine

    async def go():
        assert stream.sync() == 0                         # the LSTM engine's jobs, not the streaming one's
        assert mon.sync() == 6
        written = {}
        for k in range(12):
            clock.t = T0 + 60 * k
            written.update(await mon.tick())
        return written
    written = asyncio.run(go())
    assert mon.shard.trainer.steps >= mon.pretrain_steps and mon.shard.cal is not None
    assert written.get(ids["app2"]) == "completed_unhealth", written
    info = json.loads(store.get(ids["app2"])["anomalyInfo"])
    assert set(info) == {"latency", "error5xx"} and info["latency"]["tags"] == "lstm"
    assert all(written.get(ids[a]) is None for a in apps if a != "app2")
    assert mon.shard.n >= 6 and len(mon.jobs) == 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _serve(app, port):
    import uvicorn
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    for _ in range(100):
        if server.started:
            return server
        time.sleep(0.05)
    raise RuntimeError("fake prometheus did not start")


def _node(tmp_path, nproc, extra_env, apps, bad):
    from foremast_amd.store.jobstore import SqliteJobStore
    prom = FakePrometheus()
    now = time.time()
    add_series(prom, apps, bad=bad, at=now + 5)
    port = _free_port()
    server = _serve(prom.asgi_app(), port)
    db = str(tmp_path / "jobs.db")
    store = SqliteJobStore(db)
    ids = {a: svc.register(store, job(a, f"http://127.0.0.1:{port}/api/v1/", now=now, end=now + 3600))[1]["jobId"]
           for a in apps}
    env = dict(os.environ, FOREMAST_RING_LEN="2880", FOREMAST_HEARTBEAT_S="5", OMP_NUM_THREADS="1",
               ML_ALGORITHM="lstm", ML_LSTM_THRESHOLD="4", FOREMAST_LSTM_WINDOW="16", FOREMAST_LSTM_HIDDEN="16",
               FOREMAST_LSTM_PRETRAIN="20", FOREMAST_PUBLISH_EVERY_S="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "foremast_amd.brain", "--streaming", "--nproc", str(nproc), "--store",
           f"sqlite://{db}", "--metrics-port", "0", "--tick-seconds", "1", "--window", "5"]
    log_path = tmp_path / "node.log"
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=open(log_path, "w"), stderr=subprocess.STDOUT,
                            start_new_session=True)
    return store, ids, proc, server, log_path


def _stop(proc, server):
    os.killpg(proc.pid, signal.SIGTERM)
    try:
        proc.wait(timeout=30)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
    server.should_exit = True


@pytest.mark.slow
def test_lstm_node_two_ranks_dp_replicas_identical(tmp_path):
    """``python -m foremast_amd.brain --streaming --nproc 2`` with ML_ALGORITHM=lstm:
    the continuous 2-metric jobs are split over two gloo ranks, one DP step per
    tick keeps both replicas identical (weight CRC in the node table), and the
    degraded app's job finishes unhealthy naming its metrics."""
    apps = [f"app{i}" for i in range(8)]
    store, ids, proc, server, log_path = _node(
        tmp_path, 2, {"FOREMAST_DEVICE": "cpu", "CUDA_VISIBLE_DEVICES": "", "FOREMAST_DIST_BACKEND": "gloo"},
        apps, bad="app3")
    try:
        t_end = time.time() + 240
        seen_two = None
        owners = {}  # app -> owning rank, over every two-rank snapshot (finished apps leave the table)
        while time.time() < t_end and proc.poll() is None:
            t = store.get_meta("cluster_health") or {}
            mem = t.get("members", [])
            if t.get("ranks") == 2 and all(m.get("lstm_model") for m in mem):
                seen_two = t
                owners.update({a.split("/")[1]: v["rank"] for a, v in t.get("apps", {}).items()})
                if store.get(ids["app3"])["status"] == "completed_unhealth":
                    break
            time.sleep(0.5)
        log = log_path.read_text()[-3000:]
        assert seen_two is not None, log
        digests = {m["lstm_model"] for m in seen_two["members"]}
        assert len(digests) == 1, seen_two["members"]              # bit-identical replicas
        assert set(owners.values()) == {0, 1}, owners
        d = store.get(ids["app3"])
        assert d["status"] == "completed_unhealth", (d["status"], log)
        assert set(json.loads(d["anomalyInfo"])) == {"latency", "error5xx"}
    finally:
        _stop(proc, server)


@pytest.mark.gpu
def test_lstm_node_gpu_forced_collectives(tmp_path):
    """The same path on the GPU: one rank, RCCL group, collectives forced
    (gradient all-reduce + node exchange as with 8 ranks)."""
    apps = [f"app{i}" for i in range(6)]
    store, ids, proc, server, log_path = _node(tmp_path, 1, {"FOREMAST_FORCE_COLLECTIVES": "1",
                                                            "FOREMAST_LSTM_WINDOW": "32", "FOREMAST_LSTM_HIDDEN": "64"},
                                               apps, bad="app3")
    try:
        t_end = time.time() + 150
        t = {}
        while time.time() < t_end and proc.poll() is None:
            t = store.get_meta("cluster_health") or {}
            if store.get(ids["app3"])["status"] == "completed_unhealth":
                break
            time.sleep(0.5)
        log = log_path.read_text()[-3000:]
        assert store.get(ids["app3"])["status"] == "completed_unhealth", log
        assert t.get("backend") == "nccl" and t.get("collectives") is True, t
        assert t["members"][0].get("lstm_model")
    finally:
        _stop(proc, server)


def test_anomaly_info_is_json_dumps():
    """The verdict's anomalyInfo string is built without the json encoder's per-call
    setup; it must stay string-equal to json.dumps (NaN / Infinity / escapes included)."""
    import json
    from foremast_amd.brain.lstm_monitor import anomaly_info
    cases = [(1.7e9, [("latency", 1.5), ("error_rate", float("nan"))]),
             (0.0, [('a"b', float("inf")), ("é", -0.0), ("c", float("-inf"))]),
             (60.0, [("x", 3.0000001192092896)])]
    for t, pairs in cases:
        assert anomaly_info(t, pairs) == json.dumps({k: {"tags": "lstm", "values": [t, v]} for k, v in pairs})
