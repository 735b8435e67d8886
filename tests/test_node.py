"""Node brain: app-sharded ranks, one all-gather of per-app counters per tick,
the node health table behind GET /v1/healthcheck/cluster, and survival of a
rank kill (gloo on CPU; the GPU run uses the same code with RCCL)."""

import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import pytest
import torch

from foremast_amd.brain.node import owner_of
from foremast_amd.parallel.cluster import ClusterHealth
from foremast_amd.promql import synth
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.service import app as svc
from foremast_amd.store.jobstore import SqliteJobStore
from foremast_amd.utils.timeutil import format_rfc3339

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M = "namespace_app_per_pod:http_server_requests_error_5xx"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _job(app, endpoint, now):
    q = f'{M}{{namespace="ns",app="{app}"}}'
    params = {"endpoint": endpoint, "query": q, "step": 60}
    return {"appName": app, "startTime": format_rfc3339(now), "endTime": format_rfc3339(now + 86400),
            "strategy": "continuous",
            "metrics": {"current": {"error5xx": {"dataSourceType": "prometheus",
                                                 "parameters": dict(params, start=int(now), end=int(now + 600))}},
                        "historical": {"error5xx": {"dataSourceType": "prometheus",
                                                    "parameters": dict(params, start=int(now - 86400),
                                                                       end=int(now))}}}}


def test_owner_of_is_stable_and_spread():
    owners = [owner_of("ns", f"app{i}", 4) for i in range(400)]
    assert owners == [owner_of("ns", f"app{i}", 4) for i in range(400)]
    assert min(owners.count(r) for r in range(4)) > 60


def test_cluster_health_single_rank_table():
    h = ClusterHealth("cpu", cap=2)
    names = [("ns", "a"), ("ns", "b"), ("ns", "c")]
    counts = torch.tensor([[1, 5], [0, 5], [0, 3]], dtype=torch.int32)
    t = h.exchange(names, counts, 1, 13, {"member": "m0"})
    # the record held 2 apps this tick and asked for 4 rows: the third shows up next tick
    assert sorted(t["apps"]) == ["ns/a", "ns/b"] and h.cap == 4
    t = h.exchange(names, counts, 1, 13, {"member": "m0"})
    assert t["apps"]["ns/c"] == {"anomalous": 0, "scored": 3, "rank": 0}
    assert t["anomalous_apps"] == ["ns/a"] and t["members"][0]["series"] == 13
    assert h.roster_exchanges == 0 and h.last_roster_bytes == 0  # one rank: no peer roster to read


def _serve(app, port):
    import uvicorn
    cfg = uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning")
    server = uvicorn.Server(cfg)
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    for _ in range(100):
        if server.started:
            return server
        time.sleep(0.05)
    raise RuntimeError("fake prometheus did not start")


@pytest.mark.slow
def test_node_brain_two_ranks_cluster_table_and_rank_kill(tmp_path):
    prom = FakePrometheus()
    apps = [f"app{i}" for i in range(8)]
    for i, app in enumerate(apps):
        gen = synth.error_rate(base=0.3 + 0.02 * i, spread=0.05, seed=i)
        if app == "app3":
            gen = synth.step_change(gen, at=time.time() - 150, factor=0.0, add=40.0)  # inside the current window
        prom.add(M, {"namespace": "ns", "app": app}, gen)
    port = _free_port()
    server = _serve(prom.asgi_app(), port)
    db = str(tmp_path / "jobs.db")
    store = SqliteJobStore(db)
    now = time.time()
    ids = {app: svc.register(store, _job(app, f"http://127.0.0.1:{port}/api/v1/", now))[1]["jobId"] for app in apps}
    env = dict(os.environ, FOREMAST_RING_LEN="240", FOREMAST_HEARTBEAT_S="2", FOREMAST_COLLECTIVE_TIMEOUT_S="20",
               MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", ML_ALGORITHM="moving_average_all", OMP_NUM_THREADS="1",
               FOREMAST_DEVICE="cpu", CUDA_VISIBLE_DEVICES="", FOREMAST_DIST_BACKEND="gloo",
               metric_type_threshold_count="1", metric_type0="error5xx", threshold0="6", bound0="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "foremast_amd.brain", "--streaming", "--nproc", "2", "--store", f"sqlite://{db}",
           "--metrics-port", "0", "--tick-seconds", "1", "--window", "5"]
    log_path = tmp_path / "node.log"
    launcher = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=open(log_path, "w"), stderr=subprocess.STDOUT,
                                start_new_session=True)

    def table():
        return store.get_meta("cluster_health") or {}

    def wait(pred, what, timeout=120):
        t_end = time.time() + timeout
        while time.time() < t_end:
            t = table()
            if t and pred(t):
                return t
            if launcher.poll() is not None:
                break
            time.sleep(0.5)
        raise AssertionError(f"{what}: last table {json.dumps(table())[:600]}\n{log_path.read_text()[-3000:]}")

    try:
        t = wait(lambda t: t["ranks"] == 2 and len(t["apps"]) == len(apps), "both ranks publish")
        owners = {a.split("/")[1]: v["rank"] for a, v in t["apps"].items()}
        assert set(owners.values()) == {0, 1}
        assert all(owners[a] == owner_of("ns", a, 2) for a in apps)
        # the anomalous app's job finishes unhealthy on its owner
        t_end = time.time() + 60
        while store.get(ids["app3"])["status"] != "completed_unhealth" and time.time() < t_end:
            time.sleep(0.5)
        assert store.get(ids["app3"])["status"] == "completed_unhealth"
        # the service serves the published table
        from fastapi.testclient import TestClient
        c = TestClient(svc.create_app(store=store, query_endpoint="http://127.0.0.1:1/"))
        body = c.get("/v1/healthcheck/cluster").json()
        assert body["ranks"] == 2 and "ns/app0" in body["apps"]
        # kill rank 0's process: the survivor re-forms alone, takes over every app at once
        victim = [m for m in t["members"] if m["rank"] == 0][0]
        os.kill(victim["pid"], signal.SIGKILL)
        live = [a for a in apps if a != "app3"]
        t = wait(lambda t: t["ranks"] == 1 and t.get("generation", 0) >= 1
                 and all(f"ns/{a}" in t["apps"] for a in live), "survivor takes over", timeout=90)
        assert {v["rank"] for v in t["apps"].values()} == {0}
        for a in live:
            d = store.get(ids[a])
            assert d["status"] == "preprocess_inprogress", (a, d["status"])
            assert d["claimed_by"] == "node-" + t["members"][0]["member"], (a, d["claimed_by"])
    finally:
        os.killpg(launcher.pid, signal.SIGTERM)
        try:
            launcher.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(launcher.pid, signal.SIGKILL)
        server.should_exit = True


@pytest.mark.gpu
def test_node_brain_gpu_rccl_one_rank(tmp_path):
    """The production node brain on the GPU: one rank launched by
    ``--nproc 1``, its ElasticWorld formed over RCCL (``nccl``), collectives
    forced in the 1-rank group (``FOREMAST_FORCE_COLLECTIVES=1``: the per-tick
    counter all-gather and roster exchange run as with 8 ranks); the node table
    is published and the injected app's job ends unhealthy."""
    prom = FakePrometheus()
    apps = [f"app{i}" for i in range(6)]
    for i, app in enumerate(apps):
        gen = synth.error_rate(base=0.3 + 0.02 * i, spread=0.05, seed=i)
        if app == "app3":
            gen = synth.step_change(gen, at=time.time() - 150, factor=0.0, add=40.0)
        prom.add(M, {"namespace": "ns", "app": app}, gen)
    port = _free_port()
    server = _serve(prom.asgi_app(), port)
    db = str(tmp_path / "jobs.db")
    store = SqliteJobStore(db)
    now = time.time()
    ids = {app: svc.register(store, _job(app, f"http://127.0.0.1:{port}/api/v1/", now))[1]["jobId"] for app in apps}
    env = dict(os.environ, FOREMAST_RING_LEN="240", FOREMAST_HEARTBEAT_S="5", FOREMAST_COLLECTIVE_TIMEOUT_S="30",
               MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", ML_ALGORITHM="moving_average_all", OMP_NUM_THREADS="2",
               FOREMAST_FORCE_COLLECTIVES="1", metric_type_threshold_count="1", metric_type0="error5xx",
               threshold0="6", bound0="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "FOREMAST_DEVICE", "FOREMAST_DIST_BACKEND", "CUDA_VISIBLE_DEVICES"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "foremast_amd.brain", "--streaming", "--nproc", "1", "--store", f"sqlite://{db}",
           "--metrics-port", "0", "--tick-seconds", "1", "--window", "5"]
    log_path = tmp_path / "node.log"
    launcher = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=open(log_path, "w"), stderr=subprocess.STDOUT,
                                start_new_session=True)
    try:
        t_end = time.time() + 90
        t = {}
        while time.time() < t_end and launcher.poll() is None:
            t = store.get_meta("cluster_health") or {}
            live = [a for a in apps if a != "app3"]  # app3's job completes unhealthy and leaves the table
            if t.get("ranks") == 1 and all(f"ns/{a}" in t.get("apps", {}) for a in live) and \
                    store.get(ids["app3"])["status"] == "completed_unhealth":
                break
            time.sleep(0.5)
        log = log_path.read_text()
        assert t.get("ranks") == 1 and all(f"ns/{a}" in t.get("apps", {}) for a in live), log[-3000:]
        assert store.get(ids["app3"])["status"] == "completed_unhealth", log[-3000:]
        assert t.get("backend") == "nccl" and t.get("collectives") is True, t
    finally:
        os.killpg(launcher.pid, signal.SIGTERM)
        try:
            launcher.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(launcher.pid, signal.SIGKILL)
        server.should_exit = True
