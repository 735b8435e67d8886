"""Multi-process paths on CPU (gloo): health aggregation, sharding and the
bench's distributed contract (rank 0 prints ONE JSON line)."""

import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from foremast_amd.parallel.health import HealthAggregator, shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_total, A = 23, 5
        s, e, per = shard_range(n_total, world, rank, align=5)
        n = e - s
        agg = HealthAggregator(n, per, "cpu")
        stats = torch.zeros((A, 2), dtype=torch.int32)
        app = torch.arange(s, e) // 5
        verdict = torch.tensor([1 if (i % 7 == 0) else 0 for i in range(s, e)], dtype=torch.int8)
        for a, v in zip(app.tolist(), verdict.tolist()):
            stats[a, 0] += int(v == 1)
            stats[a, 1] += 1
        red, allv = agg.tick(stats, verdict)
        q.put((rank, red.tolist(), allv.tolist(), per))
    finally:
        dist.destroy_process_group()


def test_health_aggregation_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    exp = [[0, 0] for _ in range(5)]
    for i in range(23):
        exp[i // 5][0] += int(i % 7 == 0)
        exp[i // 5][1] += 1
    for rank, red, allv, per in res:
        assert red == exp
        # gathered verdict table: rank blocks of `per` padded with -1
        flat = [v for v in allv]
        got = [flat[r * per + j] for r in range(world) for j in range(per)]
        valid = [g for g in got if g != -1]
        assert len(valid) == 23


def _fused_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_total, mpa = 23, 5
        s, e, per = shard_range(n_total, world, rank, align=mpa)
        n = e - s
        agg = HealthAggregator(n, per, "cpu", apps_per_rank=per // mpa)
        assert agg.fused
        # the scorer writes straight into the send record (local app ids)
        app = torch.arange(s, e) // mpa - s // mpa
        verdict = torch.tensor([1 if (i % 7 == 0) else 0 for i in range(s, e)], dtype=torch.int8)
        agg.verdict_local.copy_(verdict)
        for a, v in zip(app.tolist(), verdict.tolist()):
            agg.app_stats_local[a, 0] += int(v == 1)
            agg.app_stats_local[a, 1] += 1
        apps, verd = agg.tick(agg.app_stats_local, agg.verdict_local)
        table = HealthAggregator.host_app_table(agg.recv.clone(), world, per // mpa)
        q.put((rank, apps.reshape(-1, 2).tolist(), table.tolist(), verd.tolist(), per))
    finally:
        dist.destroy_process_group()


def test_health_aggregation_fused_gloo():
    """Fused mode: one all-gather of [app slice | verdict bytes] records gives the
    same node table as all-reduce + all-gather."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fused_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [[0, 0] for _ in range(5)]
    for i in range(23):
        exp[i // 5][0] += int(i % 7 == 0)
        exp[i // 5][1] += 1
    for rank, apps, table, verd, per in res:
        apr = per // 5
        assert apps == table
        assert table[:5] == exp and all(r == [0, 0] for r in table[5:])
        assert len(table) == world * apr
        got = [v for row in verd for v in row]
        assert sorted(v for v in got if v != -1) == sorted(1 if i % 7 == 0 else 0 for i in range(23))


def test_shard_range_alignment():
    world = 8
    spans = [shard_range(100_000, world, r, align=5) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == 100_000
    for (s, e, per), (s2, _, _) in zip(spans, spans[1:]):
        assert e == s2 and s % 5 == 0
    assert sum(e - s for s, e, _ in spans) == 100_000


@pytest.mark.slow
@pytest.mark.parametrize("config", ["canary", "lstm", "multicluster", "selflaunch", "gaps"])
def test_bench_distributed_cpu(config):
    """Under torchrun, and (``selflaunch``) as the driver may call it: a plain
    ``python bench.py --gpus 2`` that must start its own 2-rank group.  ``gaps``:
    a fifth of the histories have a 30-minute outage (masked fit path)."""
    variant = config
    extra = {"multicluster": ["--multi-cluster"], "gaps": ["--gap-frac", "0.2"]}.get(config, [])
    launcher = config != "selflaunch"
    config = "canary" if config in ("multicluster", "selflaunch", "gaps") else config
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    pre = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}"] if launcher else [sys.executable]
    cmd = pre + [os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu", "--series", "200", "--ring", "480",
           "--season", "48", "--config", config, "--lstm-train-batch", "32", "--lstm-pretrain", "2"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["bench_config"] == config
    assert d["health"]["series_scored_last_tick"] == 200
    if variant == "multicluster":
        assert d["config"]["multi_cluster"] is True and d["detection"]["recall"] == 1.0
        assert d["config"]["affine_exchanges"] >= 3   # product router: one exchange per ingested tick
    if variant == "gaps":
        assert d["config"]["gap_frac"] == 0.2 and d["detection"]["recall"] == 1.0
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype",
              "data", "config"):
        assert k in d


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from foremast_amd.models.lstm_ae import LSTMAutoencoder
        from foremast_amd.parallel.dp import DPTrainer
        torch.manual_seed(100 + rank)  # different init per rank → broadcast must align them
        m = LSTMAutoencoder(2, 16)
        tr = DPTrainer(m, lr=1e-2, bucket_bytes=2048)  # several buckets
        g = torch.Generator().manual_seed(rank)
        for _ in range(3):
            x = torch.randn(8, 6, 2, generator=g)
            tr.step(x)
        flat = torch.cat([p.detach().flatten() for p in m.parameters()])
        q.put((rank, flat.numpy().tolist(), len(tr.buckets.buckets)))
    finally:
        dist.destroy_process_group()


def test_dp_trainer_keeps_replicas_identical():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, p0, nb), (r1, p1, _) = res
    assert nb > 1
    assert np.allclose(p0, p1, atol=1e-6)


def test_dp_single_process_matches_plain_adam():
    from foremast_amd.models.lstm_ae import LSTMAutoencoder
    from foremast_amd.parallel.dp import DPTrainer
    torch.manual_seed(0)
    a = LSTMAutoencoder(1, 8)
    b = LSTMAutoencoder(1, 8)
    b.load_state_dict(a.state_dict())
    tr = DPTrainer(a, lr=1e-2)
    opt = torch.optim.Adam(b.parameters(), lr=1e-2)
    x = torch.randn(4, 5, 1)
    for _ in range(3):
        tr.step(x)
        opt.zero_grad()
        b.recon_error(x).mean().backward()
        opt.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-6)


def _elastic_worker(mid, members, port, q, die_after):
    import datetime as _dt
    from torch.distributed import TCPStore
    from foremast_amd.parallel.elastic import ElasticWorld
    store = TCPStore("127.0.0.1", port, is_master=False, timeout=_dt.timedelta(seconds=60))
    # generous liveness margins: a live rank of a loaded CI box (parallel test
    # workers) must not miss heartbeats for 3 s; the killed one stops for good
    ew = ElasticWorld(store, mid, members, backend="gloo", heartbeat_timeout_s=3.0, collective_timeout_s=10)
    ew.start_heartbeat(0.2)
    ew.form()
    n_total = 1000
    log = []
    for tick in range(6):
        if die_after is not None and tick == die_after:
            os._exit(0)  # simulated crash: no cleanup, heartbeats stop

        def work():
            s, e, _ = shard_range(n_total, ew.world, ew.rank, align=5)
            t = torch.tensor([e - s], dtype=torch.int64)
            dist.all_reduce(t)
            return int(t.item())
        total = ew.run_tick(work)
        log.append((tick, ew.world, total))
        time.sleep(0.3)
    ew.stop_heartbeat()
    q.put((mid, log, ew.reforms))
    dist.destroy_process_group()


def test_elastic_recovery_reshards_after_rank_death():
    import datetime as _dt
    from torch.distributed import TCPStore
    port = _free_port()
    store = TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False, timeout=_dt.timedelta(seconds=60))
    members = ["m0", "m1", "m2"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_elastic_worker, args=(m, members, port, q, 2 if m == "m2" else None))
             for m in members]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    del store
    for mid, log, reforms in res:
        assert [t for t, _, _ in log] == list(range(6))
        assert all(total == 1000 for _, _, total in log), log   # every series scored every tick
        assert log[0][1] == 3 and log[-1][1] == 2 and reforms == 1, log


def _bench_line(n, extra=()):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1", "--cpu",
           "--series", "400", "--ring", "480", "--season", "48", "--anomaly-frac", "0.05"] + list(extra)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.slow
@pytest.mark.parametrize("extra", [(), ("--gap-frac", "0.2")], ids=["canary", "gaps"])
def test_bench_n_rank_equals_one_rank(extra):
    """Every datum of the bench is a function of the GLOBAL series index, so the
    1, 2, 4 and 8-rank runs (self-launched gloo groups, one all-gather per tick)
    score the same 400 series and must report the same node health table and the
    same detection against the same injected regressions."""
    ref = _bench_line(1, extra)
    assert ref["detection"]["injected_apps"] > 0 and ref["health"]["series_scored_last_tick"] == 400
    for n in (2, 4, 8):
        d = _bench_line(n, extra)
        assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}"
        assert d["health"] == ref["health"], n
        assert d["detection"] == ref["detection"], n


class _FlakyStore:
    """A store whose ``set`` fails ``fail`` times, then works (a transient TCPStore error)."""

    def __init__(self, fail: int) -> None:
        self.kv, self.fail, self.calls = {}, fail, 0

    def set(self, k, v):
        self.calls += 1
        if self.fail > 0:
            self.fail -= 1
            raise RuntimeError("store hiccup")
        self.kv[k] = v.encode() if isinstance(v, str) else v

    def check(self, keys):
        return all(k in self.kv for k in keys)

    def get(self, k):
        return self.kv[k]


def test_heartbeat_thread_survives_a_transient_store_error():
    """one failing ``hb_store.set`` must not end the heartbeat (the rank
    would be voted out while healthy); a thread that does give up is recorded so
    ``changed()`` beats on the main thread."""
    from foremast_amd.parallel.elastic import ElasticWorld
    main, hb = _FlakyStore(0), _FlakyStore(1)
    ew = ElasticWorld(main, "a", ["a"], heartbeat_timeout_s=0.4, heartbeat_store=hb)
    ew.start_heartbeat(period_s=0.02)
    t_end = time.time() + 5
    while "hb/a" not in hb.kv and time.time() < t_end:
        time.sleep(0.01)
    assert "hb/a" in hb.kv and hb.calls >= 2   # the first set failed, a later one landed
    assert not ew._hb_dead.is_set()
    ew.stop_heartbeat()
    # a store that stays down: the thread gives up and says so; changed() then beats itself
    dead = _FlakyStore(10 ** 6)
    ew2 = ElasticWorld(main, "b", ["b"], heartbeat_timeout_s=0.1, heartbeat_store=dead)
    ew2.start_heartbeat(period_s=0.01)
    assert ew2._hb_dead.wait(5.0)
    main.kv.pop("hb/b", None)
    assert not ew2.changed()
    assert "hb/b" in main.kv
