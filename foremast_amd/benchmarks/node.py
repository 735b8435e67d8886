"""``bench.py --config node``: the product path at node scale.

The kernel headline (``--config canary``) times a ``StreamingShard`` the bench
assembles itself.  This config times what production runs: N canary jobs x 5
metrics registered through the service's create handler (the barrelman
request, ``controller/queries.py`` = ``metricsquery.go``), claimed and scored by
the production :class:`~foremast_amd.brain.node.NodeBrain` (streaming monitor
+ rollout monitor, ``brain/rollout.py``), with every datum arriving as
Prometheus ``query_range`` JSON:

* setup (untimed): synthetic Prometheus bodies for every query the brain will
  issue are rendered in advance (an in-process server answers by URL — the
  time of rendering JSON is Prometheus', not the brain's); the node is *warm*:
  the resident 7-day history of every (app, metric) is in HBM, as after
  earlier deployments or a snapshot restore (``brain/resident.py``);
* register: every job goes through ``service.register`` (timed, reported);
* intake tick (timed, reported separately): claim + plan of every job,
  admission — the Holt-Winters grid fit of each (job, metric) on its history
  ending at the job start (100k fits), baseline-pod windows fetched as JSON and
  decoded;
* scoring ticks (the timed steps; ``value``): from "this minute's bodies are
  available" to "verdicts written to the job store": heartbeat, history
  advance (one ``namespace_app_per_pod`` body per metric family), pod windows
  (one ``namespace_pod`` body per family: every new pod's newest point),
  native keyed decode, H2D, scatter, rank tests, band / verdict / per-app
  counters, D2H, fail-fast writes of anomalous jobs, node health exchange;
* completion tick (reported): every job reaches ``endTime`` and is written
  ``completed_health`` (or stays unhealthy).

Detection quality comes from the job statuses the brain wrote (x3 regressions
on ``--anomaly-frac`` of the (job, metric) series, in the new pods only).
"""

from __future__ import annotations

import asyncio
import gc
import os
import time
from typing import Dict, List, Tuple
from urllib.parse import parse_qs, unquote, urlsplit

import numpy as np
import torch

T0 = 1_700_000_040.0     # deployment time of every job (aligned to the minute)
STEP = 60.0
METRICS = ("http_server_requests_error_5xx", "http_server_requests_latency", "http_server_requests_count",
           "process_cpu_usage", "jvm_memory_used_bytes")
ENDPOINT = "http://prometheus:9090/api/v1/"


def _fmt(v: np.ndarray) -> List[str]:
    return np.char.mod("%.9g", np.asarray(v, dtype=np.float64)).tolist()


def _body(items: List[str]) -> bytes:
    return ('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(items) + "]}}").encode()


def _series(metric: str, labels: str, ts: np.ndarray, vals: List[str]) -> str:
    pts = ",".join(f'[{int(t)},"{v}"]' for t, v in zip(ts.tolist(), vals))
    return f'{{"metric":{{"__name__":"{metric}",{labels}}},"values":[{pts}]}}'


class BodyServer:
    """In-process Prometheus stand-in for the bench: ``fetch_raw_many`` returns
    pre-rendered ``query_range`` bodies — per tick one body per family of every
    app's (``namespace_app_per_pod``) or every new pod's (``namespace_pod``)
    newest point; per family the baseline window of each old pod as a fragment,
    joined for the pods a query's ``pod=~`` matcher names."""

    def __init__(self) -> None:
        self.tick_bodies: Dict[Tuple[str, float], bytes] = {}
        self.fragments: Dict[Tuple[str, float], Dict[str, str]] = {}
        self.requests = 0
        self.bytes_served = 0
        # cold node: week loads rendered on request -- history(metric, apps, start, n) -> body
        self.history = None
        self.serve_s = 0.0

    async def fetch_raw_many(self, urls) -> List[object]:
        t0 = time.perf_counter()
        out = [self._one(u) for u in urls]
        self.serve_s += time.perf_counter() - t0
        return out

    def _one(self, url: str):
        self.requests += 1
        q, start, end = _split_range_url(url)
        if "%7B" not in q:
            body = self.tick_bodies.get((unquote(q), end), _body([]))
        else:
            name = unquote(q.split("%7B", 1)[0])
            if self.history is not None and name.startswith("namespace_app_per_pod:"):
                body = self.history(name, _encoded_values(q, "app"), start, int(round((end - start) / STEP)) + 1)
            else:
                frags = self.fragments.get((name, start), {})
                body = _body([frags[p] for p in _encoded_pods(q) if p in frags])
        self.bytes_served += len(body)
        return body


def node_world(world: int, rank: int, dev):
    """The deployed exchange for an N-rank node bench: under ``torch.distributed.run``
    (``WORLD_SIZE`` > 1) every rank joins an :class:`~foremast_amd.parallel.elastic.ElasticWorld`
    on the launcher's store, exactly as a production rank does
    (:func:`~foremast_amd.brain.node.elastic_world_from_env`): heartbeats, the
    deadline-guarded ``run_tick``, generation-prefixed roster deltas, re-formation.
    ``FOREMAST_FORCE_COLLECTIVES=1`` gives a 1-member world (one GPU, real RCCL).
    None for a plain 1-rank run."""
    from ..brain.node import elastic_world_from_env
    from ..parallel import comm
    if world <= 1 and not comm.force_collectives():
        return None
    ew = elastic_world_from_env(dev, force=comm.force_collectives())
    if ew is not None and f"m{rank}" != ew.members[rank]:
        raise SystemExit(f"node bench: member order {ew.members} does not put m{rank} at rank {rank}")
    return ew


def _exchange_bd(node, bd: Dict) -> None:
    """The node health exchange of the tick into its breakdown record."""
    t = node.table or {}
    bd["exchange_ms"] = round(float(t.get("collective_ms", 0.0)), 3)
    bd["roster_bytes"] = int(t.get("roster_bytes", 0))
    bd["generation"] = int(t.get("generation", 0))


def _start_node(node, ew) -> None:
    if ew is not None:
        node.start()


def _brainworker_share(docs, cfg) -> int:
    """Jobs no resident monitor keys (they would reach BrainWorker); the plan memo is
    reset afterwards so the timed claims decode as in production."""
    from ..brain import plans as pl
    from ..brain.lstm_monitor import lstm_features
    from ..brain.streaming import is_continuous
    ps = pl.plan_many(list(docs), cfg.algorithm)
    pl._PLANS.clear()
    return sum(1 for d, p in zip(docs, ps)
               if p is None and not (is_continuous(d) and lstm_features(d, cfg) is not None))


def _cold_record(st, intake_s, standin_s, ticks, n_cold, M, R, n_warm) -> Dict:
    """Cold-node history ingest: the week of n_cold x M series loaded from Prometheus
    JSON by the node's history path while its warm jobs keep scoring."""
    brain_s = intake_s - standin_s
    return {"cold_jobs": n_cold, "warm_jobs": n_warm, "series": n_cold * M, "points_per_series": R,
            "json_gb": round(st["body_bytes"] / 1e9, 3),
            "decode_gb_per_s": round(st["body_bytes"] / 1e9 / max(st["decode_s"], 1e-9), 2),
            "decode_s": round(st["decode_s"], 3),
            "h2d_gb_per_s": round(st["h2d_bytes"] / 1e9 / max(st["h2d_s"], 1e-9), 2),
            "load_batches": st["batches"],
            "seconds_to_admission_brain": round(brain_s, 2),
            "seconds_to_admission_wall": round(intake_s, 2),
            "standin_render_s": round(standin_s, 2),
            "intake_ticks": len(ticks) + 1,
            "ticks": ticks}


def setup_node(args, world, rank, dev):
    from ..brain.node import NodeBrain, owner_of
    from ..brain.rollout import RolloutMonitor
    from ..brain.streaming import StreamingMonitor
    from ..brain.engine import synthetic_eval, synthetic_params
    from ..ingest import native
    from ..api import crd
    from ..api import rest as r
    from ..controller import queries
    from ..service import app as svc
    from ..store import MemoryJobStore
    from ..utils.config import BrainConfig, reference_default_env
    from ..utils.timeutil import format_rfc3339

    if dev.type == "cpu" and args.series > 20000:
        args.series, args.ring = 500, 2880
    # --multi-cluster (BASELINE config 4 through the product): cluster c is scraped by rank
    # c mod world; a rank's jobs run their new pods in its own cluster, and every other app's
    # baseline pods run in the next cluster, so those baseline windows are fetched and decoded
    # by the rank serving that cluster and cross ranks in the rollout engine's lockstep
    # exchange (parallel/affine.py) -- at one rank the same exchange runs through the
    # collectives with FOREMAST_FORCE_COLLECTIVES=1 (the rank serves the other cluster itself)
    multi = bool(getattr(args, "multi_cluster", False))
    n_clusters = max(world, 2)

    def cluster_ep(c: int) -> str:
        return f"http://prom-{c}:9090/api/v1/"
    home_ep = cluster_ep(rank) if multi else ENDPOINT
    M = len(METRICS)
    n_apps = args.series // M
    P = args.pods
    W = args.window
    R, season = args.ring, args.season
    ticks = args.warmup + args.steps + 1
    if ticks > W:
        raise SystemExit(f"--config node: warmup + steps + 1 = {ticks} ticks must fit in the {W}-minute watch window "
                         f"(jobs finish at endTime); raise --window or lower --steps")
    # this rank's apps: the node brain's ownership function (the shared store sees all jobs;
    # each rank keeps its share, so a rank-local store holds exactly what that rank claims)
    owner = [owner_of(f"ns{a % 200}", f"app{a}", world) for a in range(n_apps)]
    mine = [a for a in range(n_apps) if owner[a] == rank]
    na = len(mine)

    def base_cluster(a: int) -> int:  # cluster of app a's baseline pods
        return (owner[a] + (a & 1)) % n_clusters if multi else owner[a]
    # apps whose baseline windows this rank's Prometheus serves
    served = [a for a in range(n_apps) if base_cluster(a) % world == rank] if multi else mine
    t_setup = time.perf_counter()
    clock = {"t": T0}
    server = BodyServer()
    env = reference_default_env()
    env.update(ML_ALGORITHM=args.algorithm, ML_PAIRWISE_ALGORITHM=args.pairwise,
               MIN_HISTORICAL_DATA_POINT_TO_MEASURE="0", threshold="4", bound="3")
    for i in range(5):  # every metric type: the headline's threshold 4, both bounds
        env[f"threshold{i}"], env[f"bound{i}"] = "4", "3"
    cfg = BrainConfig.from_env(env)
    cfg.ring_len = R
    cfg.season = season
    store = MemoryJobStore()

    # --- synthetic series: one seasonal model per (app, metric) ------------------------------
    g = torch.Generator().manual_seed(1234)
    gid = torch.tensor([a * M + j for a in mine for j in range(M)], dtype=torch.int64)  # global series id
    params = synthetic_params(args.series, torch.device("cpu"), seed=1234)
    params = {k: v[gid] for k, v in params.items()}
    n_bad = int(round(args.anomaly_frac * args.series))
    bad_global = set(torch.randperm(args.series, generator=g)[:n_bad].tolist())
    bad = np.array([int(x) in bad_global for x in gid.tolist()])                   # [na * M]
    truth_apps = sorted({mine[i // M] for i in np.nonzero(bad)[0].tolist()})
    noise = 0.03 * params["lvl"][:, 0].numpy()
    rng = np.random.default_rng(99 + rank)
    ns = [f"ns{a % 200}" for a in mine]
    app = [f"app{a}" for a in mine]

    # --- history: resident (warm node), generated in chunks on the device ----------------------
    roll = RolloutMonitor(store, cfg, prom=server, device=dev, worker_id=f"node-m{rank}-rollout", step=STEP,
                          window=W, pods=P, clock=lambda: clock["t"], ring_len=R, min_capacity=na * M,
                          decode_threads=args.decode_threads, apps_per_query=256)
    if multi:
        from ..parallel.affine import ClusterRouter
        roll.router = ClusterRouter(lambda ep, w: int(ep.split("prom-")[1].split(":")[0]) % max(w, 1), dev,
                                    home=[home_ep])
    keys = [(home_ep, "namespace_app_per_pod:" + m, ns[i], app[i]) for i in range(na) for m in METRICS]
    hist = roll.history
    hist.clock = lambda: clock["t"]
    # --cold: only the first cold_warm apps are resident; the week of every other (app, metric)
    # is loaded through the node's history path from Prometheus JSON (rendered on request)
    n_warm = na if not getattr(args, "cold", False) else min(na, int(args.cold_warm_jobs))
    warm_keys = keys[:n_warm * M]
    hist.want(warm_keys, T0)
    asyncio.run(hist.assign_only(T0))
    dparams = {k: v.to(dev) for k, v in params.items()}
    for c0 in range(0, len(warm_keys), 16384):
        c1 = min(len(warm_keys), c0 + 16384)
        sub = {k: v[c0:c1] for k, v in dparams.items()}
        hist.load_rows(warm_keys[c0:c1], synthetic_eval(sub, 0, R, season, noise_seed=4321 + c0))
    hist.unwant(warm_keys, T0)  # retained for retain_s after their last job: the jobs re-reference them
    if n_warm < na:
        if args.cold_budget_s > 0:
            hist.load_budget_s = args.cold_budget_s
        row_of = {(f"namespace_app_per_pod:{m}", app[i]): i * M + j for i in range(na) for j, m in enumerate(METRICS)}
        lab_of = {(f"namespace_app_per_pod:{m}", app[i]): f'"__name__":"namespace_app_per_pod:{m}","namespace":'
                                                         f'"{ns[i]}","app":"{app[i]}"'
                  for i in range(na) for m in METRICS}

        def history(name, apps, start, n):
            """The week of the named apps as query_range JSON (model time R - 1 is T0)."""
            hit = [(row_of[(name, a)], lab_of[(name, a)]) for a in apps if (name, a) in row_of]
            if not hit:
                return _body([])
            rr = torch.tensor([h for h, _ in hit])
            sub = {k: v[rr] for k, v in params.items()}
            t0c = int(round((start - T0) / STEP)) + R - 1
            # noise seeded by the time chunk: a seed repeated per chunk would repeat the noise with
            # the season's period, which a seasonal model fits exactly
            vals = synthetic_eval(sub, t0c, n, season, noise_seed=4321 + t0c).numpy()
            return native.render_matrix(native.label_blob([lab for _, lab in hit]), vals, start, STEP)
        server.history = history

    # --- Prometheus bodies -------------------------------------------------------------------
    # the newest point of minute T0 + 60 k is model time R - 1 + k; the job's baseline window
    # [T0 - W min, T0] is model time R - 1 - W .. R - 1
    new_pods = [[f"{app[i]}-v2-{p}-7d9f8b6c5d" for p in range(P)] for i in range(na)]
    old_pods = [[f"{app[i]}-v1-{p}-5b6c7d8e9f" for p in range(P)] for i in range(na)]
    app_lab = [f'"namespace":"{ns[i]}","app":"{app[i]}"' for i in range(na)]
    newp_lab = [f'"namespace":"{ns[i]}","pod":"{pod}"' for i in range(na) for pod in new_pods[i]]
    model = synthetic_eval(params, R - 1 - W, W + 1 + ticks + 1, season, None).numpy()   # [na*M, T] no noise
    # the baseline model of the served apps (rows of other ranks' apps too, under --multi-cluster)
    sgid = torch.tensor([a * M + j for a in served for j in range(M)], dtype=torch.int64)
    sparams = {k: v[sgid] for k, v in synthetic_params(args.series, torch.device("cpu"), seed=1234).items()}
    smodel = synthetic_eval(sparams, R - 1 - W, W + 1, season, None).numpy().reshape(len(served), M, W + 1)
    base_model = [smodel[:, j, :] for j in range(M)]
    snoise = 0.03 * sparams["lvl"][:, 0].numpy().reshape(len(served), M)
    base_noise = [dict(zip(served, snoise[:, j].tolist())) for j in range(M)]
    del smodel, sparams
    t_axis = T0 + STEP * (np.arange(model.shape[1]) - W)                                   # time of each column
    col = {float(t): i for i, t in enumerate(t_axis.tolist())}
    bad_m = bad.reshape(na, M)
    for j, m in enumerate(METRICS):
        rows = np.arange(na) * M + j
        for k in range(ticks + 1):
            ts = T0 + STEP * k
            c = col[ts]
            vals = model[rows, c] + rng.standard_normal(na) * noise[rows]
            server.tick_bodies[("namespace_app_per_pod:" + m, ts)] = _body(
                [f'{{"metric":{{"__name__":"namespace_app_per_pod:{m}",{lab}}},"values":[[{int(ts)},"{v}"]]}}'
                 for lab, v in zip(app_lab, _fmt(vals))])
            pv = (model[rows, c][:, None] + rng.standard_normal((na, P)) * noise[rows][:, None])
            pv = np.where(bad_m[:, j][:, None], pv * 3.0, pv)    # the regressed deployments' new pods
            server.tick_bodies[("namespace_pod:" + m, ts)] = _body(
                [f'{{"metric":{{"__name__":"namespace_pod:{m}",{lab}}},"values":[[{int(ts)},"{v}"]]}}'
                 for lab, v in zip(newp_lab, _fmt(pv.reshape(-1)))])
        # baseline windows of the old pods: [T0 - W min, T0], for the apps whose baselines this
        # rank's cluster serves; noise seeded per (app, metric): every layout serves the same data
        bt = t_axis[:W + 1]
        frags = {}
        for a, bm in zip(served, base_model[j]):
            bg = np.random.default_rng(7_000_003 + a * M + j)
            base = bm[None, :] + bg.standard_normal((P, W + 1)) * base_noise[j][a]
            for p in range(P):
                pod = f"app{a}-v1-{p}-5b6c7d8e9f"
                frags[pod] = _series("namespace_pod:" + m, f'"namespace":"ns{a % 200}","pod":"{pod}"', bt,
                                     _fmt(base[p]))
        server.fragments[("namespace_pod:" + m, float(bt[0]))] = frags
    del model

    # --- jobs: the barrelman request of a canary rollout per app, through the service ---------
    mets = crd.Metrics(data_source_type="prometheus", endpoint=home_ep,
                       monitoring=[crd.Monitoring(metric_name=m, metric_alias=f"m{j}") for j, m in enumerate(METRICS)])
    reqs = []
    for i in range(na):
        info = queries.create_metrics_info(ns[i], app[i], [new_pods[i], old_pods[i]], mets, W, "canary", now=T0)
        body = r.ApplicationHealthAnalyzeRequest(app_name=app[i], start_time=format_rfc3339(T0),
                                                 end_time=format_rfc3339(T0 + W * STEP), metrics=info,
                                                 strategy="canary").to_dict()
        bc = base_cluster(mine[i])
        if multi and bc != rank:  # this app's baseline pods run in another cluster
            for q in body["metrics"]["baseline"].values():
                q["parameters"]["endpoint"] = cluster_ep(bc)
        reqs.append(body)
    setup_s = time.perf_counter() - t_setup
    t0 = time.perf_counter()
    job_of = {}
    for i, body in enumerate(reqs):
        code, resp = svc.register(store, body)
        assert code == 200, resp
        job_of[resp["jobId"]] = mine[i]
    register_s = time.perf_counter() - t0
    del reqs
    n_worker = _brainworker_share(list(store._docs.values()), cfg)

    stream = StreamingMonitor(store, cfg, prom=server, device=dev, worker_id=f"node-m{rank}", ring_len=R,
                              window=W, clock=lambda: clock["t"])
    ew = node_world(world, rank, dev)
    node = NodeBrain(stream, ew, store, dev, publish=False, extra=(roll,))
    node.owns = lambda d: True  # the rank-local store holds exactly this rank's share
    for mon in node.monitors:
        mon.owns = None
    _start_node(node, ew)
    loop = asyncio.new_event_loop()
    flagged = set()

    def run_tick():
        table = loop.run_until_complete(node.tick())
        return table

    # --- intake tick: claim + admission of every job --------------------------------------------
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    cold_ticks: List[Dict[str, float]] = []
    cold = n_warm < na
    serve0 = server.serve_s
    run_tick()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if cold:
        # the node keeps ticking while the week loads: every intake loads within its budget and
        # admits the jobs whose history is complete; the admitted jobs are scored every tick
        for k in range(1, 100000):  # (the intake ticks stay at the deploy minute: no window time passes)
            st = dict(hist.load_stats)
            cold_ticks.append({"tick": k - 1, "admitted_total": len(roll.jobs), "live_rows": roll.n_live,
                               **{kk: round(v, 3) for kk, v in node.timings.items()}})
            done = len(roll.jobs) == na
            if ew is not None:  # lockstep: every rank runs the same number of intake ticks
                flag = torch.tensor([int(done)], dtype=torch.int32, device=dev)
                torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
                done = bool(flag.item())
            if done:
                break
            clock["t"] = T0 + STEP * 0  # the intake ticks all run at the deploy minute
            run_tick()
            if dev.type == "cuda":
                torch.cuda.synchronize()
    intake_s = time.perf_counter() - t0
    standin_s = server.serve_s - serve0
    assert len(roll.jobs) == na, f"admitted {len(roll.jobs)} of {na} jobs"
    intake_timings = dict(roll.timings)

    health = torch.zeros((n_apps, 2), dtype=torch.int32)
    health[mine, 1] = 1
    scored: List[int] = []
    breakdowns: List[Dict[str, float]] = []

    gc_pause = {"t": 0.0, "t0": 0.0, "n": 0}

    def _gc_cb(phase, info):  # cyclic-GC pauses inside the timed ticks (reported per tick)
        if phase == "start":
            gc_pause["t0"] = time.perf_counter()
        else:
            gc_pause["t"] += time.perf_counter() - gc_pause["t0"]
            gc_pause["n"] += 1

    def tick(k):
        clock["t"] = T0 + STEP * (k + 1)
        n_rows = roll.n_live
        gc_pause["t"], gc_pause["n"] = 0.0, 0
        gc.callbacks.append(_gc_cb)
        try:
            table = run_tick()
        finally:
            gc.callbacks.remove(_gc_cb)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        scored.append(n_rows)
        bd = {k: round(v, 2) for k, v in roll.timings.items() if k != "admit_ms"}
        bd["gc_ms"], bd["gc_runs"] = round(gc_pause["t"] * 1e3, 2), gc_pause["n"]
        _exchange_bd(node, bd)
        breakdowns.append(bd)
        for a in table["anomalous_apps"]:
            flagged.add(int(a.split("/app")[1]))
        return table

    def finish():
        """The completion tick (every job past endTime) and the verdicts written."""
        clock["t"] = T0 + STEP * W
        t0 = time.perf_counter()
        run_tick()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        fin = time.perf_counter() - t0
        st: Dict[str, int] = {}
        for d in store.all():
            st[d["status"]] = st.get(d["status"], 0) + 1
            if d["status"] == r.ST_COMPLETED_UNHEALTH:
                health[job_of[d["id"]], 0] = 1
        return fin, st

    meta = {
        "model": f"{args.algorithm} + pairwise {args.pairwise} canary jobs on the production node brain "
                 f"(rollout engine: model fitted at admission, per-tick pod windows)",
        "global_batch": args.series,
        "seq_len": R,
        "season": season,
        "jobs": n_apps,
        "metrics_per_job": M,
        "pods_new_old": [P, P],
        "watch_window_min": W,
        "path": "service.register -> store claim -> plan -> resident history -> fit at admission -> per tick: "
                "pod windows as query_range JSON -> native decode -> H2D -> scatter -> rank tests "
                "-> cached-state band/verdict -> D2H -> fail-fast writes -> node health exchange [detect latency] "
                "-> endTime writes, history advance, claims, admission",
        "warm_node": "resident 7-day history of every (app, metric) in HBM before the jobs arrive",
        "multi_cluster": ({"clusters": n_clusters, "cross_cluster_baselines": "every other app",
                           "exchange": "rollout engine: baseline windows requested at admission, served by the "
                                       "cluster's rank, one all_to_all into a device buffer, scattered on the device",
                           "admission": {k: intake_timings.get(k) for k in ("affine_ms", "affine_bytes",
                                                                            "affine_requests")},
                           "values_moved": int(roll.router.values_moved),
                           "request_bytes": int(roll.router.request_bytes),
                           "exchanges_with_requests": int(roll.router.exchanges)} if multi else False),
        "setup_s": round(setup_s, 2),
        "register_s": round(register_s, 3),
        "register_jobs_per_s": round(na / max(register_s, 1e-9), 1),
        "jobs_to_brainworker": n_worker,
        "intake_s": round(intake_s, 3),
        "intake_breakdown_ms": {k: round(v, 2) for k, v in intake_timings.items()},
        **({"cold": _cold_record(hist.load_stats, intake_s, standin_s, cold_ticks, na - n_warm, M, R, n_warm)}
           if cold else {}),
        "_scored_rows": scored,
        "_breakdowns": breakdowns,
        "_finish": finish,
        "_roll": roll,
        "_server": server,
        "_flagged": flagged,
        "_truth": (truth_apps, n_apps),
    }
    return tick, health, meta, "bf16" if dev.type == "cuda" else "fp32", na * M


# --------------------------------------------------------------------------- steady arrivals
def _split_range_url(url: str) -> Tuple[str, float, float]:
    """(percent-encoded query, start, end) of a ``resident.range_url`` URL: the
    stand-ins split the four parameters directly (urllib's parse_qs on a 30 KB
    selector of 1,280 pods costs milliseconds per query, which would be charged to
    the brain's tick)."""
    qs = url.split("query_range?", 1)[1]
    q, st, en = "", 0.0, 0.0
    for part in qs.split("&"):
        k, _, v = part.partition("=")
        if k == "query":
            q = v
        elif k == "start":
            st = float(v)
        elif k == "end":
            en = float(v)
    return q, st, en


def _encoded_pods(q: str) -> List[str]:
    """Pod names of an encoded ``pod=~"a|b"`` matcher."""
    return _encoded_values(q, "pod")


def _encoded_values(q: str, label: str) -> List[str]:
    """Values of an encoded ``<label>=~"a|b"`` matcher."""
    key = label + "%3D~%22"
    i = q.find(key)
    if i < 0:
        return []
    body = q[i + len(key):q.find("%22", i + len(key))]
    return [unquote(p) if "%" in p else p for p in body.split("%7C")]


class ArrivalServer:
    """Prometheus stand-in of the steady-arrival bench: per tick one pre-rendered
    body per family (every app's newest point; every live new pod's newest point),
    and baseline windows rendered on request for the pods a query names (native
    encoder, so the stand-in's own time stays small next to the brain's)."""

    def __init__(self) -> None:
        self.tick_bodies: Dict[Tuple[str, float], bytes] = {}
        # (family, window start) -> (pod -> row, label objects, values [pods, W + 1])
        self.windows: Dict[Tuple[str, float], Tuple[Dict[str, int], List[str], np.ndarray]] = {}
        self.requests = 0
        self.bytes_served = 0
        self.serve_s = 0.0
        self.serve_tick_s = 0.0     # the tick's family bodies (scoring half)
        self.serve_window_s = 0.0   # selector queries: baseline windows of admissions (intake half)

    async def fetch_raw_many(self, urls) -> List[object]:
        out = []
        for u in urls:
            t0 = time.perf_counter()
            out.append(self._one(u))
            dt = time.perf_counter() - t0
            self.serve_s += dt
            if "%7B" in u:
                self.serve_window_s += dt
            else:
                self.serve_tick_s += dt
        return out

    def _one(self, url: str):
        from ..ingest import native
        self.requests += 1
        q, start, end = _split_range_url(url)
        if "%7B" not in q:
            body = self.tick_bodies.get((unquote(q), end), _body([]))
        else:
            name = unquote(q.split("%7B", 1)[0])
            win = self.windows.get((name, start))
            pods = _encoded_pods(q)
            if win is None:
                body = _body([])
            else:
                idx, labels, vals = win
                rows = [idx[p] for p in pods if p in idx]
                body = native.render_matrix(native.label_blob([labels[i] for i in rows]), vals[rows], start, STEP)
        self.bytes_served += len(body)
        return body


def setup_arrival(args, world, rank, dev):
    """``--config node --arrival-per-tick J``: the product path under a steady
    deployment stream.  Every tick J canary rollouts start (one job per app, 5
    metrics, P new + P old pods: the barrelman request of ``Barrelman.go:783-899``
    with the 10-minute watch of ``:52``), each finishes at its endTime; at steady
    state the node holds ~J x W jobs (2,000 x 10 = 20,000 jobs = 100k live rows by
    default).  Arrivals are registered by the service's create handler at setup
    (the service's work, not the brain's) and enter the job store at their start
    minute.  Each timed tick is NodeBrain.tick: scoring of the running jobs, the
    node health exchange (detect latency ends here), then the claim and admission
    of that minute's arrivals (decode, rows, slots, Holt-Winters fit of 5 J
    histories, baseline windows).  The node is warm: the 7-day history of every
    (app, metric) is resident (``brain/resident.py``)."""
    from ..api import crd
    from ..api import rest as r
    from ..brain.engine import synthetic_eval, synthetic_params
    from ..brain.node import NodeBrain, owner_of
    from ..brain.rollout import RolloutMonitor
    from ..brain.streaming import StreamingMonitor
    from ..controller import queries
    from ..ingest import native
    from ..service import app as svc
    from ..store import MemoryJobStore
    from ..utils.config import BrainConfig, reference_default_env
    from ..utils.timeutil import format_rfc3339

    M, P, W = len(METRICS), args.pods, args.window
    R, season = args.ring, args.season
    J = int(args.arrival_per_tick)
    if dev.type == "cpu" and not os.environ.get("FOREMAST_BENCH_CPU_FULL"):
        J, R = min(J, 40), min(R, 2880)
    ticks = args.warmup + args.steps + 1
    A_all = J * (W + 1)                       # app pool: an app redeploys once its last job ended
    mine = [a for a in range(A_all) if owner_of(f"ns{a % 200}", f"app{a}", world) == rank]
    local = {a: i for i, a in enumerate(mine)}
    na = len(mine)
    t_setup = time.perf_counter()
    clock = {"t": T0}
    server = ArrivalServer()
    env = reference_default_env()
    env.update(ML_ALGORITHM=args.algorithm, ML_PAIRWISE_ALGORITHM=args.pairwise,
               MIN_HISTORICAL_DATA_POINT_TO_MEASURE="0", threshold="4", bound="3")
    for i in range(5):
        env[f"threshold{i}"], env[f"bound{i}"] = "4", "3"
    cfg = BrainConfig.from_env(env)
    cfg.ring_len, cfg.season = R, season
    store = MemoryJobStore()
    ns = [f"ns{a % 200}" for a in mine]
    app = [f"app{a}" for a in mine]
    gid = torch.tensor([a * M + j for a in mine for j in range(M)], dtype=torch.int64)
    params = {k: v[gid] for k, v in synthetic_params(A_all * M, torch.device("cpu"), seed=1234).items()}
    noise = 0.03 * params["lvl"][:, 0].numpy()
    rng = np.random.default_rng(99 + rank)

    # --- resident history (warm node) ---------------------------------------------------------
    roll = RolloutMonitor(store, cfg, prom=server, device=dev, worker_id=f"node-m{rank}-rollout", step=STEP,
                          window=W, pods=P, clock=lambda: clock["t"], ring_len=R, min_capacity=max(64, J * W * M),
                          decode_threads=args.decode_threads, apps_per_query=256)
    keys = [(ENDPOINT, "namespace_app_per_pod:" + m, ns[i], app[i]) for i in range(na) for m in METRICS]
    hist = roll.history
    hist.clock = lambda: clock["t"]
    hist.want(keys, T0)
    asyncio.run(hist.assign_only(T0))
    dparams = {k: v.to(dev) for k, v in params.items()}
    for c0 in range(0, len(keys), 16384):
        c1 = min(len(keys), c0 + 16384)
        hist.load_rows(keys[c0:c1], synthetic_eval({k: v[c0:c1] for k, v in dparams.items()}, 0, R, season,
                                                   noise_seed=4321 + c0))
    hist.unwant(keys, T0)

    # --- the deployment schedule: tick k deploys apps (k J .. k J + J) mod A (revision k // (W + 1))
    deploys: List[List[int]] = []    # per tick: local app indices deploying
    for k in range(ticks):
        deploys.append([local[a % A_all] for a in range(k * J, k * J + J) if a % A_all in local])
    rev = lambda k: k // (W + 1) + 1                                              # noqa: E731
    new_pods = lambda i, k: [f"{app[i]}-v{rev(k) + 1}-{p}-7d9f8b6c5d" for p in range(P)]  # noqa: E731
    old_pods = lambda i, k: [f"{app[i]}-v{rev(k)}-{p}-5b6c7d8e9f" for p in range(P)]      # noqa: E731
    n_bad = int(round(args.anomaly_frac * M * sum(len(d) for d in deploys)))
    bad_set = set(rng.choice(sum(len(d) for d in deploys) * M, size=n_bad, replace=False).tolist()) if n_bad else set()
    model = synthetic_eval(params, R - 1 - W, W + 1 + ticks + W + 1, season, None).numpy()  # [na*M, T] no noise
    col = lambda t: int(round((t - T0) / STEP)) + W                                # noqa: E731

    # --- jobs: the barrelman request of each rollout, through the service (staged) ------------
    mets = crd.Metrics(data_source_type="prometheus", endpoint=ENDPOINT,
                       monitoring=[crd.Monitoring(metric_name=m, metric_alias=f"m{j}") for j, m in enumerate(METRICS)])
    staging = MemoryJobStore()
    arrivals: List[List[Dict]] = []
    truth: Dict[str, bool] = {}
    job_bad: List[List[np.ndarray]] = []   # per tick, per deploying app: [M] injected flags
    t_reg = time.perf_counter()
    seq = 0
    for k in range(ticks):
        tk = T0 + STEP * k
        docs, flags = [], []
        for i in deploys[k]:
            info = queries.create_metrics_info(ns[i], app[i], [new_pods(i, k), old_pods(i, k)], mets, W, "canary",
                                               now=tk)
            req = r.ApplicationHealthAnalyzeRequest(app_name=app[i], start_time=format_rfc3339(tk),
                                                    end_time=format_rfc3339(tk + W * STEP), metrics=info,
                                                    strategy="canary").to_dict()
            code, resp = svc.register(staging, req)
            assert code == 200, resp
            f = np.array([(seq * M + j) in bad_set for j in range(M)])
            seq += 1
            flags.append(f)
            d = staging._docs[resp["jobId"]]
            truth[d["id"]] = bool(f.any())
            docs.append(d)
        arrivals.append(docs)
        job_bad.append(flags)
    register_s = time.perf_counter() - t_reg

    # --- Prometheus bodies (native encoder) ---------------------------------------------------
    app_lab = {m: native.label_blob([f'"__name__":"namespace_app_per_pod:{m}","namespace":"{ns[i]}","app":"{app[i]}"'
                                     for i in range(na)]) for m in METRICS}
    for k in range(ticks + W + 1):
        tk = T0 + STEP * k
        c = col(tk)
        live = [(kk, i, n) for kk in range(max(0, k - W), min(k + 1, ticks)) for n, i in enumerate(deploys[kk])]
        for j, m in enumerate(METRICS):
            rows = np.arange(na) * M + j
            vals = (model[rows, c] + rng.standard_normal(na) * noise[rows]).astype(np.float32)
            server.tick_bodies[("namespace_app_per_pod:" + m, tk)] = native.render_matrix(app_lab[m], vals[:, None],
                                                                                          tk, STEP)
            if live:
                li = np.array([i for _, i, _ in live])
                lv = model[li * M + j, c][:, None] + rng.standard_normal((len(live), P)) * noise[li * M + j][:, None]
                badf = np.array([job_bad[kk][n][j] for kk, _, n in live])
                lv = np.where(badf[:, None], lv * 3.0, lv).astype(np.float32).reshape(-1)
                labels = [f'"__name__":"namespace_pod:{m}","namespace":"{ns[i]}","pod":"{pod}"'
                          for kk, i, _ in live for pod in new_pods(i, kk)]
                server.tick_bodies[("namespace_pod:" + m, tk)] = native.render_matrix(
                    native.label_blob(labels), lv[:, None], tk, STEP)
        if k < ticks and deploys[k]:  # baseline windows [tk - W, tk] of this tick's old pods
            bt0 = tk - W * STEP
            for j, m in enumerate(METRICS):
                pods = [(i, pod) for i in deploys[k] for pod in old_pods(i, k)]
                rows = np.array([i * M + j for i, _ in pods])
                base = model[rows, c - W:c + 1] + rng.standard_normal((len(pods), W + 1)) * noise[rows][:, None]
                server.windows[("namespace_pod:" + m, bt0)] = (
                    {pod: n for n, (_, pod) in enumerate(pods)},
                    [f'"__name__":"namespace_pod:{m}","namespace":"{ns[i]}","pod":"{pod}"' for i, pod in pods],
                    base.astype(np.float32))
    del model
    setup_s = time.perf_counter() - t_setup

    stream = StreamingMonitor(store, cfg, prom=server, device=dev, worker_id=f"node-m{rank}", ring_len=R,
                              window=W, clock=lambda: clock["t"])
    ew = node_world(world, rank, dev)
    node = NodeBrain(stream, ew, store, dev, publish=False, extra=(roll,))
    node.owns = lambda d: True  # the rank-local store holds exactly this rank's share
    for mon in node.monitors:
        mon.owns = None
    _start_node(node, ew)
    loop = asyncio.new_event_loop()
    flagged: set = set()
    scored: List[int] = []
    breakdowns: List[Dict[str, float]] = []
    gc_pause = {"t": 0.0, "t0": 0.0, "n": 0}

    def _gc_cb(phase, info):
        if phase == "start":
            gc_pause["t0"] = time.perf_counter()
        else:
            gc_pause["t"] += time.perf_counter() - gc_pause["t0"]
            gc_pause["n"] += 1

    arrived = {"next": 0}   # first tick whose arrivals have not reached the store

    def arrive(k):
        """This minute's rollout requests reach the job store (the service wrote them)."""
        if k >= len(arrivals) or k < arrived["next"]:
            return
        for d in arrivals[k]:
            store._docs[d["id"]] = d
            store._index(d)
        arrived["next"] = k + 1

    def tick(k):
        clock["t"] = T0 + STEP * k
        arrive(k)
        n_rows = roll.n_live
        gc_pause["t"], gc_pause["n"] = 0.0, 0
        gc.callbacks.append(_gc_cb)
        serve0, st0, sw0 = server.serve_s, server.serve_tick_s, server.serve_window_s
        t0 = time.perf_counter()
        try:
            table = loop.run_until_complete(node.tick())
        finally:
            gc.callbacks.remove(_gc_cb)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        scored.append(n_rows)
        bd = {kk: round(v, 3) for kk, v in roll.timings.items()}
        bd.update({kk: round(v, 3) for kk, v in node.timings.items()})
        bd["tick_total_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        bd["prometheus_standin_ms"] = round((server.serve_s - serve0) * 1e3, 3)
        # the stand-in runs inside this process: the brain's own time is the phase minus its share
        st_ms, sw_ms = (server.serve_tick_s - st0) * 1e3, (server.serve_window_s - sw0) * 1e3
        if "detect_ms" in bd:
            bd["detect_net_ms"] = round(bd["detect_ms"] - st_ms, 3)
        if "intake_ms" in bd:
            bd["intake_net_ms"] = round(bd["intake_ms"] - sw_ms, 3)
        bd["tick_net_ms"] = round(bd["tick_total_ms"] - st_ms - sw_ms, 3)
        bd["live_rows"] = roll.n_live
        bd["gc_ms"], bd["gc_runs"] = round(gc_pause["t"] * 1e3, 2), gc_pause["n"]
        _exchange_bd(node, bd)
        breakdowns.append(bd)
        for a in table["anomalous_apps"]:
            flagged.add(a)
        return table

    def finish():
        """Completion ticks: the arrivals of the minutes the timed loop did not reach
        are delivered (round 4 counted the last minute's 2,000 jobs, never delivered,
        as misses: all 97 "FN" of ``arrival_r4_k.json``), then every job runs past its
        endTime; detection over every job, with each miss described."""
        t0 = time.perf_counter()
        for k in range(arrived["next"], ticks + W + 1):
            clock["t"] = T0 + STEP * k
            arrive(k)
            loop.run_until_complete(node.tick())
        fin = time.perf_counter() - t0
        st: Dict[str, int] = {}
        tp = fp = fn = 0
        misses = []
        for jid, bad in truth.items():
            d = store._docs.get(jid)
            s = d["status"] if d is not None else "never-arrived"
            st[s] = st.get(s, 0) + 1
            hit = s == r.ST_COMPLETED_UNHEALTH
            tp += bad and hit
            fp += (not bad) and hit
            fn += bad and not hit
            if bad and not hit and len(misses) < 50:
                misses.append({"job": jid[:12], "status": s, "reason": (d or {}).get("reason", ""),
                               "start": (d or {}).get("startTime"), "app": (d or {}).get("appName")})
        return fin, st, {"jobs": len(truth), "injected_jobs": sum(truth.values()), "tp": tp, "fp": fp, "fn": fn,
                         "recall": round(tp / max(1, tp + fn), 4), "false_positive_rate":
                         round(fp / max(1, len(truth) - sum(truth.values())), 6), "misses": misses}

    health = torch.zeros((1, 2), dtype=torch.int32)
    meta = {
        "model": f"{args.algorithm} + pairwise {args.pairwise} canary jobs on the production node brain, steady "
                 f"arrivals ({J} rollouts per minute, {W}-minute watch)",
        "global_batch": J * W * M * world,
        "seq_len": R,
        "season": season,
        "arrivals_per_tick": J,
        "watch_window_min": W,
        "metrics_per_job": M,
        "pods_new_old": [P, P],
        "app_pool": A_all,
        "path": "per tick: score running jobs (pod windows as query_range JSON -> native decode "
                "-> H2D -> scatter -> rank tests -> cached-state band/verdict -> D2H -> fail-fast writes) "
                "-> node health exchange [detect latency] -> endTime writes + row release, history advance, "
                "claim + native job decode + admission (rows, slots, HW fit of the new rows, baseline windows) "
                "of this minute's arrivals",
        "warm_node": "resident 7-day history of every (app, metric) in HBM",
        "setup_s": round(setup_s, 2),
        "register_s": round(register_s, 3),
        "register_jobs_per_s": round(sum(len(a) for a in arrivals) / max(register_s, 1e-9), 1),
        "jobs_to_brainworker": _brainworker_share([d for a in arrivals for d in a], cfg),
        "_scored_rows": scored,
        "_breakdowns": breakdowns,
        "_arrival_finish": finish,
        "_roll": roll,
        "_server": server,
    }
    return tick, health, meta, "bf16" if dev.type == "cuda" else "fp32", J * W * M


def setup_node_lstm(args, world, rank, dev):
    """``--config node-lstm``: BASELINE configs 3 / 5 through the product path.
    Continuous multi-metric jobs (``--lstm-features F`` metrics each: 5 = the design
    doc's 3+-metric LSTM dispatch over 100k series; 2 = config 5's latency +
    error-rate entities) are registered through the service's create handler and
    scored by the production node brain: ``NodeBrain`` + :class:`LstmMonitor` — the
    resident 7-day history of every (app, metric) advanced each tick from
    ``query_range`` JSON (native decode), one data-parallel Adam step of the node's
    shared LSTM autoencoder, calibration of joining entities, fused MFMA scoring of
    every entity's newest window, fail-fast verdicts into the job store.  A fresh
    node pretrains the model over the warmup ticks (``FOREMAST_LSTM_PRETRAIN`` steps,
    ``FOREMAST_LSTM_PRETRAIN_PER_TICK`` per tick), as in production.  ``--anomaly-frac``
    of the jobs triple every metric two minutes into the timed ticks."""
    from ..api import rest as r
    from ..brain.engine import synthetic_eval, synthetic_params
    from ..brain.lstm_monitor import LstmMonitor
    from ..brain.node import NodeBrain, owner_of
    from ..brain.resident import ResidentHistory
    from ..brain.streaming import StreamingMonitor
    from ..ingest import native
    from ..service import app as svc
    from ..store import MemoryJobStore
    from ..utils.config import BrainConfig, reference_default_env
    from ..utils.timeutil import format_rfc3339

    F = max(2, int(args.lstm_features))
    mets = METRICS[:F]
    R, season = args.ring, args.season
    n_jobs = max(1, args.series // F)
    if dev.type == "cpu" and not os.environ.get("FOREMAST_BENCH_CPU_FULL"):
        n_jobs, R, season = min(n_jobs, 64), min(R, 2880), min(season, 1440)
    pre = int(os.environ.get("FOREMAST_LSTM_PRETRAIN", "800" if dev.type == "cuda" else "20"))
    per = int(os.environ.get("FOREMAST_LSTM_PRETRAIN_PER_TICK", "100" if dev.type == "cuda" else "20"))
    ticks = args.warmup + args.steps + 1
    mine = [a for a in range(n_jobs) if owner_of(f"ns{a % 200}", f"app{a}", world) == rank]
    na = len(mine)
    clock = {"t": T0}
    t_setup = time.perf_counter()
    env = reference_default_env()
    env.update(ML_ALGORITHM="lstm", ML_LSTM_THRESHOLD=str(args.lstm_threshold),
               FOREMAST_LSTM_LEVEL_THRESHOLD=str(args.lstm_level_threshold), FOREMAST_LSTM_WINDOW=str(args.lstm_window))
    cfg = BrainConfig.from_env(env)
    cfg.ring_len, cfg.season = R, season
    store = MemoryJobStore()
    server = ArrivalServer()
    ns = [f"ns{a % 200}" for a in mine]
    app = [f"app{a}" for a in mine]
    # every job's F series: synthetic seasonal weeks (the history the node holds), continued by the ticks
    gid = torch.tensor([a * F + j for a in mine for j in range(F)], dtype=torch.int64)
    params = {k: v[gid] for k, v in synthetic_params(n_jobs * F, torch.device("cpu"), seed=4321).items()}
    hist = ResidentHistory(server, dev, R, STEP, clock=lambda: clock["t"], decode_threads=args.decode_threads)
    keys = [(ENDPOINT, "namespace_app_per_pod:" + m, ns[i], app[i]) for i in range(na) for m in mets]
    hist.want(keys, T0)
    asyncio.run(hist.assign_only(T0))
    dparams = {k: v.to(dev) for k, v in params.items()}
    for c0 in range(0, len(keys), 16384):
        c1 = min(len(keys), c0 + 16384)
        hist.load_rows(keys[c0:c1], synthetic_eval({k: v[c0:c1] for k, v in dparams.items()}, 0, R, season,
                                                   noise_seed=77 + c0))
    hist.unwant(keys, T0)
    # per-tick bodies: the newest minute of every (app, metric); injected jobs x3 from tick `at`
    rng = np.random.default_rng(5 + rank)
    n_bad = int(round(args.anomaly_frac * na))
    bad = set(rng.choice(na, size=n_bad, replace=False).tolist()) if n_bad else set()
    at = args.warmup + 2
    cont = synthetic_eval(params, R, ticks + 2, season, None).numpy()          # [na * F, ticks] no noise
    noise = 0.03 * params["lvl"][:, 0].numpy()
    badm = np.zeros(na * F, dtype=bool)
    for i in bad:
        badm[i * F:(i + 1) * F] = True
    labels = {m: native.label_blob([f'"__name__":"namespace_app_per_pod:{m}","namespace":"{ns[i]}","app":"{app[i]}"'
                                    for i in range(na)]) for m in mets}
    for k in range(ticks + 1):
        tk = T0 + STEP * k
        v = cont[:, k] + rng.standard_normal(na * F) * noise
        if k >= at:
            v = np.where(badm, v * 3.0, v)
        v = v.astype(np.float32).reshape(na, F)
        for j, m in enumerate(mets):
            server.tick_bodies[("namespace_app_per_pod:" + m, tk)] = native.render_matrix(labels[m], v[:, j:j + 1],
                                                                                          tk, STEP)
    del cont
    # --- jobs through the service: continuous, F metrics each -------------------------------------
    truth: Dict[str, bool] = {}
    t_reg = time.perf_counter()
    for i in range(na):
        cur, hst = {}, {}
        for m in mets:
            q = f'namespace_app_per_pod:{m}{{namespace="{ns[i]}",app="{app[i]}"}}'
            p = {"endpoint": ENDPOINT, "query": q, "step": int(STEP)}
            cur[m] = {"dataSourceType": "prometheus", "parameters": dict(p, start=int(T0), end=int(T0 + 86400))}
            hst[m] = {"dataSourceType": "prometheus", "parameters": dict(p, start=int(T0 - 7 * 86400), end=int(T0))}
        code, resp = svc.register(store, {"appName": app[i], "startTime": format_rfc3339(T0),
                                          "endTime": format_rfc3339(T0 + 86400), "strategy": "continuous",
                                          "metrics": {"current": cur, "historical": hst}})
        assert code == 200, resp
        truth[resp["jobId"]] = i in bad
    register_s = time.perf_counter() - t_reg
    prec = getattr(args, "lstm_precision", "auto")
    fp8 = prec == "fp8" or (prec == "auto" and F == 2)   # config 5: fp8 on the CDNA4 block-scaled MFMA
    lstm = LstmMonitor(store, cfg, prom=server, device=dev, worker_id=f"node-m{rank}-lstm", step=STEP,
                       clock=lambda: clock["t"], ring_len=R, features=F, window=args.lstm_window,
                       train_batch=args.lstm_train_batch, min_capacity=max(64, na), history=hist,
                       decode_threads=args.decode_threads, fp8=fp8)
    stream = StreamingMonitor(store, cfg, prom=server, device=dev, worker_id=f"node-m{rank}", ring_len=R,
                              window=10, clock=lambda: clock["t"])
    stream.exclude = lstm.is_mine
    ew = node_world(world, rank, dev)
    node = NodeBrain(stream, ew, store, dev, publish=False, extra=(lstm,))
    node.owns = lambda d: True
    for mon in node.monitors:
        mon.owns = None
    _start_node(node, ew)
    loop = asyncio.new_event_loop()
    setup_s = time.perf_counter() - t_setup
    breakdowns: List[Dict[str, float]] = []
    scored: List[int] = []

    gc_pause = {"t": 0.0, "t0": 0.0, "n": 0}

    def _gc_cb(phase, info):  # cyclic-GC pauses inside a tick
        if phase == "start":
            gc_pause["t0"] = time.perf_counter()
        else:
            gc_pause["t"] += time.perf_counter() - gc_pause["t0"]
            gc_pause["n"] += 1

    def _mem():
        if dev.type != "cuda":
            return 0, 0
        ms = torch.cuda.memory_stats(dev)
        return int(ms.get("segment.all.allocated", 0)), int(ms.get("num_alloc_retries", 0))

    def tick(k):
        clock["t"] = T0 + STEP * k
        n_live = lstm._n_series
        seg0, retry0 = _mem()
        gc_pause["t"], gc_pause["n"] = 0.0, 0
        st0 = lstm.shard.ticks
        t0 = time.perf_counter()
        gc.callbacks.append(_gc_cb)
        try:
            loop.run_until_complete(node.tick())
        finally:
            gc.callbacks.remove(_gc_cb)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        bd = {kk: round(v, 3) for kk, v in lstm.timings.items()}
        bd.update({kk: round(v, 3) for kk, v in node.timings.items()})
        bd["tick_total_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        bd["entities"] = len(lstm.jobs)
        # what a slow tick did besides the steady-state work (the tail attribution below)
        seg1, retry1 = _mem()
        re = lstm.shard.restat_every
        bd["restat"] = any((t + 1) % re == 0 for t in range(st0, lstm.shard.ticks)) if re else False
        bd["gc_ms"], bd["gc_runs"] = round(gc_pause["t"] * 1e3, 2), gc_pause["n"]
        bd["hip_mallocs"], bd["alloc_retries"] = seg1 - seg0, retry1 - retry0
        _exchange_bd(node, bd)
        breakdowns.append(bd)
        scored.append(n_live)

    def finish():
        st: Dict[str, int] = {}
        tp = fp = fn = 0
        for jid, b in truth.items():
            s = store._docs[jid]["status"]
            st[s] = st.get(s, 0) + 1
            hit = s == r.ST_COMPLETED_UNHEALTH
            tp += b and hit
            fp += (not b) and hit
            fn += b and not hit
        return 0.0, st, {"jobs": len(truth), "injected_jobs": sum(truth.values()), "tp": tp, "fp": fp, "fn": fn,
                         "recall": round(tp / max(1, tp + fn), 4),
                         "false_positive_rate": round(fp / max(1, len(truth) - sum(truth.values())), 6)}

    meta = {
        "model": f"continuous {F}-metric jobs on the production node brain: NodeBrain + LstmMonitor (shared LSTM "
                 f"autoencoder F={F}, H={lstm.shard.model.H}, window {args.lstm_window}, one DP Adam step per tick, "
                 f"fused {'fp8 block-scaled (v_mfma_scale_f32_32x32x64_f8f6f4)' if lstm.shard.fp8 else 'bf16'} "
                 f"MFMA scoring)",
        "global_batch": n_jobs * F,
        "seq_len": args.lstm_window,
        "history": R,
        "entities": n_jobs,
        "features": F,
        "path": "service.register (continuous) -> claim -> resident 7-day history -> per tick: query_range JSON of "
                "every (app, metric) -> native decode -> ring append -> DP train step -> fused scoring -> verdicts",
        "pretrain_steps": pre, "pretrain_per_tick": per,
        "warm_node": "resident 7-day history of every (app, metric) in HBM before the jobs arrive",
        "setup_s": round(setup_s, 2),
        "register_s": round(register_s, 3),
        "jobs_to_brainworker": _brainworker_share(list(store._docs.values()), cfg),
        "_scored_rows": scored,
        "_breakdowns": breakdowns,
        "_arrival_finish": finish,
    }
    dt = ("fp8_e4m3" if lstm.shard.fp8 else "bf16") if dev.type == "cuda" else "fp32"
    return tick, torch.zeros((1, 2), dtype=torch.int32), meta, dt, n_jobs * F
