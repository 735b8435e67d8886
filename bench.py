#!/usr/bin/env python
"""Headline benchmark: metric-series scored/sec (whole node) + p50 detect
latency on the 100k-series canary (BASELINE.json).

One scoring tick = the full canary pipeline for every series of the job:

  1. ingest: this tick's canary-pod and baseline-pod points arrive in pinned
     host memory (as the Prometheus ingest would deliver them), are copied
     H2D and streamed into the HBM rings (K10: new points in, oldest current
     points graduate into the sliding 7-day history);
  2. pairwise canary test: baseline vs current Mann-Whitney U + Wilcoxon +
     Kruskal (ML_PAIRWISE_ALGORITHM=ALL), per series (K5/K11);
  3. model: additive Holt-Winters (daily season, 60 s step, 7-day window =
     10,080 points) refit from scratch on the slid window over a 64-point
     alpha/beta/gamma grid, forecast of the 50 current points, band,
     anomalies, verdict, per-app counters — one fused launch (K3 + K9);
  4. cluster aggregation: per-app counters all-reduced and verdicts
     all-gathered over RCCL/xGMI (RC1 + RC2);
  5. the aggregated health table is copied back to the host — the verdict
     is "available" and the tick's detect latency stops here.

Nothing is cached across ticks: every tick refits every model on new data.
Strong scaling: the 100k series are sharded over the ranks.

Other BASELINE configs (same metric/JSON contract, ``--config``):

* ``lstm`` (config 3): 100k univariate series, LSTM autoencoder; every tick
  runs one DP Adam step (gradient all-reduce over RCCL) and re-scores every
  series' latest window with the fused MFMA kernel;
* ``multivariate`` (config 5): 50k entities x (latency, error-rate) = 100k
  metric-series, LSTM-AE scored with fp8 e4m3 MFMA.

Usage: ``python bench.py --gpus N --steps K --warmup W``.  With N > 1 and no
launcher the script starts its own ``torch.distributed.run`` group of N ranks
(one per GPU, RCCL); under a launcher it checks WORLD_SIZE == N.  Rank 0 prints
ONE JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import NamedTuple

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from foremast_amd.brain.engine import (ShardSpec, StreamingShard, global_randn, synthetic_eval,  # noqa: E402
                                       synthetic_history, synthetic_params)
from foremast_amd.parallel import comm  # noqa: E402
from foremast_amd.parallel.health import HealthAggregator, shard_range  # noqa: E402
from foremast_amd.utils.config import BrainConfig  # noqa: E402

METRIC = "metric-series scored/sec (whole node) + p50 detect latency, 100k-series canary"
# The reference publishes no number (BASELINE.json "published": {}).  vs_baseline is
# measured against this repo's CPU re-creation of the reference brain's design: the
# same scorer as a per-series numpy/scipy loop on ONE core (bench.py --config
# cpu_baseline, models/cpu_baseline.py; BASELINE.md "CPU per-series baseline").
CPU_BASELINE_SERIES_PER_S = {"canary": 16.08, "hw10k": 16.08, "lstm": 256.4, "multivariate": 418.6}
METRICS_PER_APP = 5


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed ticks (default 20; node: 8)")
    p.add_argument("--warmup", type=int, default=None, help="untimed ticks (default 5; node: 1)")
    p.add_argument("--series", type=int, default=100_000)
    p.add_argument("--ring", type=int, default=10080)
    p.add_argument("--season", type=int, default=1440)
    p.add_argument("--pods", type=int, default=5)
    p.add_argument("--window", type=int, default=10)
    p.add_argument("--algorithm", default="holt_winters")
    p.add_argument("--pairwise", default="ALL")
    p.add_argument("--pairwise-shift", type=float, default=None,
                   help="canary: mean-shift rule threshold in sigmas (ML_PAIRWISE_SHIFT; 0 = off; "
                        "default: the BrainConfig default)")
    p.add_argument("--pairwise-shift-spread", choices=["one-step", "horizon"], default=None,
                   help="canary: the mean-shift rule's spread (ML_PAIRWISE_SHIFT_ONE_STEP; default: the "
                        "BrainConfig default, one-step)")
    p.add_argument("--anomaly-frac", type=float, default=0.01)
    p.add_argument("--anomaly-kind", default="scale3", choices=["scale3", "shift3sigma", "scale", "shift"],
                   help="injected canary regression: values x3, or a level shift of +3 noise sigma; "
                        "scale / shift take their size from --anomaly-size")
    p.add_argument("--anomaly-size", type=float, default=3.0,
                   help="scale: values multiplied by this; shift: level shift in noise sigmas")
    p.add_argument("--gap-frac", type=float, default=0.0,
                   help="canary: fraction of series whose 7-day history has a 30-minute scrape outage (NaN run) "
                        "after the first season (production-like gaps; those series take the masked kernels)")
    p.add_argument("--miss-rate", type=float, default=0.0,
                   help="canary: probability of an isolated missed scrape per history point (NaN; e.g. 1e-3 = "
                        "~10 per series-week); gapped series pairs take the masked-season Holt-Winters kernel")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--graph", dest="graph", action="store_true", default=True,
                   help="(default) canary: the GPU part of a steady-state tick (ring advance, ingest, rank tests, "
                        "fit, deferred detect) is one HIP-graph replay; the host only copies the health table "
                        "back and waits. Falls back to eager launches where the shard cannot be captured")
    p.add_argument("--eager", dest="graph", action="store_false",
                   help="canary: launch every kernel of a tick from Python (no HIP graph)")
    p.add_argument("--pipeline", action="store_true",
                   help="canary: enqueue tick k+1 before waiting for tick k's health table (the GPU never idles on "
                        "the host; detect latency then includes the queueing behind the previous tick). Measured "
                        "+3%% series/s at 12.5k series per GPU for 2x the p50 latency, so it is off by default")
    p.add_argument("--refit-every", type=int, default=1,
                   help="Holt-Winters model cache: full 64-point grid refit every K ticks, O(1) state update + "
                        "detect in between (1 = refit every tick: the headline)")
    p.add_argument("--ingest", default="pinned", choices=["pinned", "prom"],
                   help="pinned: a tick's points arrive decoded in pinned memory; prom: they arrive as "
                        "Prometheus query_range JSON bodies (one per metric family and canary/baseline pod "
                        "set), decoded in the timed tick by the native keyed parser on a thread pool, "
                        "double-buffered so tick k+1 decodes while the GPU scores tick k")
    p.add_argument("--decode-threads", type=int, default=16)
    p.add_argument("--zero-copy", action="store_true",
                   help="pinned ingest: the ingest kernel reads each tick's points straight from pinned host "
                        "memory and a kernel writes the health table into pinned host memory (no H2D / D2H "
                        "memcpy operations in the tick); measured neutral on one MI355X (12.5k series: 1.435-1.451 "
                        "vs 1.436-1.445 ms; 100k: 10.54 vs 10.57 ms), so off by default")
    p.add_argument("--prefetch", action="store_true",
                   help="pinned ingest: prefetch tick k+1's points H2D on a copy stream during tick k "
                        "(double-buffered) instead of copying them on the main stream at the start of the tick; "
                        "measured neutral at 12.5k series per GPU (1.458 vs 1.436 ms), so off by default")
    p.add_argument("--graph-prefetch", dest="graph_prefetch", action="store_true", default=True,
                   help="(default) canary graph ticks: the points of tick k+1 are copied H2D on a copy stream into "
                        "the second of two input buffers (one captured graph each) while tick k runs, so a tick "
                        "starts with its input on the device; the tick itself is never queued behind the previous")
    p.add_argument("--no-graph-prefetch", dest="graph_prefetch", action="store_false")
    p.add_argument("--doorbell", dest="doorbell", action="store_true", default=False,
                   help="canary graph ticks: tick k+1's graph is enqueued (with its input copy) while tick k runs "
                        "and starts by waiting for a doorbell, a pinned host counter the host bumps when it releases "
                        "the tick after tick k's results are in: the gap between ticks is a PCIe write instead of "
                        "a graph launch; the detect latency is timed from the doorbell")
    p.add_argument("--no-doorbell", dest="doorbell", action="store_false")
    p.add_argument("--spin-wait", dest="spin_wait", action="store_true", default=False,
                   help="canary: wait for a tick's completion by polling its event instead of a blocking stream "
                        "synchronize (shorter host wake-up between ticks)")
    p.add_argument("--overlap-pairwise", action="store_true",
                   help="run the rank tests on a side stream beside the fit at any shard size (the default from "
                        "16,384 series per rank, engine.OVERLAP_MIN_SERIES)")
    p.add_argument("--serial-pairwise", action="store_true",
                   help="run the rank tests on the main stream before the fit (fused detect epilogue) "
                        "instead of on a side stream concurrently with it")
    p.add_argument("--cpu", action="store_true", help="force CPU (reference path; tiny sizes only)")
    p.add_argument("--baseline-sample", type=int, default=48,
                   help="cpu_baseline: series scored by the per-series CPU loop (the rate is per core)")
    p.add_argument("--baseline-model", default="canary", choices=["canary", "lstm", "multivariate"],
                   help="cpu_baseline: which GPU config's scorer the per-series CPU loop re-creates")
    p.add_argument("--config", default="canary",
                   choices=["canary", "single", "hw10k", "lstm", "multivariate", "cpu_baseline", "node", "node-lstm"],
                   help="canary = headline (BASELINE configs 2/4 at 100k); single = config 1 (one latency "
                        "series, moving average, CPU brain plumbing end to end); hw10k = config 2 (10k series); "
                        "lstm = config 3; multivariate = config 5 (fp8 LSTM, latency + error-rate); node = the product "
                        "path: canary jobs registered through the service and scored by the production node brain "
                        "from Prometheus JSON (foremast_amd/benchmarks/node.py)")
    p.add_argument("--cold", action="store_true",
                   help="node config: a cold node -- only --cold-warm-jobs apps are resident; the week of every other "
                        "(app, metric) loads from Prometheus JSON through the node's history path, within "
                        "--cold-budget-s per tick, while the warm jobs keep scoring (record under config.cold)")
    p.add_argument("--cold-warm-jobs", type=int, default=2000)
    p.add_argument("--cold-budget-s", type=float, default=2.0)
    p.add_argument("--arrival-per-tick", type=int, default=0,
                   help="node config: steady arrivals -- this many canary rollouts start every minute and finish at "
                        "endTime (--window minutes later); ~J x window jobs live at steady state "
                        "(foremast_amd/benchmarks/node.py setup_arrival)")
    p.add_argument("--multi-cluster", action="store_true",
                   help="config 4 layout: each rank scrapes the baseline cluster of its neighbour's shard; "
                        "baseline windows reach their owner through one RCCL all-to-all per tick")
    p.add_argument("--lstm-window", type=int, default=32)
    p.add_argument("--lstm-features", type=int, default=5,
                   help="node-lstm config: metrics per continuous job (5: the 3+-metric LSTM dispatch over --series "
                        "series = config 3 through the product; 2: latency + error-rate entities = config 5)")
    p.add_argument("--lstm-train-batch", type=int, default=4096)
    p.add_argument("--lstm-train-every", type=int, default=1)
    p.add_argument("--lstm-pretrain", type=int, default=800,
                   help="DP training steps of model initialisation before the timed ticks (untimed)")
    p.add_argument("--lstm-restat-every", type=int, default=16,
                   help="ticks between refreshes of the per-series normalisation statistics (window_stats over the ring)")
    p.add_argument("--lstm-autograd", action="store_true", help="train with autograd instead of the fused K7 kernel")
    p.add_argument("--lstm-threshold", type=float, default=5.0,
                   help="AE reconstruction z threshold (5: the level term carries the small shifts)")
    p.add_argument("--mv-bf16", action="store_true", help="multivariate config: bf16 scoring instead of fp8")
    p.add_argument("--lstm-precision", default="auto", choices=["auto", "bf16", "fp8"],
                   help="node-lstm scoring precision; auto: fp8 (CDNA4 block-scaled MFMA) for the 2-feature "
                        "config 5 (BASELINE.json: 'fp8 LSTM on CDNA4 MFMA'), bf16 otherwise")
    p.add_argument("--lstm-cal-ewma", type=float, default=1.0 / 32,
                   help="per-series calibration refresh rate of healthy windows")
    p.add_argument("--lstm-level-threshold", type=float, default=5.5,
                   help="level-term |z| threshold (<= 0: no level term)")
    p.add_argument("--lstm-no-overlap", action="store_true",
                   help="run the training step and scoring back to back instead of on two HIP streams")
    a = p.parse_args()
    if a.steps is None:
        a.steps = (100 if a.arrival_per_tick else 8) if a.config == "node" else 20
    if a.warmup is None:
        a.warmup = (a.window + 1 if a.arrival_per_tick else 1) if a.config == "node" else 5
        if a.config == "node-lstm":  # a fresh node pretrains its shared model over the warmup ticks
            import os as _os
            gpu = not a.cpu
            pre = int(_os.environ.get("FOREMAST_LSTM_PRETRAIN", "800" if gpu else "20"))
            per = int(_os.environ.get("FOREMAST_LSTM_PRETRAIN_PER_TICK", "100" if gpu else "20"))
            a.warmup = -(-pre // max(1, per)) + 2
    if a.zero_copy or a.prefetch:
        a.graph = False  # these modes stage the tick's I/O from the host: eager launches
    return a


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(args, argv) -> int:
    """``--gpus N`` without a launcher: start N ranks (one per GPU) as ONE child
    ``torch.distributed.run`` process group and forward its exit code.

    Runs before this process touches the GPU (no HIP call, no
    ``torch.cuda.is_available()``): the parent only waits; rank 0's JSON line
    reaches stdout through the inherited file descriptors."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


P99_MIN = 100   # samples below which a p99 is not reported (the max is)


def _sum_detection(parts) -> dict:
    """Detection records of every rank summed into the node's."""
    out = {k: sum(p[k] for p in parts) for k in ("jobs", "injected_jobs", "tp", "fp", "fn")}
    out["recall"] = round(out["tp"] / max(1, out["tp"] + out["fn"]), 4)
    out["false_positive_rate"] = round(out["fp"] / max(1, out["jobs"] - out["injected_jobs"]), 6)
    out["misses"] = [m for p in parts for m in p.get("misses", [])][:50]
    out["ranks"] = len(parts)
    return out


def _exchange_summary(bds, steps: int, world: int, config: str) -> dict:
    """The node health exchange over the timed ticks (rank 0's view): deployed path
    (ElasticWorld under N ranks), generation, collective time, roster bytes."""
    xs = [b for b in bds[-steps:] if "exchange_ms" in b]
    ms = [b["exchange_ms"] for b in xs]
    by = [b["roster_bytes"] for b in xs]

    def q(v, p):
        if not v or (p == 99 and len(v) < P99_MIN):
            return None
        return round(float(np.percentile(v, p)), 3)
    return {"path": "ElasticWorld run_tick + ClusterHealth roster deltas" if world > 1 or comm.force_collectives()
            else "single rank (no collectives)", "ranks": world,
            "generation": max((b.get("generation", 0) for b in xs), default=0),
            "exchange_ms_p50_p99_max": [q(ms, 50), q(ms, 99), q(ms, 100)],
            "roster_bytes_p50_max": [q(by, 50), q(by, 100)], "samples": len(xs)}


def _tail_attribution(bds, factor: float = 2.5) -> dict:
    """Ticks slower than ``factor`` x the p50 tick, each with what it did besides the
    steady-state work: a statistics refresh (window_stats over every ring), cyclic-GC
    pauses, new device segments from the caching allocator (hipMalloc) or allocator
    retries, verdict writes, the node exchange."""
    tt = [b.get("tick_total_ms") for b in bds if b.get("tick_total_ms") is not None]
    if not tt:
        return {}
    p50 = float(np.percentile(tt, 50))
    out = []
    for i, b in enumerate(bds):
        t = b.get("tick_total_ms")
        if t is None or t <= factor * p50:
            continue
        why = []
        if b.get("restat"):
            why.append("restat")
        if b.get("gc_ms", 0) > 0.2 * (t - p50):
            why.append(f"gc {b['gc_ms']} ms")
        if b.get("hip_mallocs", 0) or b.get("alloc_retries", 0):
            why.append(f"allocator ({b.get('hip_mallocs', 0)} new segments, {b.get('alloc_retries', 0)} retries)")
        if b.get("exchange_ms", 0) > 0.2 * (t - p50):
            why.append(f"exchange {b['exchange_ms']} ms")
        nw = int(b.get("verdicts_written", 0))
        if nw >= 20:  # a burst of fail-fast / endTime writes to the job store
            why.append(f"{nw} verdict writes")
        out.append({"tick": i, "ms": t, "x_p50": round(t / p50, 2), "causes": why or ["unattributed"],
                    **{k: b[k] for k in ("intake_ms", "tick_ms", "gc_ms") if k in b}})
    return {"p50_ms": round(p50, 3), "max_ms": round(max(tt), 3), "max_over_p50": round(max(tt) / p50, 2),
            "threshold_x_p50": factor, "outliers": out, "samples": len(tt)}


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and not args.cpu
    if use_gpu:
        local = local % max(1, torch.cuda.device_count())  # >1 rank per GPU only in gloo tests
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if args.config in ("node", "node-lstm"):
        # the product configs join the node as a deployed rank does: an ElasticWorld on the
        # launcher's store forms the process group (benchmarks/node.py node_world)
        return world, rank, dev
    # FOREMAST_FORCE_COLLECTIVES=1 (tests/test_rccl_gpu.py): a 1-rank group that still runs
    # every collective, so one GPU exercises the RCCL path of the N-GPU tick
    if world > 1 or comm.force_collectives():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("FOREMAST_DIST_BACKEND", "nccl" if use_gpu else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:
            dist.init_process_group(backend)  # gloo: CPU runs, or several ranks sharing one GPU in tests
    return world, rank, dev


def barrier(dev):
    if dist.is_initialized():
        if dev.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()


NOISE = 0.03  # synthetic noise sigma as a fraction of the level (engine.synthetic_eval default)


def make_ticks(params, pods, nticks, season, t0, seed, anomaly_frac, kind="scale3", want_bad=False, size=3.0,
               row0=0, n_global=None):
    """Per-tick per-pod values ``[nticks, n, pods]`` continuing each series'
    synthetic model past the history (same noise level as the history), with a
    fraction of series turned anomalous: ``scale3`` (canary regression, values
    x3) or ``shift3sigma`` (level shift of +3 noise sigma); ``scale`` / ``shift``
    use ``size`` instead of 3.  ``want_bad``: also return the regressed series'
    LOCAL indices (detection-quality ground truth).  ``row0`` / ``n_global``: the
    local series are global ``row0 ..`` of ``n_global``; noise and the regressed
    set are functions of the global index, so every sharding scores the same data."""
    lvl = params["lvl"]
    n, dev = lvl.shape[0], lvl.device
    n_global = n if n_global is None else n_global
    vals = synthetic_eval(params, t0, nticks, season, None).T.contiguous()  # [nticks, n]
    eps = global_randn(lambda r: (nticks, r, pods), n, row0, seed + 17, dev, dim=1)
    out = vals[..., None] + eps * (NOISE * lvl[:, 0])[None, :, None]
    n_bad = int(n_global * anomaly_frac)
    bad = torch.zeros(0, dtype=torch.int64, device=dev)
    if n_bad:
        g = torch.Generator().manual_seed(seed + 17)
        gbad = torch.randperm(n_global, generator=g)[:n_bad]
        bad = (gbad[(gbad >= row0) & (gbad < row0 + n)] - row0).to(dev)
        k = 3.0 if kind in ("scale3", "shift3sigma") else float(size)
        if kind.startswith("scale"):
            out[:, bad, :] *= k
        else:
            out[:, bad, :] += (k * NOISE * lvl[bad, 0])[None, :, None]
    return (out.float(), bad) if want_bad else out.float()


def detection_report(table: torch.Tensor, truth_apps, n_apps: int) -> dict:
    """Per-app detection quality of the last tick against the injected ground
    truth: an app is flagged when any of its series is anomalous."""
    flagged = (table[:n_apps, 0] > 0).numpy()
    truth = np.zeros(n_apps, dtype=bool)
    truth[np.asarray(sorted(truth_apps), dtype=np.int64)] = True
    tp = int((flagged & truth).sum())
    fp = int((flagged & ~truth).sum())
    fn = int((~flagged & truth).sum())
    healthy = int((~truth).sum())
    return {"apps": n_apps, "injected_apps": int(truth.sum()), "tp": tp, "fp": fp, "fn": fn,
            "precision": round(tp / max(tp + fp, 1), 4), "recall": round(tp / max(tp + fn, 1), 4) if truth.any() else None,
            "false_positive_rate": round(fp / max(healthy, 1), 5)}


def setup_canary(args, world, rank, dev):
    """Config 4 / headline: HW + pairwise canary scorer over the sharded 100k series."""
    if dev.type == "cpu" and args.series > 4096:
        # the CPU path is the reference implementation: keep it small
        args.series, args.ring, args.season = 256, 480, 48
    cfg = BrainConfig()
    cfg.min_historical_points = 0
    if args.pairwise_shift is not None:
        cfg.pairwise_shift = args.pairwise_shift
    if args.pairwise_shift_spread is not None:
        cfg.pairwise_shift_one_step = args.pairwise_shift_spread == "one-step"
    s, e, per = shard_range(args.series, world, rank, align=METRICS_PER_APP)
    n_local = e - s
    n_apps = (args.series + METRICS_PER_APP - 1) // METRICS_PER_APP
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    spec = ShardSpec(n_series=n_local, ring_len=args.ring, season=args.season, pods=args.pods,
                     window=args.window, algorithm=args.algorithm, pairwise=args.pairwise,
                     dtype=dtype, n_apps=n_apps, refit_every=args.refit_every)
    app_id = (torch.arange(s, e, device=dev, dtype=torch.int64) // METRICS_PER_APP).to(torch.int32)
    # shards are app-aligned, so each rank owns a disjoint slice of the app table: the
    # health exchange is ONE all-gather of per-rank records the scorer writes in place
    apps_per_rank = per // METRICS_PER_APP
    agg = HealthAggregator(n_local, per, dev, apps_per_rank=apps_per_rank if comm.active() else None)
    fused = {}
    if agg.fused:
        app_id = app_id - (s // METRICS_PER_APP)
        spec.n_apps = apps_per_rank
        fused = dict(app_stats=agg.app_stats_local, verdict_out=agg.verdict_local)
    shard = StreamingShard(spec, cfg, dev, app_id=app_id,
                           threshold=torch.full((n_local,), 4.0, device=dev),
                           bound=torch.full((n_local,), 3, dtype=torch.int8, device=dev), **fused)
    if args.serial_pairwise:
        shard.overlap_pairwise = False
    elif args.overlap_pairwise:
        shard.overlap_pairwise = True
    PW_OVERLAP[0] = bool(shard.overlap_pairwise)
    # --- synthetic data (outside the timed region) ---------------------------------
    # every datum is a function of the GLOBAL series index: N ranks score exactly the
    # series the one-rank run scores (tests/test_parallel.py::test_bench_n_rank_equals_one_rank)
    params = synthetic_params(args.series, dev, seed=1234, rows=(s, e))
    hist = synthetic_eval(params, 0, args.ring, args.season, noise_seed=4321, row0=s)
    if args.gap_frac > 0:
        g = torch.Generator().manual_seed(77)
        grows = torch.randperm(args.series, generator=g)[: int(round(args.gap_frac * args.series))]
        gstarts = torch.randint(args.season, args.ring - 30, (grows.numel(),), generator=g)
        mine = (grows >= s) & (grows < e)
        rows, starts = grows[mine] - s, gstarts[mine]
        cols = (starts[:, None] + torch.arange(30)[None, :]).reshape(-1)
        hist[rows.repeat_interleave(30).to(hist.device), cols.to(hist.device)] = float("nan")
    if args.miss_rate > 0:
        # isolated misses at a hash of the GLOBAL (series, column): every sharding drops the same points
        gr = torch.arange(s, e, device=hist.device, dtype=torch.int64)[:, None]
        gc = torch.arange(hist.shape[1], device=hist.device, dtype=torch.int64)[None, :]
        h = (gr * 1_000_003 + gc) * 6364136223846793005 + 1442695040888963407
        u = ((h >> 33) & 0xFFFFFF).double() / float(1 << 24)
        hist[u < args.miss_rate] = float("nan")
        del gr, gc, h, u
    shard.load_history(hist)
    del hist
    W, P = args.window, args.pods
    total_ticks = args.warmup + args.steps
    # per tick: P canary-pod values (a fraction of series regressed) and P
    # baseline-pod values (healthy, same times) -> [ticks, N, 2P]
    cur_t, bad = make_ticks(params, P, total_ticks + W, args.season, args.ring, 99, args.anomaly_frac,
                            args.anomaly_kind, want_bad=True, size=args.anomaly_size, row0=s, n_global=args.series)
    truth_apps = sorted(set(((bad.cpu() + s) // METRICS_PER_APP).tolist()))
    exch = None
    if args.multi_cluster:
        # each rank scrapes ONE cluster: rank r's canaries run in cluster r, their baselines in
        # cluster r-1, whose rank decodes them and ships them through the product's ClusterRouter
        # (parallel/affine.py: published requests, one all_to_all per tick)
        import asyncio
        from foremast_amd.parallel.affine import ClusterRouter
        served = (rank + 1) % world               # this rank's cluster holds the baselines of that shard
        r0, r1, _ = shard_range(args.series, world, served, METRICS_PER_APP)
        r_params = synthetic_params(args.series, dev, seed=1234, rows=(r0, r1))
        base_t = make_ticks(r_params, P, total_ticks + W, args.season, args.ring, 7, 0.0, row0=r0,
                            n_global=args.series)
        router = ClusterRouter(lambda ep, w: int(ep[len("cluster"):]) % w, dev)
        loop = asyncio.new_event_loop()
        family = (f"cluster{(rank - 1) % world}", "namespace_pod:baseline")
        shard_pod = [("bench", f"shard{rank}")]

        async def serve(reqs):
            # every request for this cluster's baselines comes from the shard it holds
            return [base_host[int(q[1])].reshape(1, -1).numpy() for q in reqs]

        def exch(k):
            # device values: the all-to-all's output is the owner's baseline block (no host copy)
            (vals,) = loop.run_until_complete(router.exchange([(family, float(k), n_local * P, shard_pod)], serve))
            return vals.view(n_local, P)
        ticks = cur_t
        base_host = base_t.cpu()
        if dev.type == "cuda":
            base_host = base_host.pin_memory()
        del base_t
    else:
        base_t = make_ticks(params, P, total_ticks + W, args.season, args.ring, 7, 0.0, row0=s, n_global=args.series)
        ticks = torch.cat([cur_t, base_t], 2)
        del base_t
    del cur_t
    pin = dev.type == "cuda"
    host_ticks = ticks.cpu()
    if pin:
        host_ticks = host_ticks.pin_memory()
    del ticks
    # --prefetch (pinned eager ticks): tick k+1's points are copied H2D on a copy stream into
    # the other of two device buffers while the GPU scores tick k
    prefetch = (dev.type == "cuda" and exch is None and args.ingest == "pinned" and not args.graph
                and args.prefetch)
    if exch is None:
        newvb = torch.empty((n_local, 2 * P), dtype=torch.float32, device=dev)
        newv, newb = newvb[:, :P], newvb[:, P:]
        if prefetch:
            copy_stream = torch.cuda.Stream(dev)
            in_bufs = [newvb, torch.empty_like(newvb)]
            in_ready = [torch.cuda.Event(), torch.cuda.Event()]
            in_free = [None, None]  # event of the ingest launch that last read the buffer
            staged = {}

            def stage(k):
                b = k % 2
                with torch.cuda.stream(copy_stream):
                    if in_free[b] is not None:
                        copy_stream.wait_event(in_free[b])
                    in_bufs[b].copy_(host_ticks[k], non_blocking=True)
                    in_ready[b].record(copy_stream)
                staged[k] = b
    else:
        newvb = torch.empty((n_local, P), dtype=torch.float32, device=dev)
        newv, newb = newvb, torch.empty((n_local, P), dtype=torch.float32, device=dev)

    decoder = None
    if args.ingest == "prom":
        if exch is not None:
            raise SystemExit("--ingest prom covers the single-cluster canary layout")
        decoder, bodies = prom_bodies(host_ticks, s, P, args.ring, args.decode_threads, pin)
        del host_ticks
        pending = {}

    def load_tick(k):
        """Make tick k's points available to the ingest launch; returns the
        (canary, baseline) device views to ingest and, with prefetch, the buffer
        index whose release event the caller records after the ingest."""
        if prefetch:
            b = staged.pop(k) if k in staged else (stage(k), staged.pop(k))[1]
            torch.cuda.current_stream().wait_event(in_ready[b])
            return in_bufs[b][:, :P], in_bufs[b][:, P:], b
        if zero_copy:
            return host_ticks[k][:, :P], host_ticks[k][:, P:], None
        load_tick_copy(k)
        return newv, newb, None

    def released(k, b):
        """After tick k's ingest was enqueued: free its buffer, stage tick k+1."""
        if b is None:
            return
        ev = torch.cuda.Event()
        ev.record()
        in_free[b] = ev
        if k + 1 < host_ticks.shape[0]:
            stage(k + 1)

    def load_tick_copy(k):
        if decoder is not None:
            fut = pending.pop(k, None) or decoder.submit(bodies[k], T_STEP * (args.ring + k), T_STEP)
            LAT_START[k - W] = fut.t_submit  # detect latency includes this tick's decode
            block, _ = fut.result()
            newvb.copy_(block.view(n_local, 2 * P), non_blocking=pin)
            if k + 1 < len(bodies):  # decode the next tick while the GPU scores this one
                pending[k + 1] = decoder.submit(bodies[k + 1], T_STEP * (args.ring + k + 1), T_STEP)
            return
        newvb.copy_(host_ticks[k], non_blocking=pin)
        if exch is not None:
            newb.copy_(exch(k), non_blocking=True)  # RC5: baseline windows to their owners (D2D)
    # host copy of the node health table (fused: the whole gathered record buffer)
    health_src = agg.recv if agg.fused else shard.app_stats
    # two host copies of the node health table: tick k+1's D2H may be enqueued while the
    # host still reads tick k's (pipelined ticks)
    health_hosts = [torch.empty_like(health_src, device="cpu") for _ in range(2)]
    if pin:
        health_hosts = [h.pin_memory() for h in health_hosts]
    health_host = health_hosts[0]
    pipelined = dev.type == "cuda" and args.pipeline and args.ingest == "pinned"
    zero_copy = (dev.type == "cuda" and args.zero_copy and args.ingest == "pinned" and exch is None
                 and not args.graph and not prefetch)
    # prefill the current window so every tick scores a full 10-minute window
    for k in range(W):
        nv, nb, b = load_tick(k)
        shard.ingest_tick(nv, nb)
        released(k, b)

    def graph_tail():
        """Captured at the end of the tick graph: the fused health all-gather (RCCL, when
        collectives run) and the copy of the node health table to pinned host memory."""
        if agg.fused:
            agg._gather_fused(shard.app_stats, shard.out["verdict"])
        health_hosts[0].copy_(agg.recv if agg.fused else shard.app_stats, non_blocking=pin)

    # double-buffered graph input: tick k+1's points are copied into the other buffer while
    # tick k runs (each buffer has its own captured graph)
    gpf = (args.graph and args.graph_prefetch and pin and exch is None and args.ingest == "pinned"
           and not pipelined)
    main_stream = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    if gpf:
        gbufs = [newvb, torch.empty_like(newvb)]
        gviews = [(g[:, :P], g[:, P:]) for g in gbufs]
        cstream = torch.cuda.Stream(dev)
        gstaged = [None, None]

        def gstage(i):
            """Copy tick i's points into its buffer on the copy stream and order the main
            stream after the copy (enqueued now, behind the tick in flight: the next tick's
            launch then has no wait to enqueue on the host's critical path)."""
            b = i % 2
            with torch.cuda.stream(cstream):
                gbufs[b].copy_(host_ticks[i], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cstream)
            main_stream.wait_event(ev)
            gstaged[b] = i

    def wait_tick():
        if dev.type != "cuda":
            return
        if args.spin_wait:
            ev = torch.cuda.Event()
            ev.record()
            while not ev.query():
                pass
        else:
            main_stream.synchronize()

    bell = gpf and args.doorbell and dev.type == "cuda"
    if bell:
        shard.enable_doorbell()
        DOORBELL[0] = shard
    queued = {}  # doorbell mode: tick index -> (outputs, completion event) of a tick enqueued ahead
    n_ticks_total = args.warmup + args.steps

    def tick_bell(k):
        """Doorbell graph tick k: ring the tick enqueued ahead (or enqueue it now), enqueue
        tick k + 1 behind it, then wait for tick k."""
        i = W + k
        b = i % 2
        hit = queued.pop(k, None)
        if hit is None:
            if gstaged[b] != i:
                gstage(i)
            out = shard.tick_graph(gviews[b][0], gviews[b][1], post=graph_tail)
            ev = torch.cuda.Event()
            ev.record()
        else:
            out, ev = hit
        LAT_START[k] = time.perf_counter()
        shard.ring()  # tick k starts (its input was copied before it was enqueued)
        # enqueue tick k + 1 (not across the warmup / timed boundary, whose synchronize would
        # wait on a tick no one rings)
        if k + 1 < n_ticks_total and k + 1 != args.warmup and i + 1 < host_ticks.shape[0]:
            gstage(i + 1)  # the other buffer's reader (tick k - 1) has completed
            nxt = shard.tick_graph(gviews[1 - b][0], gviews[1 - b][1], post=graph_tail)
            ev1 = torch.cuda.Event()
            ev1.record()
            queued[k + 1] = (nxt, ev1)
        REFIT_FLAGS[k] = shard.last_refit
        GRAPH_TAIL[0] = bool(out.get("post_in_graph"))
        if args.spin_wait:
            while not ev.query():
                pass
        else:
            ev.synchronize()
        if not out.get("post_in_graph"):
            stats, _ = agg.tick(shard.app_stats, out["verdict"])
            health_hosts[0].copy_(agg.recv if agg.fused else stats, non_blocking=pin)
            main_stream.synchronize()
        return out

    def tick(k):
        if bell and shard.graph_ready():  # every replay of a doorbell graph is rung by tick_bell
            return tick_bell(k)
        if gpf and shard.graph_ready():
            i = W + k
            b = i % 2
            if gstaged[b] != i:
                gstage(i)
            out = shard.tick_graph(gviews[b][0], gviews[b][1], post=graph_tail)
            if i + 1 < host_ticks.shape[0]:
                gstage(i + 1)  # the other buffer's reader (tick i - 1) has completed
            REFIT_FLAGS[k] = shard.last_refit
            if out.get("post_in_graph"):
                GRAPH_TAIL[0] = True
                wait_tick()
                return out
            stats, _ = agg.tick(shard.app_stats, out["verdict"])
            health_hosts[0].copy_(agg.recv if agg.fused else stats, non_blocking=pin)
            wait_tick()
            return out
        nv, nb, b = load_tick(W + k)
        if args.graph:
            # ingest + score (+ the health collective and the table's copy back) as one replay
            out = shard.tick_graph(nv, nb, post=graph_tail if (pin and not pipelined) else None)
        else:
            shard.ingest_tick(nv, nb)
            released(W + k, b)
            out = shard.score()
        REFIT_FLAGS[k] = shard.last_refit
        if out.get("post_in_graph"):
            GRAPH_TAIL[0] = True
            wait_tick()
            return out
        stats, _ = agg.tick(shard.app_stats, out["verdict"])
        hh = health_hosts[k % 2 if pipelined else 0]
        if zero_copy:
            from foremast_amd.ops import kernels as K
            K.copy_to_host(hh.view(-1), (agg.recv if agg.fused else stats).view(-1))
        else:
            hh.copy_(agg.recv if agg.fused else stats, non_blocking=pin)
        if pipelined:
            ev = torch.cuda.Event()
            ev.record()
            return InFlight(ev, hh)  # the caller waits for it after enqueueing the next tick
        if dev.type == "cuda":
            torch.cuda.current_stream().synchronize()
        return out

    meta = {
        "model": f"{args.algorithm} + pairwise {args.pairwise} (MW U / Wilcoxon / Kruskal) canary scorer",
        "global_batch": args.series,
        "seq_len": args.ring,
        "season": args.season,
        "pods": P,
        "current_window": W,
        "grid_points": int(shard.grid.shape[0]),
        "multi_cluster": bool(args.multi_cluster),
        "affine_exchanges": router.exchanges if args.multi_cluster else 0,
        "gap_frac": args.gap_frac,
        "miss_rate": args.miss_rate,
        "prune_hints": ("previous winners first (exact: the branch and bound's order only)"
                        if os.environ.get("FOREMAST_HW_HINTS", "1") != "0" else "off (grid order)"),
        "pairwise_shift_sigma": cfg.pairwise_shift,
        "pairwise_shift_spread": "one-step sigma" if cfg.pairwise_shift_one_step else "horizon-scaled sigma",
        "health_collectives": "1 fused all_gather" if agg.fused else ("all_reduce + all_gather" if agg.active else "none"),
        "hip_graph": bool(args.graph and dev.type == "cuda"),
        "ingest": args.ingest,
        "pipelined_ticks": pipelined,
        "input_prefetch": prefetch or ("double-buffered H2D of tick k+1 during tick k (graph ticks)" if gpf else False),
        "spin_wait": bool(args.spin_wait),
        "doorbell": bool(bell),
        "zero_copy": zero_copy,
        "model_cache": ("none: every tick refits every series" if args.refit_every <= 1 else
                        f"refit every {args.refit_every} ticks, O(1) Holt-Winters state update + detect in between"),
    }
    if decoder is not None:
        meta["ingest_bytes_per_tick"] = int(sum(len(b) for b in bodies[0]))
        meta["_decoder"] = decoder
    if agg.fused:
        meta["_table"] = lambda h: HealthAggregator.host_app_table(h, world, apps_per_rank)
    dt = "bf16" if dtype == torch.bfloat16 else "fp32"
    meta["_agg"] = agg
    meta["_truth"] = (truth_apps, n_apps)
    meta["_graph_used"] = lambda: shard._graph is not None  # captured (vs eager fallback)
    if dev.type == "cuda" and args.algorithm == "holt_winters":
        from foremast_amd.ops import kernels as K
        d0 = K.hw_deferred_total(dev)
        # series pairs per fit that took the gapped-series kernel (a pair with a missing point
        # past season 0), averaged over every tick run
        meta["_deferred"] = lambda ticks: round((K.hw_deferred_total(dev) - d0) / max(1, ticks), 2)
    return tick, health_host, meta, dt, args.series


T_STEP = 60.0  # query step (metricsquery.go:43)


class InFlight(NamedTuple):
    """A pipelined tick's completion event and the host copy its health table lands in."""
    event: "torch.cuda.Event"
    host: torch.Tensor
LAT_START = {}  # timed tick -> perf_counter time its data arrived (set by the prom ingest path)
REFIT_FLAGS = {}  # tick -> whether it refit the model (canary --refit-every)
GRAPH_TAIL = [False]  # canary: the health collective + copy back ran inside the tick graph
DOORBELL = [None]     # canary --doorbell: the shard (its doorbell waits that timed out are recorded)
PW_OVERLAP = [None]   # canary: rank tests on a side stream beside the fit (True) or before it


def prom_bodies(host_ticks, s, P, ring, threads, pin):
    """Render every tick's points as Prometheus ``query_range`` bodies (untimed
    setup): per metric family one body for the canary pods and one for the
    baseline pods, one series per (app, pod) — the shape the brain gets from
    ``namespace_pod:<metric>{...}`` at a 60 s step.  Returns the decoder (key
    tables from the bodies' own label order) and ``bodies[tick][family*2+kind]``."""
    from foremast_amd.ingest import native
    from foremast_amd.ingest.tickdecode import TickDecoder, pod_matrix_body
    nt, n, twoP = host_ticks.shape
    gid = np.arange(n) + s                     # global series id: app = gid // 5, family = gid % 5
    labels, rows, sel = [], [], []
    for m in range(METRICS_PER_APP):
        ids = np.nonzero(gid % METRICS_PER_APP == m)[0]
        for kind, tag in enumerate(("c", "b")):
            labels.append([f'"namespace":"ns{a % 200}","app":"app{a}","pod":"app{a}-{tag}{p}-7d9f8b6c5d"'
                           for a in (gid[ids] // METRICS_PER_APP).tolist() for p in range(P)])
            rows.append((ids[:, None] * twoP + kind * P + np.arange(P)[None, :]).reshape(-1))
            sel.append((ids, kind))
    vals = host_ticks.numpy()
    bodies = []
    for k in range(nt):
        ts = T_STEP * (ring + k)
        bodies.append([pod_matrix_body(f"namespace_pod:metric{j // 2}", labels[j], ts,
                                       vals[k, ids, kind * P:(kind + 1) * P].reshape(-1))
                       for j, (ids, kind) in enumerate(sel)])
    tables = [native.KeyTable.from_hashes(native.series_keys(b, "app", "pod"), r, "app", "pod")
              for b, r in zip(bodies[0], rows)]
    return TickDecoder(tables, n * twoP, 1, pinned=pin, threads=threads), bodies


def setup_lstm(args, world, rank, dev, n_features, fp8):
    """Config 3 (univariate LSTM-AE, DP training + scoring) and config 5
    (multivariate latency + error-rate entities, fp8 MFMA scoring).

    Per tick: ingest one point per metric-series, one DP training step
    (gradient all-reduce over RCCL), device-side weight repack, fused LSTM-AE
    scoring of every entity's latest window, cluster aggregation, D2H."""
    from foremast_amd.brain.lstm_engine import LstmShard
    F = n_features
    if dev.type == "cpu" and args.series > 4096:
        args.series, args.ring, args.season, args.lstm_train_batch = 256, 480, 48, 64
    n_ent = args.series // F  # entities; each has F metric-series
    s, e, per = shard_range(n_ent, world, rank, align=1)
    n_local = e - s
    ent_per_app = max(1, METRICS_PER_APP // F)
    n_apps = (n_ent + ent_per_app - 1) // ent_per_app
    app_id = (torch.arange(s, e, device=dev, dtype=torch.int64) // ent_per_app).to(torch.int32)
    shard = LstmShard(n_local, args.ring, F, window=args.lstm_window, hidden=64, fp8=fp8, device=dev,
                      app_id=app_id, n_apps=n_apps, threshold=args.lstm_threshold,
                      train_batch=args.lstm_train_batch, lr=1e-3, seed=0, fused_train=not args.lstm_autograd,
                      restat_every=args.lstm_restat_every, season=args.season, cal_ewma=args.lstm_cal_ewma,
                      level_threshold=args.lstm_level_threshold if args.lstm_level_threshold > 0 else None)
    params = [synthetic_params(n_ent, dev, seed=1234 + 7 * f, rows=(s, e)) for f in range(F)]
    shard.load_history([synthetic_eval(p, 0, args.ring, args.season, noise_seed=555 + f, row0=s)
                        for f, p in enumerate(params)])
    total = args.warmup + args.steps
    # the same entities regress on every metric (seed shared across features)
    tk = [make_ticks(p, 1, total, args.season, args.ring, 99, args.anomaly_frac, args.anomaly_kind,
                     want_bad=True, size=args.anomaly_size, row0=s, n_global=n_ent) for p in params]
    ticks = torch.stack([t[..., 0] for t, _ in tk], 2)  # [ticks, n, F]
    truth_apps = sorted(set(((tk[0][1].cpu() + s) // ent_per_app).tolist()))
    bad_local = tk[0][1].cpu()
    del tk
    pin = dev.type == "cuda"
    host_ticks = ticks.cpu()
    if pin:
        host_ticks = host_ticks.pin_memory()
    del ticks
    newx = torch.empty((n_local, F), dtype=torch.float32, device=dev)
    agg = HealthAggregator(n_local, per, dev)
    health_host = torch.empty_like(shard.app_stats, device="cpu")
    if pin:
        health_host = health_host.pin_memory()
    # model initialisation (outside the timed region): a few DP steps + calibration
    for _ in range(args.lstm_pretrain):
        shard.train_step()
    shard.calibrate(args.lstm_train_batch)

    def tick(k):
        newx.copy_(host_ticks[k], non_blocking=pin)
        out = shard.tick(newx, train=(k % args.lstm_train_every == 0), overlap=not args.lstm_no_overlap)
        stats, _ = agg.tick(shard.app_stats, out["verdict"])
        health_host.copy_(stats, non_blocking=pin)
        if dev.type == "cuda":
            torch.cuda.current_stream().synchronize()
        return out

    meta = {
        "model": f"LSTM autoencoder (F={F}, H=64, window {args.lstm_window}), DP Adam step "
                 f"(batch {args.lstm_train_batch}/rank) every {args.lstm_train_every} tick(s) + fused scoring",
        "global_batch": n_ent,
        "seq_len": args.lstm_window,
        "history": args.ring,
        "entities": n_ent,
        "features": F,
        "train_batch_per_rank": args.lstm_train_batch,
        "scoring_dtype": "fp8_e4m3" if fp8 else "bf16",
        "training": "fused K7 kernel + hipBLASLt weight-grad GEMMs" if shard.fused_train else "autograd",
        "entity": ("one (app, caller) pair: the latency + error-rate series of the requests a calling service "
                   "sends to a deployed app (downstream impact, metricType: downstream)" if F == 2 else
                   "one univariate metric-series"),
        "train_score_overlap": not args.lstm_no_overlap,
    }
    # compute dtype of the scoring (the metric's work): fp8 e4m3 block-scaled MFMA for config 5,
    # bf16 MFMA otherwise (training: fp32 master weights either way)
    dt = "fp8_e4m3" if fp8 else "bf16"
    meta["_agg"] = agg
    meta["_truth"] = (truth_apps, n_apps)
    meta["_shard"], meta["_bad"], meta["_ticks"], meta["_params"] = shard, bad_local, host_ticks, params
    return tick, health_host, meta, dt, n_ent * F


def setup_single(args, world, rank, dev):
    """Config 1: one ``http_server_requests_latency`` series per rank, moving
    average on CPU, through the whole brain path per step: register a job via
    the service API, claim, fetch the three windows from (fake) Prometheus
    over HTTP/ASGI, parse, score, write the verdict and export the band."""
    import asyncio
    import httpx
    from foremast_amd.brain.batch import BatchScorer
    from foremast_amd.brain.worker import BrainWorker
    from foremast_amd.promql import synth
    from foremast_amd.promql.client import PromClient
    from foremast_amd.promql.fake import FakePrometheus
    from foremast_amd.service import app as svc
    from foremast_amd.store import MemoryJobStore
    from foremast_amd.utils.config import reference_default_env
    from foremast_amd.utils.timeutil import format_rfc3339
    metric = "http_server_requests_latency"
    t0 = 1_700_000_000.0
    state = {"now": t0}
    prom = FakePrometheus(clock=lambda: state["now"])
    prom.add("namespace_app_per_pod:" + metric, {"namespace": "ns", "app": "demo"},
             synth.seasonal(level=0.12, amp=0.02, noise=0.004, seed=rank))
    prom.add("namespace_pod:" + metric, {"namespace": "ns", "pod": "demo-v2"},
             synth.seasonal(level=0.12, amp=0.02, noise=0.004, seed=100 + rank))
    store = MemoryJobStore()
    env = reference_default_env()
    env["ML_ALGORITHM"] = "moving_average_all"
    cfg = BrainConfig.from_env(env)
    loop = asyncio.new_event_loop()
    brain = BrainWorker(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                        scorer=BatchScorer(cfg, device=torch.device("cpu")), worker_id=f"bench-{rank}",
                        clock=lambda: state["now"])

    def job(k):
        start = t0 + 600 * k
        q = {"endpoint": "http://prometheus:9090/api/v1/", "step": 60}
        return {"appName": "demo", "startTime": format_rfc3339(start), "endTime": format_rfc3339(start + 600),
                "strategy": "rollingupdate", "metrics": {
                    "current": {"latency": {"dataSourceType": "prometheus", "parameters": dict(
                        q, query=f'namespace_pod:{metric}{{namespace="ns",pod="demo-v2"}}',
                        start=int(start), end=int(start + 600))}},
                    "historical": {"latency": {"dataSourceType": "prometheus", "parameters": dict(
                        q, query=f'namespace_app_per_pod:{metric}{{namespace="ns",app="demo"}}',
                        start=int(start - 7 * 86400), end=int(start))}}}}

    last = {}

    def tick(k):
        state["now"] = t0 + 600 * k + 660  # the window is over: the job finishes this cycle
        code, body = svc.register(store, job(k))
        assert code == 200, body
        n = loop.run_until_complete(brain.cycle())
        assert n == 1
        last["status"] = store.get(body["jobId"])["status"]
        return last

    health = torch.zeros((1, 2), dtype=torch.int32)

    def tick_and_health(k):
        out = tick(k)
        health[0, 0] = int(out["status"] == "completed_unhealth")
        health[0, 1] = 1
        return out

    meta = {"model": "moving_average_all on one http_server_requests_latency series (CPU brain, end to end)",
            "global_batch": world, "seq_len": 10080, "path": "service register -> claim -> Prometheus HTTP -> "
            "native parse -> score -> verdict write"}
    return tick_and_health, health, meta, "fp32", world


def run_cpu_baseline_lstm(args, F: int) -> None:
    """Comparator of configs 3 / 5: one entity at a time on ONE core — z-score
    its F histories, run the LSTM autoencoder (H=64) over its latest window,
    compare the reconstruction error — scoring only (no training, which only
    favours the baseline)."""
    from foremast_amd.models.lstm_ae import LSTMAutoencoder
    torch.set_num_threads(1)
    dev = torch.device("cpu")
    n, T = args.baseline_sample, args.lstm_window
    torch.manual_seed(0)
    model = LSTMAutoencoder(F, 64).eval()
    params = [synthetic_params(n, dev, seed=1234 + 7 * f) for f in range(F)]
    hist = np.stack([synthetic_eval(p, 0, args.ring, args.season, noise_seed=555 + f).numpy()
                     for f, p in enumerate(params)], 2)  # [n, R, F]
    t0 = time.perf_counter()
    flagged = 0
    with torch.no_grad():
        for i in range(n):
            h = hist[i]
            mu, sd = h.mean(0), np.maximum(h.std(0), 1e-6)
            x = torch.from_numpy(((h[-T:] - mu) / sd).astype(np.float32))[None]
            err = float(model.recon_error(x))
            flagged += int(err > 1.0 + 4.0 * 0.5)
    dt = time.perf_counter() - t0
    rate = n * F / dt
    print(json.dumps({
        "metric": METRIC, "value": round(rate, 3), "unit": "series/s", "n_gpus": 0, "steps": 1, "warmup": 0,
        "ms_per_entity": round(dt / n * 1e3, 3), "higher_is_better": True, "scaling": "none", "vs_baseline": 1.0,
        "dtype": "fp32", "data": "synthetic (same generator as the lstm bench); random-init weights",
        "config": {"model": f"LSTM autoencoder (F={F}, H=64, window {T}) scoring, per entity",
                   "bench_config": "cpu_baseline", "baseline_model": args.baseline_model, "global_batch": n,
                   "seq_len": T, "history": args.ring, "device": "cpu, 1 core (torch CPU, batch 1)",
                   "reference_budget_100m_cpu_series_per_s": round(rate * 0.1, 4)}}), flush=True)


def run_cpu_baseline(args) -> None:
    """The comparator: the headline canary scorer as a per-series numpy/scipy
    loop on ONE CPU core (models/cpu_baseline.py) over a sample of the same
    synthetic series, windows and injected regressions."""
    if args.baseline_model != "canary":
        return run_cpu_baseline_lstm(args, 1 if args.baseline_model == "lstm" else 2)
    from foremast_amd.models import cpu_baseline as cb
    from foremast_amd.models import smoothing as sm
    torch.set_num_threads(1)
    dev = torch.device("cpu")
    n, P, W = args.baseline_sample, args.pods, args.window
    cfg = BrainConfig()
    grid = sm.make_grid(sm.MODE_HW, cfg.hw_alpha, cfg.hw_beta, cfg.hw_gamma).numpy()
    params = synthetic_params(n, dev, seed=1234)
    hist = synthetic_eval(params, 0, args.ring, args.season, noise_seed=4321).numpy()
    cur, bad = make_ticks(params, P, W, args.season, args.ring, 99, max(args.anomaly_frac, 1.0 / n),
                          args.anomaly_kind, want_bad=True, size=args.anomaly_size)
    base = make_ticks(params, P, W, args.season, args.ring, 7, 0.0)
    cur = cur.permute(1, 2, 0).reshape(n, P * W).numpy()    # pod-major windows, as the engine's
    base = base.permute(1, 2, 0).reshape(n, P * W).numpy()
    hz = np.tile(np.arange(1, W + 1), P)
    t0 = time.perf_counter()
    verdicts = [cb.score_series(hist[i], cur[i], base[i], hz, args.season, grid, threshold=4.0, bound=3,
                                alpha=cfg.pairwise_threshold, pairwise_scale=cfg.pairwise_scale,
                                pw_min_points=cfg.pairwise_min_points,
                                shift_threshold=cfg.pairwise_shift,
                                shift_min_points=cfg.pairwise_shift_min_points,
                                shift_one_step=cfg.pairwise_shift_one_step).verdict for i in range(n)]
    dt = time.perf_counter() - t0
    truth = set(bad.tolist())
    flagged = {i for i, v in enumerate(verdicts) if v == 1}
    rate = n / dt
    print(json.dumps({
        "metric": METRIC, "value": round(rate, 3), "unit": "series/s", "n_gpus": 0, "steps": 1, "warmup": 0,
        "ms_per_series": round(dt / n * 1e3, 2), "higher_is_better": True, "scaling": "none", "vs_baseline": 1.0,
        "dtype": "fp64", "data": "synthetic (same generator and seeds as the canary bench)",
        "config": {"model": "holt_winters (64-point grid) + scipy mannwhitneyu/wilcoxon/kruskal, per series",
                   "bench_config": "cpu_baseline", "baseline_model": "canary", "global_batch": n,
                   "seq_len": args.ring, "season": args.season,
                   "pods": P, "current_window": W, "device": "cpu, 1 core (numpy/scipy loop)",
                   "reference_budget_100m_cpu_series_per_s": round(rate * 0.1, 4)},
        "detection": {"injected": len(truth), "tp": len(truth & flagged), "fp": len(flagged - truth)},
    }), flush=True)


def main():
    args = parse()
    if args.config == "cpu_baseline":
        run_cpu_baseline(args)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, sys.argv[1:]))
    if args.config == "hw10k":
        args.series = 10_000  # BASELINE config 2: same pipeline as the headline at 10k series
        args.config = "canary"
        args.config_name = "hw10k"
    world, rank, dev = init_dist(args)
    if args.config == "single":
        tick, health_host, meta, dtype_name, n_series = setup_single(args, world, rank, dev)
    elif args.config == "canary":
        tick, health_host, meta, dtype_name, n_series = setup_canary(args, world, rank, dev)
    elif args.config == "node" and args.arrival_per_tick > 0:
        from foremast_amd.benchmarks.node import setup_arrival
        tick, health_host, meta, dtype_name, n_series = setup_arrival(args, world, rank, dev)
    elif args.config == "node-lstm":
        from foremast_amd.benchmarks.node import setup_node_lstm
        tick, health_host, meta, dtype_name, n_series = setup_node_lstm(args, world, rank, dev)
    elif args.config == "node":
        from foremast_amd.benchmarks.node import setup_node
        tick, health_host, meta, dtype_name, n_series = setup_node(args, world, rank, dev)
    elif args.config == "lstm":
        tick, health_host, meta, dtype_name, n_series = setup_lstm(args, world, rank, dev, 1, False)
    else:
        tick, health_host, meta, dtype_name, n_series = setup_lstm(args, world, rank, dev, 2, not args.mv_bf16)

    agg = meta.pop("_agg", None)
    table = meta.pop("_table", None)
    decoder = meta.pop("_decoder", None)
    truth = meta.pop("_truth", None)
    scored_rows = meta.pop("_scored_rows", None)   # node: rows actually scored per tick
    node_finish = meta.pop("_finish", None)
    arrival_finish = meta.pop("_arrival_finish", None)
    node_roll = meta.pop("_roll", None)
    node_breakdowns = meta.pop("_breakdowns", None)
    graph_used = meta.pop("_graph_used", None)
    deferred = meta.pop("_deferred", None)
    for k in [k for k in meta if k.startswith("_")]:
        meta.pop(k)
    if truth is not None and world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, truth[0])
        truth = (sorted(set().union(*parts)), truth[1])
    pending = None  # pipelined ticks: (event, health copy, start time) of the tick in flight

    def run(k):
        """One tick; returns the detect latency of the tick that completed (or None)."""
        nonlocal pending, health_host
        ts = time.perf_counter()
        r = tick(k)
        if not isinstance(r, InFlight):
            return time.perf_counter() - LAT_START.pop(k, ts)
        done, pending = pending, (r.event, r.host, LAT_START.pop(k, ts))
        if done is None:
            return None
        done[0].synchronize()
        health_host = done[1]
        return time.perf_counter() - done[2]

    def drain():
        nonlocal pending, health_host
        if pending is None:
            return None
        pending[0].synchronize()
        health_host = pending[1]
        lat_s = time.perf_counter() - pending[2]
        pending = None
        return lat_s

    for k in range(args.warmup):
        run(k)
    drain()
    if agg is not None:
        agg.flush_timings()
        agg.timings_ms.clear()
    barrier(dev)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    lat = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        x = run(args.warmup + k)
        if x is not None:
            lat.append(x)
    x = drain()
    if x is not None:
        lat.append(x)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    barrier(dev)
    elapsed = time.perf_counter() - t0
    if graph_used is not None:
        meta["hip_graph"] = bool(graph_used())
    if deferred is not None:
        meta["gapped_pairs_per_tick"] = deferred(args.warmup + args.steps)
    if args.config in ("canary", "hw10k") or getattr(args, "config_name", "") == "hw10k":
        meta["health_tail_in_graph"] = GRAPH_TAIL[0]
        if DOORBELL[0] is not None:
            meta["doorbell_timeouts"] = DOORBELL[0].doorbell_timeouts()
        if PW_OVERLAP[0] is not None:
            meta["pairwise_overlap"] = "side stream beside the fit" if PW_OVERLAP[0] else "before the fit (fused detect)"
        if GRAPH_TAIL[0] and meta.get("health_collectives", "none") != "none":
            meta["health_collectives"] += " (captured in the tick graph)"
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    lat_t = torch.tensor(lat, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(lat_t, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    lat_ms = lat_t.cpu().numpy() * 1e3
    timed_rows = None
    if scored_rows is not None:
        rows_t = torch.tensor([float(sum(scored_rows[args.warmup:]))], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(rows_t)
        timed_rows = float(rows_t.item())
        tick_breakdown = {k: round(v, 3) for k, v in node_roll.timings.items()} if node_roll is not None else {}
        if arrival_finish is not None:
            fin_s, statuses, arrival_det = arrival_finish()
            if world > 1:  # every rank's jobs: the node's detection, not rank 0's share
                parts = [None] * world
                dist.all_gather_object(parts, arrival_det)
                arrival_det = _sum_detection(parts)
        else:
            fin_s, statuses = node_finish()
    coll_ms = agg.flush_timings() if agg is not None else []
    if table is not None:
        health_host = table(health_host)
    anomalous_apps = int((health_host[:, 0] > 0).sum())
    scored = int(health_host[:, 1].sum())
    if rank == 0:
        value = (timed_rows if timed_rows is not None else n_series * args.steps) / elapsed
        cfg_name = getattr(args, "config_name", args.config)
        config = {"model": meta.pop("model"), "global_batch": meta.pop("global_batch"),
                  "seq_len": meta.pop("seq_len"), "parallelism": f"dp{world}",
                  "bench_config": getattr(args, "config_name", args.config)}
        config.update(meta)
        config["device"] = str(dev) if dev.type == "cpu" else torch.cuda.get_device_name(dev)
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "series/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (round(value / CPU_BASELINE_SERIES_PER_S[cfg_name], 1)
                            if cfg_name in CPU_BASELINE_SERIES_PER_S else None),
            "dtype": dtype_name,
            "data": "synthetic (seasonal Prometheus-like range-vectors, random per-series params; random-init weights)",
            "config": config,
            "p50_detect_latency_ms": round(float(np.percentile(lat_ms, 50)), 3),
            # a p99 needs >= 100 samples; with fewer only the max is a statistic worth printing
            "p99_detect_latency_ms": (round(float(np.percentile(lat_ms, 99)), 3) if len(lat_ms) >= P99_MIN
                                      else None),
            "max_detect_latency_ms": round(float(np.max(lat_ms)), 3) if len(lat_ms) else None,
            "latency_samples": int(len(lat_ms)),
            # device time of the per-tick health collectives (fused all-gather, or RC2 all-reduce +
            # RC1 all-gather), rank 0
            "collective_ms_p50": round(float(np.percentile(coll_ms, 50)), 4) if coll_ms else None,
            "health": {"apps": int(health_host.shape[0]), "anomalous_apps": anomalous_apps,
                       "series_scored_last_tick": scored},
        }
        if decoder is not None:
            res["decode_ms_last_tick"] = round(decoder.last_decode_ms, 3)
        if timed_rows is not None and arrival_finish is not None and args.config == "node-lstm":
            res["tails"] = _tail_attribution((node_breakdowns or [])[-args.steps:])
        if timed_rows is not None and arrival_finish is not None:
            bds = (node_breakdowns or [])[-args.steps:]

            def pct(key, q):
                xs = [b[key] for b in bds if key in b]
                if q == 99 and len(xs) < P99_MIN:
                    return None
                return round(float(np.percentile(xs, q)), 3) if xs else None
            adm = [b for b in bds if b.get("admitted")]
            res["p50_detect_latency_ms"] = pct("detect_ms", 50)
            res["p99_detect_latency_ms"] = pct("detect_ms", 99)
            res["max_detect_latency_ms"] = pct("detect_ms", 100)
            res["latency_samples"] = len([b for b in bds if "detect_ms" in b])
            res["node"] = {
                "series_scored_timed": int(timed_rows),
                "detect_ms_p50_p99_max": [pct("detect_ms", 50), pct("detect_ms", 99), pct("detect_ms", 100)],
                "tick_total_ms_p50_p99_max": [pct("tick_total_ms", 50), pct("tick_total_ms", 99),
                                              pct("tick_total_ms", 100)],
                "intake_ms_p50_p99_max": [pct("intake_ms", 50), pct("intake_ms", 99), pct("intake_ms", 100)],
                # the same phases without the in-process Prometheus stand-in's own serving time
                "net_of_standin": {k: [pct(k, 50), pct(k, 99), pct(k, 100)]
                                   for k in ("detect_net_ms", "intake_net_ms", "tick_net_ms")},
                "admitted_per_tick_mean": round(float(np.mean([b.get("admitted", 0) for b in bds])), 1) if bds else 0,
                "admission_ms_p50": {k: (round(float(np.percentile([b.get(k, 0.0) for b in adm], 50)), 3)
                                         if adm else None)
                                     for k in ("claim_ms", "plan_ms", "admit_ms", "admit_rows_ms", "admit_fit_ms",
                                               "admit_windows_ms")},
                "live_rows_mean": round(float(np.mean([b.get("live_rows", 0) for b in bds])), 1) if bds else 0,
                "tick_breakdown_ms": bds,
                "completion_ticks_s": round(fin_s, 3), "job_statuses_rank0": statuses}
            res["detection"] = arrival_det
        if timed_rows is not None and arrival_finish is None:
            res["node"] = {"series_scored_timed": int(timed_rows), "tick_breakdown_ms_last": tick_breakdown,
                           "tick_breakdown_ms": (node_breakdowns or [])[-args.steps:],
                           "tick_ms": [round(float(x), 2) for x in lat_ms.tolist()],
                           "completion_tick_s": round(fin_s, 3), "job_statuses_rank0": statuses}
        if timed_rows is not None:
            res["node"]["exchange"] = _exchange_summary(node_breakdowns or [], args.steps, world, args.config)
        if args.config == "canary" and args.refit_every > 1:
            flags = np.array([REFIT_FLAGS.get(args.warmup + k, True) for k in range(args.steps)])
            res["refit_ticks_timed"] = int(flags.sum())
            for name, sel in (("refit", flags), ("cached", ~flags)):
                if sel.any():
                    res[f"p50_{name}_tick_ms"] = round(float(np.percentile(lat_ms[sel], 50)), 3)
        if truth is not None:
            size = f" {args.anomaly_size:g}" if args.anomaly_kind in ("scale", "shift") else ""
            res["detection"] = dict(detection_report(health_host, truth[0], truth[1]),
                                    injected=f"{args.anomaly_kind}{size} on {args.anomaly_frac:g} of series")
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
