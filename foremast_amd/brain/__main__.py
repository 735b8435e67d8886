"""``python -m foremast_amd.brain`` — the scoring worker process.

Replaces the foremast-brain container (``deploy/foremast/3_brain/foremast-brain.yaml``):
same environment variables (``ES_ENDPOINT``, ``ML_ALGORITHM``, ``threshold``,
``bound``, ``metric_type{i}`` …, ``MAX_STUCK_IN_SECONDS``; parsed by
:class:`~foremast_amd.utils.config.BrainConfig`), same Prometheus exposition
on :8000 (``foremastbrain:<metric>_{upper,lower,anomaly}`` plus engine
metrics).  ``FOREMAST_JOB_STORE`` (``sqlite:///…`` / ``memory://``) overrides
``ES_ENDPOINT``.  Several processes can share one store: claims are leases.

Node mode (``--streaming`` with ``--nproc N``, or under torchrun): one rank per
GPU, continuous jobs sharded by app over the ranks, ONE all-gather of per-app
counters per tick (RCCL), rank 0 publishes the node health table that
``GET /v1/healthcheck/cluster`` serves; a dead rank's apps move to the
survivors (``brain/node.py``).
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal

from ..store.jobstore import open_store
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from .worker import BrainWorker


def parse(argv=None):
    p = argparse.ArgumentParser(prog="foremast-brain")
    p.add_argument("--store", default=os.environ.get("FOREMAST_JOB_STORE") or os.environ.get("ES_ENDPOINT"))
    p.add_argument("--metrics-port", type=int, default=int(os.environ.get("FOREMAST_METRICS_PORT", "8000")))
    p.add_argument("--worker-id", default=None)
    p.add_argument("--run-seconds", type=float, default=None)
    p.add_argument("--streaming", action="store_true",
                   default=os.environ.get("FOREMAST_STREAMING", "0") not in ("0", "", "false"),
                   help="serve continuous jobs from the resident streaming engine")
    p.add_argument("--model-cache", default=os.environ.get("FOREMAST_MODEL_CACHE"),
                   help="safetensors checkpoint of the LSTM model cache (loaded at start, saved at exit)")
    p.add_argument("--snapshot", default=os.environ.get("FOREMAST_SNAPSHOT"),
                   help="streaming-engine snapshot ({rank} expands): resume from it, re-save periodically and at exit")
    p.add_argument("--snapshot-every", type=int, default=int(os.environ.get("FOREMAST_SNAPSHOT_EVERY", "60")),
                   help="ticks between streaming snapshots")
    p.add_argument("--nproc", type=int, default=int(os.environ.get("FOREMAST_NPROC", "1")),
                   help="node mode: start this many brain ranks (one per GPU) around a node key-value store")
    p.add_argument("--tick-seconds", type=float, default=None,
                   help="streaming tick period (default: the query step)")
    p.add_argument("--rollout", type=int, default=int(os.environ.get("FOREMAST_ROLLOUT", "1")),
                   help="with --streaming: serve canary / rollingUpdate jobs from the resident rollout engine")
    p.add_argument("--lstm", type=int, default=(int(os.environ["FOREMAST_LSTM"]) if os.environ.get("FOREMAST_LSTM")
                                                 else None),
                   help="with --streaming: serve continuous multi-metric jobs from the resident DP LSTM engine "
                        "(default: when ML_ALGORITHM is lstm or auto)")
    p.add_argument("--pods", type=int, default=int(os.environ.get("FOREMAST_CANARY_PODS", "5")),
                   help="rollout engine: pods per side kept per (job, metric) window")
    p.add_argument("--step", type=float, default=float(os.environ.get("FOREMAST_STEP_SECONDS", "60")))
    p.add_argument("--window", type=int, default=int(os.environ.get("FOREMAST_WINDOW", "10")))
    return p.parse_args(argv)


def _bind_gpu() -> int:
    """One scorer process per GPU (launch_node or torchrun): bind LOCAL_RANK's device."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(local % torch.cuda.device_count())
    except ImportError:
        pass
    return local


async def run(args) -> BrainWorker:
    local = _bind_gpu()
    cfg = BrainConfig.from_env()
    store = open_store(args.store)
    metrics = BrainMetrics()
    if args.metrics_port:
        from prometheus_client import start_http_server
        start_http_server(args.metrics_port + local, registry=metrics.registry)
    # --streaming: continuous jobs go to the streaming monitor and keyable canary /
    # rollingUpdate jobs to the rollout monitor; the worker keeps what they cannot key
    worker = BrainWorker(store, cfg, worker_id=args.worker_id, metrics=metrics,
                         exclude_strategies=(("continuous", "canary", "rollingupdate") if args.streaming and
                                             args.rollout else ("continuous",) if args.streaming else ()))
    cache_path = None
    if args.model_cache:
        from .multivariate import LstmJobScorer, ModelCache
        cache_path = args.model_cache.replace("{rank}", str(local))
        if os.path.exists(cache_path):
            cache = ModelCache.load(cache_path, cfg.max_cache_size, device=worker.scorer.device)
            worker.lstm = LstmJobScorer(device=worker.scorer.device, cache=cache, threshold=cfg.lstm_threshold)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    if args.run_seconds is not None:
        loop.call_later(args.run_seconds, stop.set)
    tasks = [worker.run_forever(stop)]
    if args.streaming:
        from .node import NodeBrain, elastic_world_from_env, worker_id_of
        from .streaming import StreamingMonitor
        dev = worker.scorer.device
        world = elastic_world_from_env(dev)
        member = world.id if world is not None else f"{worker.worker_id}-stream"
        mon = StreamingMonitor(store, cfg, device=dev, metrics=metrics, ring_len=cfg.ring_len, step=args.step,
                               window=args.window, worker_id=worker_id_of(member) if world else member)
        period = args.tick_seconds if args.tick_seconds else args.step
        rollout = None
        if args.rollout:
            from .rollout import RolloutMonitor
            rollout = RolloutMonitor(store, cfg, device=dev, metrics=metrics, step=args.step, window=args.window,
                                     pods=args.pods, worker_id=(worker_id_of(member) if world else member) + "-rollout",
                                     ring_len=cfg.ring_len)
            if os.environ.get("FOREMAST_CLUSTER_AFFINE", "0") not in ("0", "", "false") and world is not None:
                # each rank scrapes its own clusters; cross-cluster windows cross ranks (RC5)
                from ..parallel.affine import ClusterRouter, affinity_from_env
                rollout.router = ClusterRouter(affinity_from_env(), dev)
        lstm = None
        if args.lstm is None:
            args.lstm = cfg.algorithm in ("lstm", "auto")
        if args.lstm:
            from .lstm_monitor import LstmMonitor
            lstm = LstmMonitor(store, cfg, device=dev, metrics=metrics, step=args.step, ring_len=cfg.ring_len,
                               worker_id=(worker_id_of(member) if world else member) + "-lstm")
            mon.exclude = lstm.is_mine
        if world is None and args.snapshot and rollout is None and lstm is None:
            snap = args.snapshot.replace("{rank}", str(local))
            tasks.append(mon.run_forever(stop, period=period, snapshot=snap, snapshot_every=args.snapshot_every))
        else:
            # node brain (also for one rank: it publishes the health table)
            tasks.append(NodeBrain(mon, world, store, dev, extra=(rollout, lstm)).run_forever(stop, period))
    await asyncio.gather(*tasks)
    if cache_path and worker.lstm is not None:
        worker.lstm.cache.save(cache_path)
    store.close()
    return worker


def main(argv=None) -> None:
    import sys
    logging.basicConfig(level=os.environ.get("FOREMAST_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    args = parse(argv)
    from ..parallel import comm
    # --nproc N: one launcher hosting the node store + N ranks; with forced collectives
    # (FOREMAST_FORCE_COLLECTIVES=1) also for one rank, so it runs the N-rank code path
    multi = args.nproc > 1 or (args.streaming and comm.force_collectives())
    if multi and not os.environ.get("FOREMAST_NODE_STORE") and "WORLD_SIZE" not in os.environ:
        from .node import launch_node
        raw = list(sys.argv[1:] if argv is None else argv)
        rest, skip = [], False
        for a in raw:  # the ranks get the same arguments minus --nproc
            if skip:
                skip = False
                continue
            if a == "--nproc":
                skip = True
                continue
            if a.startswith("--nproc="):
                continue
            rest.append(a)
        raise SystemExit(launch_node(args.nproc, rest))
    asyncio.run(run(args))


if __name__ == "__main__":
    main()
