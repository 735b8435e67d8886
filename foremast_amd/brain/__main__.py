"""``python -m foremast_amd.brain`` — the scoring worker process.

Replaces the foremast-brain container (``deploy/foremast/3_brain/foremast-brain.yaml``):
same environment variables (``ES_ENDPOINT``, ``ML_ALGORITHM``, ``threshold``,
``bound``, ``metric_type{i}`` …, ``MAX_STUCK_IN_SECONDS``; parsed by
:class:`~foremast_amd.utils.config.BrainConfig`), same Prometheus exposition
on :8000 (``foremastbrain:<metric>_{upper,lower,anomaly}`` plus engine
metrics).  ``FOREMAST_JOB_STORE`` (``sqlite:///…`` / ``memory://``) overrides
``ES_ENDPOINT``.  Several processes can share one store: claims are leases.
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
    return p.parse_args(argv)


def _bind_gpu() -> int:
    """One scorer process per GPU under torchrun: bind LOCAL_RANK's device.
    Ranks share nothing but the job store (lease-based claims)."""
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
    worker = BrainWorker(store, cfg, worker_id=args.worker_id, metrics=metrics,
                         exclude_strategies=("continuous",) if args.streaming else ())
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
        from .streaming import StreamingMonitor
        mon = StreamingMonitor(store, cfg, device=worker.scorer.device, metrics=metrics,
                               worker_id=f"{worker.worker_id}-stream")
        snap = args.snapshot.replace("{rank}", str(local)) if args.snapshot else None
        tasks.append(mon.run_forever(stop, snapshot=snap, snapshot_every=args.snapshot_every))
    await asyncio.gather(*tasks)
    if cache_path and worker.lstm is not None:
        worker.lstm.cache.save(cache_path)
    store.close()
    return worker


def main(argv=None) -> None:
    logging.basicConfig(level=os.environ.get("FOREMAST_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    asyncio.run(run(parse(argv)))


if __name__ == "__main__":
    main()
