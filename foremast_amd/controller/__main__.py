"""``python -m foremast_amd.controller`` — the barrelman process.

Equivalent of ``foremast-barrelman/cmd/manager/main.go``: build the API
client, construct :class:`Barrelman` and :class:`MonitorController`, and run
concurrently

* the Deployment informer → rollout handling (job creation),
* the 10 s status poller (job status → DeploymentMonitor phase),
* the DeploymentMonitor informer → remediation,
* the sync work queue (2 workers recording "Synced" events, as the reference).

Configuration: in-cluster service account or ``--kubeconfig``/``KUBECONFIG``;
``NAMESPACE`` is barrelman's own namespace (fallback DeploymentMetadata
lookup, ``Barrelman.go:139-174``).  ``--fake`` runs against an in-memory
cluster (demo / smoke).
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
from typing import Optional

from ..k8s.api import ApiError
from .barrelman import Barrelman
from .monitor import MonitorController
from .workqueue import RateLimitingQueue, run_workers

log = logging.getLogger("foremast.barrelman")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="foremast-barrelman")
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--server", default=None, help="API server URL (e.g. kubectl proxy at http://127.0.0.1:8001)")
    p.add_argument("--namespace", default=os.environ.get("NAMESPACE", "foremast"))
    p.add_argument("--poll-seconds", type=float, default=10.0)
    p.add_argument("--resync-deployments", type=float, default=30.0)
    p.add_argument("--resync-monitors", type=float, default=10.0)
    p.add_argument("--workers", type=int, default=2)
    p.add_argument("--fake", action="store_true", help="in-memory cluster (demo)")
    p.add_argument("--run-seconds", type=float, default=None, help="exit after this long (tests)")
    return p.parse_args(argv)


class _ResyncView:
    """Per-kind resync periods over one HttpKube (informer factories with
    different resyncs in the reference: 30 s Deployments, 10 s CRDs)."""

    def __init__(self, kube, periods):
        self._kube, self._periods = kube, periods

    def __getattr__(self, name):
        return getattr(self._kube, name)

    def watch(self, kind, namespace=None):
        return self._kube.watch(kind, namespace, resync=self._periods.get(kind))


def build_kube(args):
    if args.fake:
        from ..k8s.fake import FakeCluster
        return FakeCluster()
    from ..k8s.http import HttpKube, KubeConfig
    if args.server:
        kube = HttpKube(base_url=args.server)
    else:
        cfg = KubeConfig.from_kubeconfig(args.kubeconfig) if args.kubeconfig else KubeConfig.auto()
        kube = HttpKube(cfg)
    return _ResyncView(kube, {"deployments": args.resync_deployments,
                              "deploymentmonitors": args.resync_monitors})


async def run(args, kube=None, stop: Optional[asyncio.Event] = None, **barrelman_kw) -> Barrelman:
    kube = kube if kube is not None else build_kube(args)
    bm = Barrelman(kube, namespace=args.namespace, poll_seconds=args.poll_seconds, **barrelman_kw)
    mc = MonitorController(kube, bm)
    queue = RateLimitingQueue()

    async def sync(key):
        ns, name = key
        try:
            depl = await kube.get("deployments", ns, name)
        except ApiError:
            return  # deleted meanwhile
        await bm.record_event(depl, "Synced", "Deployment synced successfully")

    async def enqueue_deployments():
        async for ev in kube.watch("deployments"):
            md = ev["object"].get("metadata") or {}
            if ev["type"] != "DELETED":
                queue.add((md.get("namespace", ""), md.get("name", "")))

    workers = await run_workers(queue, sync, workers=args.workers)
    tasks = [asyncio.create_task(c) for c in (bm.watch_deployments(), bm.poll_forever(), mc.watch_monitors(),
                                               enqueue_deployments())]
    stop = stop or asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    if args.run_seconds is not None:
        loop.call_later(args.run_seconds, stop.set)
    await stop.wait()
    for t in tasks:
        t.cancel()
    queue.shutdown(len(workers))
    await asyncio.gather(*tasks, *workers, return_exceptions=True)
    await bm.drain()
    return bm


def main(argv=None) -> None:
    logging.basicConfig(level=os.environ.get("FOREMAST_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    asyncio.run(run(parse(argv)))


if __name__ == "__main__":
    main()
