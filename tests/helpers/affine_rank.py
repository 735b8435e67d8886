"""One rank of the multi-cluster canary test (tests/test_affine.py): the rank
scrapes ONLY its own cluster's Prometheus (any request to the other cluster
raises), serves rollout jobs of its cluster through the node brain, and gets
the other cluster's baseline windows over the process group (RC5)."""

import asyncio
import datetime
import json
import os
import sys

import httpx
import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from foremast_amd.brain.node import NodeBrain  # noqa: E402
from foremast_amd.brain.rollout import RolloutMonitor  # noqa: E402
from foremast_amd.brain.streaming import StreamingMonitor  # noqa: E402
from foremast_amd.parallel.affine import ClusterRouter, affinity_from_env  # noqa: E402
from foremast_amd.promql.client import PromClient  # noqa: E402
from foremast_amd.store.jobstore import SqliteJobStore  # noqa: E402
from foremast_amd.utils.config import BrainConfig, reference_default_env  # noqa: E402
from tests.test_affine import ENDPOINTS, T0, clusters  # noqa: E402


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


class AffineTransport(httpx.AsyncBaseTransport):
    """Routes by host to the cluster's fake Prometheus; refuses the other cluster."""

    def __init__(self, apps, mine):
        self.apps, self.mine = apps, mine
        self.requests = {h: 0 for h in apps}

    async def handle_async_request(self, request):
        host = request.url.host
        if host != self.mine:
            raise RuntimeError(f"rank scraped {host}, not its own cluster {self.mine}")
        self.requests[host] += 1
        return await httpx.ASGITransport(app=self.apps[host]).handle_async_request(request)


def main():
    port, rank, db, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    store_kv = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    dist.init_process_group("gloo", store=store_kv, rank=rank, world_size=2)
    clock = Clock(T0)
    proms = clusters(clock)
    mine = ["prom-a", "prom-b"][rank]
    transport = AffineTransport({h: p.asgi_app() for h, p in proms.items()}, mine)
    client = PromClient(transport=transport)
    env = reference_default_env()
    env.update(MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10", threshold0="4")
    cfg = BrainConfig.from_env(env)
    store = SqliteJobStore(db)
    if os.environ.get("AFFINE_FAIL_BEAT") == str(rank):  # a transient store error on this rank
        beat, calls = store.heartbeat, []

        def flaky(worker, now=None):
            if worker.endswith("-rollout"):
                calls.append(now)
                if len(calls) in (3, 4):
                    raise OSError("injected heartbeat failure")
            return beat(worker, now)
        store.heartbeat = flaky
    roll = RolloutMonitor(store, cfg, prom=client, device=torch.device("cpu"), window=10, pods=5, clock=clock,
                          ring_len=2880, worker_id=f"rank{rank}-rollout", min_capacity=4)
    roll.router = ClusterRouter(affinity_from_env(), torch.device("cpu"), timeout_s=30)
    stream = StreamingMonitor(store, cfg, prom=client, device=torch.device("cpu"), ring_len=2880, window=5,
                              clock=clock, worker_id=f"rank{rank}-stream")
    node = NodeBrain(stream, None, store, torch.device("cpu"), publish=False, extra=(roll,))
    lines = []

    async def go():
        for k in range(12):
            clock.t = T0 + 60 * k
            table = await node.tick()
            base_ok = {p.app[1]: int(np.isfinite(roll.base[p.rows].numpy()).sum()) for p in roll.jobs.values()}
            lines.append({"tick": k, "rank": rank, "jobs": sorted(p.app[1] for p in roll.jobs.values()),
                          "base_valid": base_ok, "anomalous": table["anomalous_apps"],
                          "exchanges": roll.router.exchanges, "values_moved": roll.router.values_moved,
                          "scrapes": transport.requests})
    asyncio.run(go())
    with open(out, "w") as f:
        for ln in lines:
            f.write(json.dumps(ln) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
