"""One rank of the product-path N-rank tests (tests/test_node_product.py).

The production node brain (streaming + rollout monitors, NodeBrain) on a SHARED
SQLite job store, joined by an ElasticWorld over gloo; every rank sees the same
deterministic fake Prometheus and a virtual clock that advances one minute per
lockstep tick.  Apps are owned by ``owner_of`` over the live members; jobs of a
member that dies are stolen by the survivors at re-formation.  Writes one JSON
line per tick (generation, members, anomalous apps, jobs held)."""

import asyncio
import datetime
import json
import os
import sys

import httpx
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from foremast_amd.brain.node import NodeBrain, worker_id_of  # noqa: E402
from foremast_amd.brain.rollout import RolloutMonitor  # noqa: E402
from foremast_amd.brain.streaming import StreamingMonitor  # noqa: E402
from foremast_amd.parallel.elastic import ElasticWorld  # noqa: E402
from foremast_amd.promql.client import PromClient  # noqa: E402
from foremast_amd.store.jobstore import SqliteJobStore  # noqa: E402
from tests.test_node_product import T0, config, scenario, world_prometheus  # noqa: E402


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def main():
    port, me, n, db, out, ticks, hb = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                                       sys.argv[5], int(sys.argv[6]), float(sys.argv[7]))
    stop_at = int(os.environ.get("NODE_RANK_STOP_AT", "-1"))
    kv = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    world = ElasticWorld(kv, f"m{me}", [f"m{i}" for i in range(n)], backend="gloo", heartbeat_timeout_s=hb,
                         collective_timeout_s=2 * hb)
    clock = Clock(T0)
    prom = world_prometheus(clock, scenario())
    client = PromClient(transport=httpx.ASGITransport(app=prom.asgi_app()))
    cfg = config()
    store = SqliteJobStore(db)
    member = f"m{me}"
    stream = StreamingMonitor(store, cfg, prom=client, device=torch.device("cpu"), ring_len=cfg.ring_len, window=10,
                              clock=clock, worker_id=worker_id_of(member))
    roll = RolloutMonitor(store, cfg, prom=client, device=torch.device("cpu"), window=10, pods=5, clock=clock,
                          ring_len=cfg.ring_len, worker_id=worker_id_of(member) + "-rollout", min_capacity=8)
    node = NodeBrain(stream, world, store, torch.device("cpu"), publish=False, extra=(roll,))
    world.form()
    node.health.reset(kv=world.pstore)
    world.start_heartbeat()

    async def go(f):
        for k in range(ticks):
            clock.t = T0 + 60 * k
            if k == stop_at:  # freeze inside the tick: after the scoring, before the exchange
                orig = node._exchange

                def frozen():
                    os.kill(os.getpid(), 19)  # SIGSTOP: the test kills this rank while it is stopped
                    return orig()
                node._exchange = frozen
            table = await node.tick()
            lstm = roll.joint_lstm
            f.write(json.dumps({"tick": k, "generation": world.generation, "members": world.members,
                                "anomalous": table["anomalous_apps"], "jobs": sorted(roll.jobs),
                                "lstm_jobs": len(lstm.jobs) if lstm is not None else 0,
                                "lstm_steps": int(lstm.shard.trainer.steps) if lstm is not None and lstm.shard is not None else 0,
                                "biv_rows": int((roll.biv_b >= 0).sum()) if roll.cap else 0}) + "\n")
            f.flush()
    with open(out, "w") as f:
        asyncio.run(go(f))
    world.stop_heartbeat()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
