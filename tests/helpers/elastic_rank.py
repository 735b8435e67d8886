"""One rank of the elastic-world fault test (tests/test_elastic_fault.py):
heartbeats, app ownership by owner_of over the current members, one health
exchange per tick through ElasticWorld.run_tick; one JSON line per tick."""

import datetime
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from foremast_amd.brain.node import owner_of  # noqa: E402
from foremast_amd.parallel.cluster import ClusterHealth  # noqa: E402
from foremast_amd.parallel.elastic import ElasticWorld  # noqa: E402


def main():
    port, me, n, hb, ticks, out = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]),
                                   int(sys.argv[5]), sys.argv[6])
    kv = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=30))
    world = ElasticWorld(kv, f"m{me}", [f"m{i}" for i in range(n)], backend="gloo", heartbeat_timeout_s=hb,
                         collective_timeout_s=2 * hb)  # gloo cannot abort in-flight work: bound it
    world.form()
    world.start_heartbeat()
    health = ClusterHealth("cpu", kv=world.pstore, timeout_s=hb)
    apps = [("ns", f"app{k}") for k in range(24)]
    state = {"mine": None, "version": 0}

    def exchange():
        mine = [a for a in apps if owner_of(a[0], a[1], world.world) == world.rank]
        if mine != state["mine"]:
            state["mine"], state["version"] = mine, state["version"] + 1
        counts = torch.tensor([[0, 1]] * len(mine), dtype=torch.int32).reshape(-1, 2)
        return health.exchange(mine, counts, state["version"], len(mine), {"member": world.id})

    with open(out, "w") as f:
        for tick in range(ticks):
            gen = world.generation
            t = world.run_tick(exchange)
            if world.generation != gen:
                health.reset(kv=world.pstore)
            f.write(json.dumps({"tick": tick, "time": time.time(), "generation": world.generation,
                                "ranks": t["ranks"], "apps": sorted(t["apps"]), "members": world.members}) + "\n")
            f.flush()
            time.sleep(0.2)
    world.stop_heartbeat()


if __name__ == "__main__":
    main()
