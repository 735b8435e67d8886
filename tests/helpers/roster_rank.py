"""One rank of the churning-roster exchange test (tests/test_roster_exchange.py).

The production NodeBrain exchange path — two engines per rank with change logs,
the merged NodeRoster, ClusterHealth roster deltas through the generation's
store, ElasticWorld.run_tick over gloo — driven by fake engines whose apps
churn every tick: at tick k the live apps are a sliding window of the app pool
(apps start and finish every tick, finished apps' indices are reused), each app
held by the rank ``owner_of`` gives it; an app's counters are a fixed function
of (app, tick).  Writes one JSON line per tick: the node table's apps and
anomalous apps, the exchange time and the roster bytes."""

import asyncio
import datetime
import json
import os
import sys
import zlib

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from foremast_amd.brain.node import NodeBrain, owner_of  # noqa: E402
from foremast_amd.parallel.elastic import ElasticWorld  # noqa: E402
from foremast_amd.parallel.roster import ChangeLog  # noqa: E402


def live_apps(k: int, per_tick: int, span: int):
    """Apps live at tick k: the window [k * per_tick, k * per_tick + span) of the pool,
    minus every 7th app of it on odd ticks (apps also leave out of order)."""
    lo = k * per_tick
    return [a for a in range(lo, lo + span) if not (k % 2 and a % 7 == 3)]


def counts_of(app: int, k: int, engine: int):
    h = zlib.crc32(f"{app}/{k}/{engine}".encode())
    return [int(h % 11 == 0), 1 + h % 5]


def engines_of(app: int):
    """Engines of the rank holding an app: 0, 1, or both (the merge path)."""
    return (0,) if app % 3 == 0 else (1,) if app % 3 == 1 else (0, 1)


class FakeEngine:
    def __init__(self, e: int) -> None:
        self.e = e
        self.names = []
        self.index = {}
        self.free = []
        self.roster_log = ChangeLog()
        self.roster_version = 0
        self.counts = torch.zeros((0, 2), dtype=torch.int32)
        self.owns = None
        self.worker_id = f"fake{e}"

    @property
    def n_live(self):
        return len(self.index)

    @property
    def apps(self):
        return self.index

    def set_apps(self, apps, k):
        want = {("ns", f"app{a}"): a for a in apps}
        for name in [n for n in self.index if n not in want]:
            i = self.index.pop(name)
            self.names[i] = None
            self.free.append(i)
            self.roster_log.note(i, None)
        for name in want:
            if name not in self.index:
                i = self.free.pop() if self.free else len(self.names)
                if i == len(self.names):
                    self.names.append(name)
                else:
                    self.names[i] = name
                self.index[name] = i
                self.roster_log.note(i, name)
        c = torch.zeros((len(self.names), 2), dtype=torch.int32)
        for name, i in self.index.items():
            c[i] = torch.tensor(counts_of(want[name], k, self.e))
        self.counts = c

    def roster_names(self):
        return self.names

    def app_counts(self):
        return self.counts

    async def tick(self):
        return {}

    def sync(self, steal_from=None):
        return 0

    def release(self, pred):
        return 0


def main():
    port, me, n, ticks, per_tick, span, out = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                               int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), sys.argv[7])
    kv = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    world = ElasticWorld(kv, f"m{me}", [f"m{i}" for i in range(n)], backend="gloo", heartbeat_timeout_s=10.0,
                         collective_timeout_s=30.0)
    engines = [FakeEngine(0), FakeEngine(1)]
    node = NodeBrain(engines[0], world, None, torch.device("cpu"), publish=False, extra=(engines[1],))
    node.start()

    async def go(f):
        for k in range(ticks):
            mine = [a for a in live_apps(k, per_tick, span) if owner_of("ns", f"app{a}", world.world) == world.rank]
            for e in (0, 1):
                engines[e].set_apps([a for a in mine if e in engines_of(a)], k)
            t = await node.tick()
            f.write(json.dumps({"tick": k, "apps": {a: [v["anomalous"], v["scored"]] for a, v in t["apps"].items()},
                                "anomalous": t["anomalous_apps"], "exchange_ms": t["collective_ms"],
                                "roster_bytes": t["roster_bytes"], "generation": t["generation"],
                                "phases": t["exchange_phases_ms"]}) + "\n")
    with open(out, "w") as f:
        asyncio.run(go(f))
    node.stop()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
