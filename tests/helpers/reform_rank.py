"""RCCL abort and re-formation inside one process (tests/test_rccl_gpu.py,
tests/test_elastic_fault.py).

A 1-member ElasticWorld (``FOREMAST_FORCE_COLLECTIVES=1``: the 1-rank group runs
every collective, on ``nccl`` = RCCL when a GPU is present) drives the node
brain's deployed exchange.  On the third tick the exchange raises
``CollectiveTimeout`` (what a peer that stopped inside the all-gather looks like
to a survivor); ``ElasticWorld.run_tick`` must abort the communicator
(``_abort_process_group``), destroy and re-create the process group over the
live members under generation 1, and the tick must complete on the new
communicator.  Then the exchange and a DP gradient all-reduce run again on it.
The process never re-execs; it prints one JSON line with what it saw."""

import json
import os
import sys
import time

os.environ["FOREMAST_FORCE_COLLECTIVES"] = "1"
os.environ.setdefault("FOREMAST_HEARTBEAT_S", "0.5")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from foremast_amd.brain.node import NodeBrain, elastic_world_from_env  # noqa: E402
from foremast_amd.parallel import comm  # noqa: E402
from foremast_amd.parallel.dp import GradBuckets  # noqa: E402
from roster_rank import FakeEngine, live_apps  # noqa: E402


def main():
    import asyncio
    dev = torch.device("cuda", 0) if (torch.cuda.is_available() and "--cpu" not in sys.argv) else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    world = elastic_world_from_env(dev, force=True)
    engines = [FakeEngine(0), FakeEngine(1)]
    for e in engines:
        e.counts = e.counts.to(dev)
    node = NodeBrain(engines[0], world, None, dev, publish=False, extra=(engines[1],))
    node.start()
    out = {"device": str(dev), "backend": dist.get_backend(), "pid": os.getpid(), "ticks": []}
    pg0 = dist.distributed_c10d._get_default_group()
    fail = {"at": 2, "n": 0}
    orig = node._exchange

    def exchange():
        if node.ticks == fail["at"] and fail["n"] == 0:
            fail["n"] += 1
            # a wedged all-gather as the survivor sees it: the deadline fires with work in flight
            x = torch.ones(4, device=dev)
            dist.all_reduce(x, async_op=True)
            raise comm.CollectiveTimeout("injected: health all-gather did not complete")
        return orig()
    node._exchange = exchange

    async def go():
        for k in range(5):
            for e in engines:
                e.set_apps([a for a in live_apps(k, 3, 20) if e.e in (0, a % 2)], k)
                e.counts = e.counts.to(dev)
            t0 = time.perf_counter()
            t = await node.tick()
            out["ticks"].append({"tick": k, "generation": t["generation"], "apps": len(t["apps"]),
                                 "want_apps": len(live_apps(k, 3, 20)), "backend": t["backend"],
                                 "collectives": t["collectives"], "ms": round((time.perf_counter() - t0) * 1e3, 2)})
    asyncio.run(go())
    pg1 = dist.distributed_c10d._get_default_group()
    # the new communicator carries a DP gradient all-reduce (weights in the same collective)
    lin = torch.nn.Linear(8, 4).to(dev)
    gb = GradBuckets(list(lin.parameters()), overlap=False)
    gb.zero()
    for p in lin.parameters():
        p.grad.fill_(3.0)
    flags = gb.finish(weight=2.0, flags=torch.tensor([1.0, 5.0], device=dev), timeout_s=30.0)
    x = torch.arange(16, dtype=torch.float32, device=dev)
    w = dist.all_reduce(x, async_op=True)
    comm.wait_bounded(w, 30.0, "post-reform all-reduce")
    if dev.type == "cuda":
        torch.cuda.synchronize()
    out.update(generation=world.generation, reforms=world.reforms, new_group=pg1 is not pg0,
               backend_after=dist.get_backend(), grads_ok=all(bool((p.grad == 3.0).all()) for p in lin.parameters()),
               flags=flags.cpu().tolist(), allreduce_ok=bool((x.cpu() == torch.arange(16.0)).all()),
               injected=fail["n"])
    node.stop()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
