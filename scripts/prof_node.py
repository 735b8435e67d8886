#!/usr/bin/env python
"""Host profile of the production node tick (``bench.py --config node``): cProfile
over the timed ticks of NodeBrain.tick, plus the per-phase timings the monitors
record.  Writes ``<out>/node_host.pstats.txt`` (top functions by self time and by
cumulative time) and ``<out>/node_host.json``.

Usage: python scripts/prof_node.py [--out DIR] [--ticks K] [bench.py node args...]
"""

from __future__ import annotations

import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    argv = sys.argv[1:]
    out, ticks = "gpurun_out/prof_node", 8
    if "--out" in argv:
        i = argv.index("--out")
        out = argv[i + 1]
        del argv[i:i + 2]
    if "--ticks" in argv:
        i = argv.index("--ticks")
        ticks = int(argv[i + 1])
        del argv[i:i + 2]
    os.makedirs(out, exist_ok=True)
    warm = [] if "--warmup" in argv else ["--warmup", "1"]
    lstm = "--lstm" in argv
    argv = [a for a in argv if a != "--lstm"]
    sys.argv = ["bench.py", "--config", "node-lstm" if lstm else "node", "--steps", str(ticks)] + warm + argv
    import torch

    import bench
    args = bench.parse()
    world, rank, dev = bench.init_dist(args)
    from foremast_amd.benchmarks.node import setup_arrival, setup_node, setup_node_lstm
    setup = setup_arrival if getattr(args, "arrival_per_tick", 0) else setup_node
    if lstm:
        setup = setup_node_lstm
    tick, _health, meta, _dt, _n = setup(args, world, rank, dev)
    for k in range(args.warmup):
        tick(k)
    prof = cProfile.Profile()
    wall = []
    for k in range(args.steps):
        t0 = time.perf_counter()
        prof.enable()
        tick(args.warmup + k)
        prof.disable()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        wall.append((time.perf_counter() - t0) * 1e3)
    buf = io.StringIO()
    for key in ("tottime", "cumulative"):
        buf.write(f"==== sorted by {key} over {args.steps} ticks ====\n")
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats(key).print_stats(45)
    prof.dump_stats(os.path.join(out, "node_host.prof"))
    with open(os.path.join(out, "node_host.pstats.txt"), "w") as f:
        f.write(buf.getvalue())
    rec = {"tick_ms": [round(x, 2) for x in wall], "breakdowns": meta["_breakdowns"],
           "intake_breakdown_ms": meta.get("intake_breakdown_ms"), "series": args.series}
    with open(os.path.join(out, "node_host.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({"tick_ms": rec["tick_ms"]}))


if __name__ == "__main__":
    main()
